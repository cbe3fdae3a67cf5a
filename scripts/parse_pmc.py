"""Sum rocprofv3 --pmc counter CSVs per kernel (kernels whose name contains argv[2], default "rollout") and print
per-dispatch averages."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
filt = sys.argv[2].split(",") if len(sys.argv) > 2 else ["rollout"]
tot = defaultdict(float)
disp = defaultdict(set)
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "")
            if not any(f in k for f in filt):
                continue
            name = row.get("Counter_Name")
            tot[(k[:75], name)] += float(row.get("Counter_Value", 0))
            disp[(k[:75], name)].add(row.get("Dispatch_Id"))
for (k, name), v in sorted(tot.items()):
    n = max(1, len(disp[(k, name)]))
    print(f"{k:75s} {name:28s} per_dispatch={v / n:16.0f}  dispatches={n}")
