"""Prints the top kernels of a rocprofv3 kernel_stats.csv (avg us, share)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>4} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
          f"pct={float(r['TotalDurationNs']) / tot * 100:5.1f}")
