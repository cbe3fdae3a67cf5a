"""trace_iter.py <kernel_trace.csv> <rollout-name-substring> [n_iters]: per-iteration timeline from a rocprofv3
--kernel-trace csv: every kernel between two consecutive rollout launches (the last n_iters iterations), its
duration and the idle gap before it, plus per-name totals averaged over those iterations. Analysis aid only."""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("at::native::", "")
    return n.split("(")[0][:90]


def main():
    path, key = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if key in r[2]]
    if len(starts) < 2:
        sys.exit("fewer than two rollout launches in the trace")
    its = list(zip(starts[:-1], starts[1:]))[-n:]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    gaps = 0.0
    span = 0.0
    for a, b in its:
        span += (rows[b][0] - rows[a][0]) / 1e3
        prev_end = None
        for r in rows[a:b]:
            nm = short(r[2])
            tot[nm] += (r[1] - r[0]) / 1e3
            cnt[nm] += 1
            if prev_end is not None:
                gaps += max(0, r[0] - prev_end) / 1e3
            prev_end = max(prev_end or 0, r[1])
        gaps += max(0, rows[b][0] - prev_end) / 1e3
    k = len(its)
    print(f"iterations {k}: {span / k:.1f} us per iteration, idle gaps {gaps / k:.1f} us")
    for nm, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {v / k:9.1f} us  x{cnt[nm] / k:4.1f}  {nm}")
    a, b = its[-1]
    print("last iteration timeline (start offset us, duration us, gap us):")
    t0 = rows[a][0]
    prev_end = None
    for r in rows[a:b]:
        gap = (r[0] - prev_end) / 1e3 if prev_end is not None else 0.0
        print(f"  {(r[0] - t0) / 1e3:9.1f} {(r[1] - r[0]) / 1e3:8.1f} {gap:7.1f}  {short(r[2])}")
        prev_end = max(prev_end or 0, r[1])


if __name__ == "__main__":
    main()
