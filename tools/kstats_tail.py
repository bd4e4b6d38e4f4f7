"""A kernel_stats.csv (rocprofv3's --stats format) over each kernel's LAST M dispatches,
from the same run's kernel_trace.csv.

The step workloads run 200 burn-in steps in the profiled process; rocprofv3's own
--stats summary averages over them too (their early calls -- the delta growing from
0, top-k's exact fallbacks -- are not the steady state the bench line times).  This
summary keeps the last M dispatches of every kernel (M = the bench's timed steps), so
its averages are comparable with the bench's event times.

    python tools/kstats_tail.py <kernel_trace.csv> <M> > <out.csv>
"""
import collections
import csv
import math
import sys


def main():
    path, m = sys.argv[1], int(sys.argv[2])
    runs = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        runs[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows = []
    for name, d in runs.items():
        d.sort()
        ns = [t for _, t in d[-m:]]
        tot = sum(ns)
        avg = tot / len(ns)
        sd = math.sqrt(sum((t - avg) ** 2 for t in ns) / len(ns))
        rows.append([name, len(ns), tot, avg, 0.0, min(ns), max(ns), sd])
    total = sum(r[2] for r in rows) or 1
    for r in rows:
        r[4] = round(100.0 * r[2] / total, 2)
    rows.sort(key=lambda r: -r[2])
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for r in rows:
        w.writerow(r)


if __name__ == "__main__":
    main()
