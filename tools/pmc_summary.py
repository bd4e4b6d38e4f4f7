"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, mean counter
value per dispatch (FETCH_SIZE/WRITE_SIZE in KB as reported)."""
import collections
import csv
import glob
import os
import sys


def main(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            name = r.get("Kernel_Name", r.get("Kernel-Name", ""))
            key = name.split("(")[0][-48:]
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(acc):
        print(k)
        for c, v in sorted(acc[k].items()):
            # several rows per dispatch (one per XCD/agent dimension) -> sum per dispatch is what matters;
            # report total / dispatches if the dispatch count is known, else the mean row
            print(f"    {c:24s} rows={len(v):5d} sum/rows={sum(v)/len(v):14.1f} total={sum(v):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
