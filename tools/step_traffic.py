"""HBM bytes per step of a bench stage from two rocprofv3 --pmc passes (FETCH_SIZE /
WRITE_SIZE of every dispatch of the named kernels, summed, divided by the steps the run
made): the line traffic of a receive that launches several kernels per step.

    python tools/step_traffic.py <fetch_dir> <write_dir> <steps> <kernel substring> ...
FETCH_SIZE is taken raw (scattered line traffic; the gfx950 streaming correction of
tools/pmc_traffic.py does not apply to 64-B line read-modify-writes)."""
import collections
import csv
import glob
import os
import sys


def totals(root, counter, subs):
    per = collections.defaultdict(float)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter:
                    for s in subs:
                        if s in r.get("Kernel_Name", ""):
                            per[s] += float(r["Counter_Value"]) * 1024
    return per


def main():
    fdir, wdir, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    subs = sys.argv[4:]
    f, w = totals(fdir, "FETCH_SIZE", subs), totals(wdir, "WRITE_SIZE", subs)
    tot = 0.0
    for s in subs:
        b = (f[s] + w[s]) / steps
        tot += b
        print(f"{s}: fetch {f[s] / steps / 1e6:.1f} MB + write {w[s] / steps / 1e6:.1f} MB per step")
    print(f"total {tot / 1e6:.1f} MB per step")


if __name__ == "__main__":
    main()
