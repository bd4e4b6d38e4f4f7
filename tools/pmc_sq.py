"""Per-kernel SQ counters from one rocprofv3 --pmc pass (the median over dispatches).

    python tools/pmc_sq.py <pmc_dir> [kernel substring ...]

Prints, per kernel, each collected counter and the derived rates (MI355X: 256 CUs,
4 SIMDs per CU):
  * VALU instructions per wave and per element are the raw SQ_INSTS_VALU;
  * VALU busy = SQ_ACTIVE_INST_VALU / (SQ_BUSY_CYCLES * 4 SIMDs) when both are present
    (SQ_ACTIVE_INST_VALU counts, per SIMD, the cycles a VALU instruction was being
    issued; SQ_BUSY_CYCLES the cycles the SQs were busy, summed over the SEs);
  * wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES (wave-cycles spent waiting on anything).
"""
import collections
import csv
import glob
import os
import statistics
import sys


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    names = {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                kn = r.get("Kernel_Name", "")
                per[kn][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
                names[kn] = kn
    return per


def main():
    root = sys.argv[1]
    subs = sys.argv[2:]
    per = load(root)
    for kn, ctrs in sorted(per.items()):
        if subs and not any(s in kn for s in subs):
            continue
        short = kn.split("(")[0][-70:]
        med = {c: statistics.median(v.values()) for c, v in ctrs.items()}
        ndisp = max(len(v) for v in ctrs.values())
        print(f"{short}  ({ndisp} dispatches)")
        for c in sorted(med):
            print(f"    {c:24s} {med[c]:16.0f}")
        if "SQ_ACTIVE_INST_VALU" in med and "SQ_BUSY_CYCLES" in med and med["SQ_BUSY_CYCLES"] > 0:
            print(f"    VALU busy (ACTIVE_INST_VALU / (BUSY_CYCLES * 4)) {med['SQ_ACTIVE_INST_VALU'] / (4 * med['SQ_BUSY_CYCLES']):.3f}")
        if "SQ_WAIT_ANY" in med and "SQ_WAVE_CYCLES" in med and med["SQ_WAVE_CYCLES"] > 0:
            print(f"    wait share (WAIT_ANY / WAVE_CYCLES) {med['SQ_WAIT_ANY'] / med['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_INSTS_VALU" in med and "SQ_WAVES" in med and med["SQ_WAVES"] > 0:
            print(f"    VALU instructions per wave {med['SQ_INSTS_VALU'] / med['SQ_WAVES']:.0f}")


if __name__ == "__main__":
    main()
