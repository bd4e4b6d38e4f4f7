"""HBM traffic per dispatch of every codec kernel from two rocprofv3 --pmc passes.

FETCH_SIZE and WRITE_SIZE are reported in KB per dispatch (summed over the TCC
instances).  gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE
counts exactly half of the bytes of a wide coalesced STREAMING read, so it is
doubled for the streaming kernels -- and NOT for the scattered read-modify-write
of the sparse accumulate (4-B gathers; the correction is uncalibrated there, so
its raw count is kept).  Writes profiles/pmc_traffic.json
{"<profile name>:<workload>:<n>": {...}}, the keys bench.py reads.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <workload> <n> [--tail M]

--tail M: the median over each kernel's LAST M dispatches only (the step workloads'
200 burn-in steps run in the same process, and their early calls -- the delta growing
from 0, exact fallbacks -- are not the steady state the bench line times).
"""
import collections
import csv
import glob
import json
import os
import sys

# bench/profile stage name -> (rocprof kernel-name substring, fetch correction)
KERNELS = {
    "topk_bounds": ("topk_bounds_kernel", 2.0),
    "topk_stream": ("topk_stream_kernel", 2.0),
    "topk_finish": ("topk_finish_kernel", 2.0),
    "topk_seg_hist": ("seg_hist_kernel", 2.0),
    "topk_seg_collect": ("seg_collect_kernel", 2.0),
    "topk_seg_fine": ("seg_fine_kernel", 2.0),
    "topk_seg_count": ("seg_count_kernel", 2.0),
    "topk_seg_bin": ("seg_bin_kernel", 2.0),
    "topk_seg_emit": ("seg_emit", 2.0),  # seg_emit_kernel (cold) / seg_emit_w_kernel (warm)
    "sparse_accumulate": ("sparse_acc_seg_kernel", 1.0),
    "randk_count": ("randk_count_kernel", 1.0),
    "randk_tile": ("randk_tile_kernel", 1.0),  # 4-B gathers: raw count (uncalibrated, like the accumulate)
    "qsgd_norm": ("qsgd_norm_kernel", 2.0),
    "qsgd_quantize": ("qsgd_quant_kernel", 2.0),
    "qsgd_recv_norm": ("qsgd_recv_gossip_norm_kernel", 2.0),
    "qsgd_accumulate": ("qsgd_decode_kernel", 2.0),
    "sign_pack": ("sign_pack", 2.0),
    "sign_accumulate": ("sign_accumulate_kernel", 2.0),
    "sign_recv_pack": ("sign_recv_rows_kernel", 2.0),
    "sign_planes": ("planes_kernel", 2.0),
    "gossip_step": ("::gossip", 2.0),  # gossip1_kernel / gossipu_kernel (not qsgd_recv_gossip_norm_kernel)
}


def per_dispatch(root, counter, kernel, tail=0):
    """The counter's per-dispatch totals (sorted), of the last `tail` dispatches if tail > 0."""
    vals = collections.defaultdict(float)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter and kernel in r.get("Kernel_Name", ""):
                    vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    ids = sorted(vals)
    if tail > 0:
        ids = ids[-tail:]
    return sorted(vals[i] for i in ids), len(vals)


def main():
    argv = sys.argv[1:]
    tail = 0
    if "--tail" in argv:
        i = argv.index("--tail")
        tail = int(argv[i + 1])
        del argv[i:i + 2]
    fdir, wdir, workload, n = argv[:4]
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    for name, (kernel, corr) in KERNELS.items():
        f, nf = per_dispatch(fdir, "FETCH_SIZE", kernel, tail)
        w, nw = per_dispatch(wdir, "WRITE_SIZE", kernel, tail)
        if not f or not w:
            continue
        fmed, wmed = f[len(f) // 2], w[len(w) // 2]
        out = {"fetch_bytes": corr * fmed * 1024, "write_bytes": wmed * 1024}
        out["bytes"] = out["fetch_bytes"] + out["write_bytes"]
        over = f"the last {len(f)}/{len(w)} of {nf}/{nw}" if tail else f"{len(f)}/{len(w)}"
        out["note"] = (f"median over {over} dispatches; FETCH_SIZE x{corr:g} "
                       f"({'gfx950 streaming-read correction' if corr != 1 else 'scattered: raw'}) + WRITE_SIZE, "
                       "KB units x1024")
        key = f"{name}:{workload}:{n}"
        data[key] = out
        print(key, out)
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
