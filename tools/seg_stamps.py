"""Phase timeline of one warm segmented top-k collect launch (W2) from the CHOCO_STAMPS
build (wall_clock64, 100 MHz): per tile {dispatched, loads issued, flags + histogram,
scan barriers, stores + histogram atomics} for multi-tile segments, {dispatched, exact
select done} for single-tile ones.

    python tools/seg_stamps.py [--lib chocosgd_amd/lib/variants/lib_stamps.so] [--layout resnet50_imagenet]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import _lib, codec  # noqa: E402

TICK_US = 0.01


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "chocosgd_amd/lib/variants/lib_stamps.so"))
    ap.add_argument("--layout", default="resnet50_imagenet")
    ap.add_argument("--ratio", type=float, default=0.99)
    a = ap.parse_args()
    lib = _lib.load(a.lib)
    fn = lib.choco_dbg_seg_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda", 0)
    lens = json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))[a.layout]
    plan = codec.SegmentPlan(lens, a.ratio, dev)
    g = torch.Generator(device=dev).manual_seed(1000)
    ds = [torch.randn(sum(lens), generator=g, device=dev) for _ in range(4)]
    for i in range(6):
        codec.topk_segmented(ds[i % 4], plan)
    torch.cuda.synchronize()
    for call in range(2):
        fn(None, 0)
        codec.topk_segmented(ds[(6 + call) % 4], plan)
        torch.cuda.synchronize()
        buf = np.zeros((4096, 4), dtype=np.uint64)
        fn(buf.ctypes.data, buf.nbytes)
        t = buf.astype(np.int64)
        ntile = sum((m + 16383) // 16384 for m in lens)
        tiles_of = np.repeat(np.arange(len(lens)), [(m + 16383) // 16384 for m in lens])
        single = np.array([((lens[s] + 16383) // 16384) == 1 for s in tiles_of])
        d, e = t[:ntile], t[2048:2048 + ntile]
        t0 = d[:, 0][d[:, 0] > 0].min()

        def q(v):
            v = v[v > 0]
            return "(none)" if v.size == 0 else \
                f"min {(v.min() - t0) * TICK_US:7.2f}  med {(np.median(v) - t0) * TICK_US:7.2f}  max {(v.max() - t0) * TICK_US:7.2f}"

        def dur(a_, b_):
            m = (a_ > 0) & (b_ > 0)
            v = (b_[m] - a_[m]) * TICK_US
            return "(none)" if v.size == 0 else f"med {np.median(v):6.2f}  p90 {np.percentile(v, 90):6.2f}  max {v.max():6.2f} us"
        print(f"call {call}: {a.layout}, {len(lens)} segments, {ntile} tiles ({single.sum()} single-tile); "
              f"us from the first dispatch")
        print(f"  dispatched (multi)      {q(d[~single, 0])}")
        print(f"  dispatched (single)     {q(d[single, 0])}")
        print(f"  stores done (multi)     {q(e[~single, 2])}")
        print(f"  exact done (single)     {q(e[single, 3])}")
        m = ~single
        print(f"  multi-tile: dispatch -> loads issued  {dur(d[m, 0], d[m, 1])}")
        print(f"              loads -> flags+hist       {dur(d[m, 1], e[m, 0])}")
        print(f"              flags -> scanned          {dur(e[m, 0], e[m, 1])}")
        print(f"              scanned -> stored         {dur(e[m, 1], e[m, 2])}")
        print(f"              whole tile                {dur(d[m, 0], e[m, 2])}")
        print(f"  single-tile: whole (exact select)     {dur(d[single, 0], e[single, 3])}")


if __name__ == "__main__":
    main()
