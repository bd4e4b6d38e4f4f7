"""Phase timeline of one fused top-k call (CHOCO_STAMPS build, wall_clock64 at 100 MHz):
per workgroup the kernel start, ticket, bounds seen, stream end, tile published,
all-tiles-done seen, select done, exit -- as percentiles over workgroups, in us
from the earliest start.

    python tools/build_variants.py fused_stamps
    python tools/fused_stamps.py [--n 100000000] [--lib chocosgd_amd/lib/variants/lib_fused_stamps.so]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import _lib, codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--ratio", type=float, default=0.99)
    ap.add_argument("--lib", default=os.path.join(ROOT, "chocosgd_amd/lib/variants/lib_fused_stamps.so"))
    a = ap.parse_args()
    lib = _lib.load(a.lib)
    fn = lib.choco_dbg_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda", 0)
    ds = [torch.randn(a.n, generator=torch.Generator(device=dev).manual_seed(s), device=dev) for s in range(3)]
    k = codec.topk_k(a.n, a.ratio)
    junk = torch.ones(256 * 1024 * 1024, device=dev)
    for i in range(4):
        codec.topk(ds[i % 3], k)
    torch.cuda.synchronize()
    buf = np.zeros((40960, 4), dtype=np.uint64)
    for rep in range(3):
        torch.sum(junk)  # cold caches
        torch.cuda.synchronize()
        fn(None, 0)
        codec.topk(ds[rep % 3], k)
        torch.cuda.synchronize()
        fn(buf.ctypes.data, buf.nbytes)
        t = buf.astype(np.int64)
        A, B, C = t[36000:36256], t[37000:37256], t[38000:38256]
        live = A[:, 0] > 0
        A, B, C = A[live], B[live], C[live]
        t0 = A[:, 0].min()
        names = ["start", "ticket", "bounds", "stream end", "published", "done seen", "select", "exit"]
        cols = [A[:, 0], A[:, 1], A[:, 2], A[:, 3], B[:, 0], B[:, 1], B[:, 2], B[:, 3]]
        print(f"rep {rep}: {live.sum()} workgroups; spilled tiles {int(C[:, 2].sum())}; "
              f"max hsum {int(C[:, 3].max())}; tiles per wg max {int(C[:, 1].max())}")
        for nm, c in zip(names, cols):
            v = (c[c > 0] - t0) * 0.01
            if v.size:
                print(f"  {nm:12s} min {v.min():7.2f}  p50 {np.median(v):7.2f}  max {v.max():7.2f} us")
        bw = C[:, 0] == 1  # ticket 0 = bounds workgroup
        if bw.any():
            print(f"  bounds wg: start {(A[bw, 0][0] - t0) * .01:.2f} published {(A[bw, 2][0] - t0) * .01:.2f}")


if __name__ == "__main__":
    main()
