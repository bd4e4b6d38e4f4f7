"""Phase timeline of one random-k call (flat, 100M, k = 1 %) from the CHOCO_STAMPS
diagnostic build (wall_clock64, 100 MHz): R1 count pass and R2 tile pass, per
workgroup.

    python tools/rk_stamps.py [--n 100000000] [--lib chocosgd_amd/lib/variants/lib_stamps.so]
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

TICK_US = 0.01  # 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--ratio", type=float, default=0.99)
    ap.add_argument("--lib", default=os.path.join(ROOT, "chocosgd_amd/lib/variants/lib_stamps.so"))
    a = ap.parse_args()
    lib = _lib.load(a.lib)
    fn = lib.choco_dbg_rk_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    ds = [torch.randn(a.n, generator=g, device=dev) for _ in range(4)]
    k = codec.topk_k(a.n, a.ratio)
    for i in range(6):
        codec.randk(ds[i % 4], k, seed=i)
    torch.cuda.synchronize()
    buf = np.zeros((16384, 8), dtype=np.uint64)
    fn(None, 0)
    codec.randk(ds[2], k, seed=99)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, buf.nbytes)
    t = buf.astype(np.int64)
    r1 = t[:8192]
    r1 = r1[r1[:, 0] > 0]
    r2 = t[8192:]
    r2 = r2[r2[:, 0] > 0]
    t0 = r1[:, 0].min()

    def row(name, v):
        v = v[v > 0]
        if v.size == 0:
            print(f"  {name:28s} (none)")
            return
        u = (v - t0) * TICK_US
        print(f"  {name:28s} min {u.min():8.2f}  med {np.median(u):8.2f}  max {u.max():8.2f} us  ({v.size})")

    print(f"n={a.n} k={k}; us from the first R1 workgroup start")
    print(f"R1 count ({len(r1)} workgroups)")
    row("start", r1[:, 0]); row("draws binned", r1[:, 1]); row("column written", r1[:, 2])
    print(f"R2 tile ({len(r2)} workgroups)")
    row("start", r2[:, 0]); row("count + offset", r2[:, 1]); row("bitmap", r2[:, 2]); row("ranks", r2[:, 3])
    row("emitted", r2[:, 4])
    d = (r2[:, 4] - r2[:, 0]) * TICK_US
    print(f"  per-workgroup duration min {d.min():.2f} med {np.median(d):.2f} max {d.max():.2f} us")
    for name, a_, b_ in (("count load", 0, 1), ("bitmap", 1, 2), ("ranks", 2, 3), ("gather+store", 3, 4)):
        x = (r2[:, b_] - r2[:, a_]) * TICK_US
        print(f"    {name:14s} med {np.median(x):.2f} max {x.max():.2f} us")


if __name__ == "__main__":
    main()
