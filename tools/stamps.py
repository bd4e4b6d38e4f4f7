"""Phase timeline of one top-k call from the CHOCO_STAMPS diagnostic build
(wall_clock64, 100 MHz): per-kernel spans, per-workgroup durations.

    python tools/stamps.py [--n 100000000] [--lib chocosgd_amd/lib/variants/lib_stamps.so]
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
    ap.add_argument("--save", default=None, help="write the raw stamp table (.npy)")
    ap.add_argument("--nbuf", type=int, default=4, help="buffers compressed in rotation (the bench's warm path)")
    ap.add_argument("--cold", action="store_true", help="stamp a cold call (warm start off: K1 runs)")
    a = ap.parse_args()
    lib = _lib.load(a.lib)
    fn = lib.choco_dbg_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    ds = [torch.randn(a.n, generator=g, device=dev) for _ in range(max(1, a.nbuf))]
    k = codec.topk_k(a.n, a.ratio)
    lib.choco_topk_set_warm_start(0 if a.cold else 1)
    for i in range(6):
        codec.topk(ds[i % len(ds)], k)
    torch.cuda.synchronize()
    buf = np.zeros((40960, 4), dtype=np.uint64)
    fn(None, 0)
    try:
        codec.topk(ds[6 % len(ds)], k)
    except RuntimeError as e:  # diagnostic builds that stop early
        print("(call failed:", e, ")")
    torch.cuda.synchronize()
    fn(buf.ctypes.data, buf.nbytes)
    if a.save:
        np.save(a.save, buf)
    t = buf.astype(np.int64)
    k2 = t[1024:1024 + 4096]
    k2 = k2[k2[:, 0] > 0]
    pro = t[20000:20000 + 2048]
    pro = pro[pro[:, 0] > 0]
    t0 = k2[:, 0].min()

    def us(v):
        return (v - t0) * TICK_US

    def row(name, v):
        v = v[v > 0]
        if v.size == 0:
            print(f"  {name:34s} (none)")
            return
        print(f"  {name:34s} min {us(v.min()):8.2f}  med {us(np.median(v)):8.2f}  max {us(v.max()):8.2f} us")

    k1 = t[30000]
    if k1[0] > 0:
        print(f"K1 bounds: sample in {(k1[1] - k1[0]) * TICK_US:.2f} us, bounds {(k1[2] - k1[0]) * TICK_US:.2f} us "
              f"after its start; K2 starts {(t0 - k1[2]) * TICK_US:.2f} us after K1's end")
        s1, s2 = t[30001], t[30002]
        print("  K1 phases (us after its start): subsample hist %.2f | F found %.2f | compacted %.2f | fine hist %.2f"
              " | before find %.2f | ranks %.2f" % tuple((v - k1[0]) * TICK_US for v in
                                                          (s1[0], s1[1], s1[2], s1[3], s2[0], s2[1])))
    print(f"n={a.n} k={k}; times in us from the first K2 workgroup start")
    print(f"K2 sample + stream ({len(k2)} workgroups)")
    row("start", k2[:, 0]); row("sample bounds", k2[:, 1]); row("streamed", k2[:, 2]); row("end", k2[:, 3])
    # per XCD (workgroup b runs on XCD b % 8): full tiles only (the last tile is partial)
    full = t[1024:1024 + 4096]
    nb = int((full[:, 0] > 0).sum())
    ends = {x: [us(full[b, 3]) for b in range(x, nb - 1, 8)] for x in range(8)}
    print("  per-XCD end of the full tiles (median / max us): " +
          "  ".join(f"X{x} {np.median(v):.1f}/{max(v):.1f}" for x, v in ends.items() if v))
    row("  sample keys in registers", pro[:, 0]); row("  subsample histogram", pro[:, 1])
    row("  keys >= F listed + fine histogram", pro[:, 2]); row("  bounds", pro[:, 3])
    tb = t[22000:22000 + 2048]
    row("  tile entries binned", tb[tb[:, 0] > 0][:, 0])
    pro = (k2[:, 1] - k2[:, 0]) * TICK_US
    dur = (k2[:, 2] - k2[:, 1]) * TICK_US
    tail = (k2[:, 3] - k2[:, 2]) * TICK_US
    print(f"  per-wg prologue min {pro.min():.2f} med {np.median(pro):.2f} max {pro.max():.2f} us;"
          f" stream min {dur.min():.2f} med {np.median(dur):.2f} max {dur.max():.2f} us;"
          f" end-of-tile min {tail.min():.2f} med {np.median(tail):.2f} max {tail.max():.2f} us")
    ws = t[32000:32000 + 8 * len(k2)].reshape(len(k2), 8, 4)
    se, be = ws[:, :4].reshape(len(k2), 16), ws[:, 4:].reshape(len(k2), 16)
    if (se > 0).all():
        spread = (se.max(1) - se.min(1)) * TICK_US
        first_be = (be.min(1) - se.max(1)) * TICK_US
        burst = (be.max(1) - be.min(1)) * TICK_US
        print(f"  per-wave stream end spread (last - first wave) min {spread.min():.2f} med {np.median(spread):.2f}"
              f" max {spread.max():.2f} us")
        print(f"  last wave's stream end -> first wave's burst end: med {np.median(first_be):.2f} max {first_be.max():.2f};"
              f" burst end spread med {np.median(burst):.2f} max {burst.max():.2f} us")
        row("  last wave stream end", se.max(1)); row("  last wave burst end", be.max(1))
    k4 = t[24576:24576 + 1000]
    k4 = k4[k4[:, 0] > 0]
    print(f"K34 select + emit ({len(k4)} workgroups)")
    row("start", k4[:, 0])
    q = t[26000:26000 + 1000]
    q = q[q[:, 0] > 0]
    q2 = t[27000:27000 + 1000]
    q2 = q2[q2[:, 0] > 0]
    row("  run starts", q[:, 0]); row("  totals in LDS", q[:, 1]); row("  j* found", q[:, 2])
    row("  table words + scan", q[:, 3]); row("  (key loads issued)", q2[:, 1])
    m = t[29000]
    print(f"  bucket j*={m[2]} holds M={m[0]} keys (shift {m[1]}); candidates {m[3]}")
    q3 = t[28000:28000 + 1000]
    q3 = q3[q3[:, 0] > 0]
    if len(q3):
        row("  (gather addresses ready)", q3[:, 0]); row("  (gather + emit loads issued)", q3[:, 1])
    row("  bucket keys stored", q2[:, 2])
    if len(q3):
        row("  (select histogram built)", q3[:, 2]); row("  (select rank found)", q3[:, 3])
    row("  T selected", q2[:, 0])
    row("offsets known", k4[:, 1])
    q5 = t[30000:30000 + 1000]
    q5 = q5[q5[:, 0] > 0]
    if len(q5):
        row("  (emission keys compared)", q5[:, 0]); row("  (emission ranks)", q5[:, 1])
        row("  (emission stores issued)", q5[:, 2])
    row("end", k4[:, 2])


if __name__ == "__main__":
    main()
