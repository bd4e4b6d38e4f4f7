"""Phase timeline of one warm top-k call on the one-launch path (CHOCO_STAMPS build):
stream phases of every workgroup, the arrival, the last workgroup's select chain, the
record hand-off and the emission (wall_clock64, 100 MHz).

    CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_stamps.so python tools/one_stamps.py [--n 100000000]
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
    ap.add_argument("--nbuf", type=int, default=4)
    ap.add_argument("--calls", type=int, default=3, help="stamped calls (one timeline each)")
    ap.add_argument("--acc", action="store_true", help="a sparse accumulate of each message between calls (bench step)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--trace", action="store_true", help="control words after each warm-up call")
    ap.add_argument("--loop", type=int, default=1, help="calls issued back to back per timeline (the last is shown)")
    a = ap.parse_args()
    lib = _lib.load()
    fn = lib.choco_dbg_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(a.seed)
    ds = [torch.randn(a.n, generator=g, device=dev) for _ in range(max(1, a.nbuf))]
    k = codec.topk_k(a.n, a.ratio)
    hat = torch.zeros(a.n, device=dev)
    mem = torch.zeros(a.n, device=dev)

    def step(i):
        v, ix = codec.topk(ds[i % len(ds)], k)
        if a.acc:
            codec.sparse_accumulate(v, ix, mem, 1.0, xhat_self=hat)
    for i in range(6):
        step(i)
        if a.trace:
            torch.cuda.synchronize()
            ws = codec._ws_cache.get((0, torch.cuda.current_stream(dev).cuda_stream, "topk"))
            w32 = ws[:256].view(torch.int32).tolist()
            b0, b1 = w32[32:36], w32[42:46]
            print(f"warm-up call {i}: fallbacks {w32[1]} cold_left {w32[2]} backoff {w32[3]} why {w32[5:10]} "
                  f"G-vs-rows mismatches {w32[10:16]} "
                  f"bounds0 (s_lo s_hi shift m) {b0} bounds1 {b1}")
    torch.cuda.synchronize()
    for call in range(a.calls):
        buf = np.zeros((40960, 4), dtype=np.uint64)
        fn(None, 0)
        codec.profile_reset()
        codec.profile_enable(True)
        for j in range(a.loop):
            step(6 + call * a.loop + j)
        torch.cuda.synchronize()
        codec.profile_enable(False)
        ev = {nm: codec.profile_read(nm)[0] * 1e3 / a.loop for nm in ("topk_stream", "topk_finish", "sparse_accumulate")}
        fn(buf.ctypes.data, buf.nbytes)
        fb = codec.topk_fallback_count()
        ws = codec._ws_cache.get((0, torch.cuda.current_stream(dev).cuda_stream, "topk"))
        why = ws[20:40].view(torch.int32).tolist() if ws is not None else None
        print(f"(exact fallbacks so far: {fb}; last one-launch fallback: overflow, G[0], G[sure], M, j* = {why})")
        t = buf.astype(np.int64)
        k2 = t[1024:1024 + 1024]
        live = np.nonzero(k2[:, 0] > 0)[0]
        k2 = k2[live]
        onef = t[24576:24576 + 1024][live]
        last = t[26000:26000 + 1024]
        lw = np.nonzero(last[:, 0] >= t[1024:1024 + 1024][live][:, 0].min())[0]  # this call's last workgroup
        t0 = k2[:, 0].min()

        def row(name, v):
            v = v[v > 0]
            if v.size == 0:
                print(f"  {name:28s} (none)")
                return
            us = (v - t0) * TICK_US
            print(f"  {name:28s} min {us.min():8.2f}  med {np.median(us):8.2f}  max {us.max():8.2f} us")
        last_end = max(onef[:, 2].max(), k2[:, 3].max())
        print(f"call {call}: n={a.n} k={k}, {len(live)} workgroups; us from the first workgroup start; "
              f"dispatch events (avg of {a.loop}): " + ", ".join(f"{nm} {v:.1f} us" for nm, v in ev.items() if v)
              + f"; in-kernel span (first start -> last stamp) {(last_end - t0) * TICK_US:.1f} us")
        te = t[22000:22000 + 1024][live]
        rk = t[28000:28000 + 1024][live]
        wv = t[32000:32000 + 8 * 1024].reshape(1024, 8, 4)[live]
        last_wave = wv[:, :4, :].reshape(len(live), 16).max(1)
        row("start", k2[:, 0]); row("window known", k2[:, 1]); row("streamed (wave 0)", k2[:, 2])
        row("streamed (last wave)", last_wave)
        row("tile scans + G adds", te[:, 0]); row("pairs binned", te[:, 1]); row("tile end", k2[:, 3])
        row("arrived (before ticket)", onef[:, 0]); row("ticket returned", onef[:, 3])
        row("record known", onef[:, 1]); row("emit: pmap ready", rk[:, 0]); row("emit: ranks", rk[:, 1])
        row("emitted", onef[:, 2])
        if lw.size:
            L = last[lw[0]]
            L2 = t[27000 + lw[0]]
            print(f"  last workgroup {lw[0]}: " + " | ".join(
                f"{nm} {(L[j] - t0) * TICK_US:.2f}" for j, nm in enumerate(["j*", "keys gathered", "T", "records"]))
                + f" | tile counts {(L2[0] - t0) * TICK_US:.2f} | scan {(L2[1] - t0) * TICK_US:.2f}")
        xcd = {}
        for i, b in enumerate(live):
            xcd.setdefault(b % 8, []).append((k2[i, 2] - t0) * TICK_US)
        print("  per-XCD streamed med/max: " + " ".join(f"X{x} {np.median(v):.1f}/{max(v):.1f}"
                                                          for x, v in sorted(xcd.items())))


if __name__ == "__main__":
    main()
