"""Warm-start behaviour of the fused top-k step over a sequence of CHOCO steps (the bench's
step_topk dynamics): per call the fallback counter, the time, the exact T and the control
block (both windows, overflow words, bucket totals G[0] / G[255] of each parity).
    python tools/drain_probe.py [n]"""
import os
import struct
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import codec  # noqa: E402

dev = torch.device('cuda', 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(n, generator=g, device=dev)
hat = x + 0.1 * torch.randn(n, generator=g, device=dev)
mem = hat + 0.05 * torch.randn(n, generator=g, device=dev)
k = codec.topk_k(n, 0.99)
vals = torch.empty(k, device=dev)
idx = torch.empty(k, dtype=torch.int32, device=dev)


def ctrl():
    ws = codec._ws_cache[(dev.index, torch.cuda.current_stream(dev).cuda_stream, "topk")]
    b = ws[:272 + 2 * 16 * 256 * 4].cpu().numpy().tobytes()
    ov = struct.unpack_from("<2I", b, 64)
    out = []
    for p in range(2):
        s_lo, s_hi, sh, m, nn, kk, valid, tp = struct.unpack_from("<4I2q2I", b, 128 + 40 * p)
        G = np.frombuffer(b, dtype=np.uint32, count=16 * 256, offset=272 + p * 16 * 256 * 4).reshape(16, 256).sum(0)
        out.append(f"par{p}: lo {s_lo:#x} hi {s_hi:#x} sh {sh} m {m} valid {valid} tprev {tp:#x} ov {ov[p]} "
                   f"G0 {G[0]} G255 {G[255]}")
    return " | ".join(out)


for s in range(14):
    torch.cuda.synchronize()
    t = time.perf_counter()
    codec.topk(x, k, xhat=hat, out=(vals, idx), gossip=(mem, 0.9))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    T = torch.topk((x - hat).abs(), k).values[-1].item()
    Tk = struct.unpack("<I", struct.pack("<f", T))[0]
    print(s, "fallbacks", codec.topk_fallback_count(), "ms %.3f" % (dt * 1e3), "T %.6g key %#x" % (T, Tk), flush=True)
    print("   ", ctrl(), flush=True)
    codec.sparse_accumulate(vals, idx, mem, 1.0, xhat_self=hat)
