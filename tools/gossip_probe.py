"""Time the standalone consensus step (choco_gossip_step) at 100M fp32 for a set of
library variants (tools/build_variants.py g_*): kernel time from dispatch-attached
events, back to back and behind a 400 MB dirtying pass.

    python tools/gossip_probe.py [lib.so ...]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import _lib, codec  # noqa: E402


def run(path, n=100_000_000, reps=20):
    _lib._lib = None
    _lib.load(path)
    x = torch.randn(n, device="cuda")
    m = torch.randn(n, device="cuda")
    h = torch.randn(n, device="cuda")
    junk = torch.empty(n, device="cuda")
    out = {}
    for mode in ("b2b", "dirty"):
        codec.profile_reset()
        for i in range(reps + 2):
            if mode == "dirty":
                junk.fill_(float(i))  # 400 MB of dirty lines ahead of the step, as in training
            codec.profile_enable(i >= 2)
            codec.gossip_step(x, m, h, 0.9)
            codec.profile_enable(False)
        torch.cuda.synchronize()
        t, c = codec.profile_read("gossip_step")
        us = t / c * 1e3
        out[mode] = (round(us, 1), round(16 * n / (us * 1e-6) / 1e12, 2))
    return out


if __name__ == "__main__":
    libs = sys.argv[1:] or [_lib.LIB_PATH]
    for p in libs:
        print(os.path.basename(p), run(p), flush=True)
