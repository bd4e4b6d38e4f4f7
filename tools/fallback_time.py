"""Time the exact top-k fallback (K34's wide_fallback) at 100M on tie-heavy inputs:
dispatch-attached event times of K1/K2/K34 per call.

    python tools/fallback_time.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import codec  # noqa: E402

n = 100_000_000
g = torch.Generator(device="cuda").manual_seed(5)
cases = {"gaussian": torch.randn(n, generator=g, device="cuda"),
         "ties_1/8": torch.round(torch.randn(n, generator=g, device="cuda") * 8) / 8,
         "all_equal": torch.full((n,), 0.5, device="cuda")}
k = codec.topk_k(n, 0.99)
for name, x in cases.items():
    codec.topk(x, k)
    codec.profile_reset()
    codec.profile_enable(True)
    reps = 5
    for _ in range(reps):
        codec.topk(x, k)
    torch.cuda.synchronize()
    codec.profile_enable(False)
    t = {nm: codec.profile_read(nm)[0] / reps * 1e3 for nm in ("topk_bounds", "topk_stream", "topk_finish")}
    print(f"{name:10s} " + " ".join(f"{a} {b:8.1f} us" for a, b in t.items()), flush=True)
