"""Debug the wide fallback queue: one top-k call on an all-equal input (the side lists
overflow, so K34 takes the fallback) with a printf-tracing library variant.

    python tools/build_variants.py wide_debug && python tools/fallback_debug.py [n]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import _lib, codec  # noqa: E402

_lib.load(os.path.join(ROOT, "chocosgd_amd/lib/variants/lib_wide_debug.so"))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
x = torch.full((n,), 0.5, device="cuda")
k = codec.topk_k(n, 0.99)
v, i = codec.topk(x, k)
torch.cuda.synchronize()
print("indices ok:", np.array_equal(i.cpu().numpy(), np.arange(k)), flush=True)
