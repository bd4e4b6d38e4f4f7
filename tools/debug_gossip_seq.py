"""Diagnostic: tests/test_gpu_topk.py::test_topk_warm_start_gossip_sequence step by step
(match per step, the workspace's fallback counter), repeated; optional segmented calls first."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import codec  # noqa: E402
from oracle import choco_oracle as O  # noqa: E402

DEV = "cuda"


def host(t):
    return t.cpu().numpy()


def run(rep):
    n = 3_000_011
    k = codec.topk_k(n, 0.99)
    g = torch.Generator(device=DEV).manual_seed(450)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    for step in range(5):
        xa = O.gossip_step(host(x), host(mem), host(hat), 0.9)
        d = (xa - host(hat)).astype(np.float32)
        vals, idx = codec.topk(x, k, xhat=hat, gossip=(mem, 0.9))
        xs = np.array_equal(host(x).view(np.uint32), xa.view(np.uint32))
        ov, oi = O.topk(d, k)
        ii = host(idx).astype(np.int64)
        ok = np.array_equal(ii, oi) and np.array_equal(host(vals).view(np.uint32), ov.view(np.uint32))
        bad = int(np.sum(ii != oi))
        print(f"rep {rep} step {step}: x {xs} sel {ok} (differing positions {bad}) "
              f"fallbacks {codec.topk_fallback_count()}", flush=True)
        codec.sparse_accumulate(vals, idx, mem, 1.0, xhat_self=hat)


if __name__ == "__main__":
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        run(rep)
