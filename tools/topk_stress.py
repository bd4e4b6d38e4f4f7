"""Randomised exactness stress of the flat top-k pipeline's warm path and its misses (the
carried windows, drift, the exact fallback through the shared select, the cold runs): random
sizes, then a random walk of deltas -- drift, jumps up and down by large factors,
tie-quantised values, zero blocks, sign flips, the fused consensus step -- every call
checked bit-exact against the oracle.
    python tools/topk_stress.py [sizes] [calls per size] [seed]
Prints one line per size (calls, exact fallbacks, sample launches; the fallback counter is
the stream's shared workspace's, which a larger size reallocates: its difference can be
negative); exits 1 at the first mismatch."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import codec  # noqa: E402
from oracle import choco_oracle as O  # noqa: E402


def main():
    nlay = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rng = np.random.default_rng(seed)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(seed)
    for li in range(nlay):
        n = int(rng.choice([65_537, 1_000_003, 3_000_001, 8_388_608, 25_000_000]))
        ratio = float(rng.choice([0.9, 0.99, 0.999]))
        k = codec.topk_k(n, ratio)
        gossip = bool(rng.integers(0, 2))
        x = torch.randn(n, generator=g, device=dev)
        hat = x + 0.1 * torch.randn(n, generator=g, device=dev)
        mem = hat + 0.05 * torch.randn(n, generator=g, device=dev)
        m0 = codec.topk_fallback_count()
        c0 = codec.launch_count("topk_bounds")
        for ci in range(calls):
            kind = rng.choice(["drift", "drift", "drift", "up", "down", "ties", "zeros", "flip"])
            if kind == "drift":
                x.add_(torch.randn(n, generator=g, device=dev), alpha=float(rng.uniform(0.001, 0.05)))
            elif kind == "up":
                x.copy_(hat + float(rng.uniform(2, 200)) * (x - hat))
            elif kind == "down":
                x.copy_(hat + float(rng.uniform(0.005, 0.5)) * (x - hat))
            elif kind == "ties":
                q = float(rng.choice([2.0, 8.0, 64.0]))
                x.copy_(hat + torch.round((x - hat) * q) / q)
            elif kind == "zeros":  # a block where x = x_hat: the delta's exact zeros
                a = int(rng.integers(0, n))
                b = min(n, a + int(rng.integers(1, n // 3 + 2)))
                x[a:b] = hat[a:b]
            else:
                x.copy_(2 * hat - x)
            if gossip:
                xa = O.gossip_step(x.cpu().numpy(), mem.cpu().numpy(), hat.cpu().numpy(), 0.9)
                vals, idx = codec.topk(x, k, xhat=hat, gossip=(mem, 0.9))
                if not np.array_equal(x.cpu().numpy().view(np.uint32), xa.view(np.uint32)):
                    print(f"size {li} call {ci} ({kind}): x_new differs")
                    return 1
                d = (xa - hat.cpu().numpy()).astype(np.float32)
            else:
                d = (x.cpu().numpy() - hat.cpu().numpy()).astype(np.float32)
                vals, idx = codec.topk(x, k, xhat=hat)
            ov, oi = O.topk(d, k)
            if not (np.array_equal(idx.cpu().numpy().astype(np.int64), oi)
                    and np.array_equal(vals.cpu().numpy().view(np.uint32), ov.view(np.uint32))):
                print(f"size {li} call {ci} ({kind}): selection differs (n {n}, ratio {ratio})")
                return 1
            if gossip:
                codec.sparse_accumulate(vals, idx, mem, 1.0, xhat_self=hat)
        codec.check_topk_status(wait=True)
        print(f"size {li}: n {n}, ratio {ratio}, gossip {gossip}: {calls} calls exact, exact fallbacks "
              f"{codec.topk_fallback_count() - m0}, K1 sample launches {codec.launch_count('topk_bounds') - c0}",
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
