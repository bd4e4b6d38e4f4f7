"""Randomised exactness stress of the segmented top-k's warm path and its missed-window
handling (the shared exact select over the segment or over the candidate lists, the
windows it writes, the cold runs): random layouts, then a random walk of deltas --
drift, jumps up and down by large factors, tie-quantised values, zero blocks, sign flips,
the fused consensus step -- every call checked bit-exact against the oracle.
    python tools/seg_stress.py [layouts] [calls per layout] [seed]
Prints one line per layout (calls, window misses, cold calls); exits 1 at the first
mismatch."""
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
        nt = int(rng.integers(3, 40))
        lens = [int(v) for v in rng.choice([1, 5, 300, 4096, 16383, 16384, 16385, 40_000, 131_072, 400_001,
                                            1_200_000, 2_359_296], size=nt)]
        n = sum(lens)
        ratio = float(rng.choice([0.9, 0.99, 0.999]))
        plan = codec.SegmentPlan(lens, ratio, dev)
        gossip = bool(rng.integers(0, 2))
        x = torch.randn(n, generator=g, device=dev)
        hat = x + 0.1 * torch.randn(n, generator=g, device=dev)
        mem = hat + 0.05 * torch.randn(n, generator=g, device=dev)
        m0 = codec.topk_fallback_count(plan=plan)
        c0 = codec.launch_count("topk_seg_hist")
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
                vals, idx = codec.topk_segmented(x, plan, xhat=hat, gossip=(mem, 0.9))
                if not np.array_equal(x.cpu().numpy().view(np.uint32), xa.view(np.uint32)):
                    print(f"layout {li} call {ci} ({kind}): x_new differs")
                    return 1
                d = (xa - hat.cpu().numpy()).astype(np.float32)
            else:
                d = (x.cpu().numpy() - hat.cpu().numpy()).astype(np.float32)
                vals, idx = codec.topk_segmented(x, plan, xhat=hat)
            ov, oi, _ = O.topk_segmented(d, lens, ratio)
            if not (np.array_equal(idx.cpu().numpy().astype(np.int64), oi)
                    and np.array_equal(vals.cpu().numpy().view(np.uint32), ov.view(np.uint32))):
                print(f"layout {li} call {ci} ({kind}): selection differs (n {n}, {nt} tensors, ratio {ratio})")
                return 1
            if gossip:
                codec.sparse_accumulate(vals, idx, mem, 1.0, xhat_self=hat)
        codec.check_topk_status(wait=True)
        print(f"layout {li}: {nt} tensors, n {n}, ratio {ratio}, gossip {gossip}: {calls} calls exact, "
              f"window misses {codec.topk_fallback_count(plan=plan) - m0}, cold calls "
              f"{codec.launch_count('topk_seg_hist') - c0}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
