"""Run the top-k compress on a 100M randn buffer `--reps` times at `--ratio`
(for rocprofv3 counter passes on the stream / finish kernels)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import codec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--ratio", type=float, default=0.99)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda", 0)
d = torch.randn(a.n, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
k = codec.topk_k(a.n, a.ratio)
for _ in range(a.reps):
    codec.topk(d, k)
torch.cuda.synchronize()
print("done", k)
