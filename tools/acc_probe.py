"""Sparse accumulate (x_hat[idx] += v, memory[idx] += w v) time vs the address
offset between the two target arrays: both are carved out of one allocation,
memory at x_hat + n + d elements.  Tests whether the two RMW streams collide in
HBM banks/channels for some offsets (the step-to-step variance of the bench).

    python tools/acc_probe.py [--n 100000000] [--k 1000000]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    if a.lib:
        from chocosgd_amd import _lib
        _lib.load(a.lib)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    idx = torch.randperm(a.n, generator=g, device=dev)[: a.k].sort().values.to(torch.int32)
    val = torch.randn(a.k, generator=g, device=dev)
    # bit-exactness vs the same arithmetic in torch (distinct indices)
    hat0 = torch.randn(a.n, generator=g, device=dev)
    mem0 = torch.randn(a.n, generator=g, device=dev)
    hat, mem = hat0.clone(), mem0.clone()
    codec.sparse_accumulate(val, idx, mem, 0.5, xhat_self=hat)
    il = idx.long()
    hr, mr = hat0.clone(), mem0.clone()
    hr[il] = hr[il] + val
    mr[il] = mr[il] + 0.5 * val
    print("bit-exact vs torch:", bool(torch.equal(hat, hr)) and bool(torch.equal(mem, mr)))
    del hat0, mem0, hat, mem, hr, mr
    extra = 1 << 22
    big = torch.zeros(2 * a.n + 2 * extra, device=dev)
    for d in [0, 1024, 1 << 20]:
        hat = big[: a.n]
        mem = big[a.n + d: 2 * a.n + d]
        ts = []
        for r in range(a.reps + 3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            codec.sparse_accumulate(val, idx, mem, 0.5, xhat_self=hat)
            e1.record()
            torch.cuda.synchronize()
            if r >= 3:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        print(f"offset {d:>8d} el ({d * 4 / 1024:8.1f} KiB): median {ts[len(ts) // 2]:7.2f} us  min {ts[0]:7.2f}")
    # separate allocations, as in the bench
    for trial in range(3):
        hat = torch.zeros(a.n, device=dev)
        mem = torch.zeros(a.n, device=dev)
        ts = []
        for r in range(a.reps + 3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            codec.sparse_accumulate(val, idx, mem, 0.5, xhat_self=hat)
            e1.record()
            torch.cuda.synchronize()
            if r >= 3:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        print(f"separate allocs #{trial} (mem - hat = {(mem.data_ptr() - hat.data_ptr()) / 2**20:.1f} MiB): "
              f"median {ts[len(ts) // 2]:7.2f} us")
        del hat, mem


if __name__ == "__main__":
    main()
