"""Sparse accumulate A/B on cold lines: x_hat[idx] += v, memory[idx] += w v for a
k = 1 % message of an n = 100M buffer, one of 4 index sets per rep (as the bench
rotates deltas), with a 1 GiB streaming read between reps so the targets are not
Infinity-Cache resident.  Checks bit-exactness against torch once.

    python tools/acc_bench.py [--lib variant.so] [--n 100000000] [--k 1000000] [--msgs 1]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import _lib, codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=1_000_000)
    ap.add_argument("--msgs", type=int, default=1, help="messages per round (self first)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--hot", action="store_true", help="no eviction between reps")
    a = ap.parse_args()
    if a.lib:
        _lib.load(a.lib)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    sets = []
    for s in range(4):
        msgs = []
        for m in range(a.msgs):
            idx = torch.randperm(a.n, generator=g, device=dev)[: a.k].sort().values.to(torch.int32)
            msgs.append((torch.randn(a.k, generator=g, device=dev), idx))
        sets.append(msgs)
    w = [1.0 / (a.msgs + 1)] * a.msgs
    hat0 = torch.randn(a.n, generator=g, device=dev)
    mem0 = torch.randn(a.n, generator=g, device=dev)
    hat, mem = hat0.clone(), mem0.clone()
    for m, (v, i) in enumerate(sets[0]):
        codec.sparse_accumulate(v, i, mem, w[m], xhat_self=hat if m == 0 else None)
    hr, mr = hat0.clone(), mem0.clone()
    for m, (v, i) in enumerate(sets[0]):
        il = i.long()
        if m == 0:
            hr[il] = hr[il] + v
        mr[il] = mr[il] + w[m] * v
    exact = bool(torch.equal(hat, hr)) and bool(torch.equal(mem, mr))
    del hat0, mem0, hr, mr
    junk = torch.ones(256 * 1024 * 1024, device=dev)
    sink = torch.empty(1, device=dev)
    ts = []
    for r in range(a.reps + 3):
        if not a.hot:
            torch.sum(junk, dim=0, keepdim=True, out=sink)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for m, (v, i) in enumerate(sets[r % 4]):
            codec.sparse_accumulate(v, i, mem, w[m], xhat_self=hat if m == 0 else None)
        e1.record()
        torch.cuda.synchronize()
        if r >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    print(f"{os.path.basename(a.lib or 'default'):28s} msgs={a.msgs} bit-exact={exact} "
          f"median {statistics.median(ts):7.2f} us  min {ts[0]:7.2f}  max {ts[-1]:7.2f}")


if __name__ == "__main__":
    main()
