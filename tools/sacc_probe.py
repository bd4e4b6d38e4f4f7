"""Sign decompress-accumulate time vs the address offset between x_hat and
memory (both carved out of one allocation, memory at x_hat + n + d elements):
the four streams (read+write of both) run at the same element offsets, so an
unlucky base distance could make them collide in HBM channels.

    python tools/sacc_probe.py [--n 345000000] [--lib path]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import _lib, codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=345_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    if a.lib:
        _lib.load(a.lib)
    dev = torch.device("cuda", 0)
    n = a.n
    x = torch.randn(n, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    packed, norms = codec.sign_compress(x)
    del x
    extra = 1 << 24
    big = torch.zeros(2 * n + extra, device=dev)
    for d in [0, 256, 4096, 65536, 1 << 20, 1 << 21, 3 << 20, (1 << 22) + 4096, 1 << 23, (1 << 24) - 512]:
        hat = big[:n]
        mem = big[n + d: 2 * n + d]
        ts = []
        for r in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            codec.sign_accumulate([(packed, norms)], [0.5], 0, n, mem, xhat_self=hat)
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        delta = (mem.data_ptr() - hat.data_ptr())
        print(f"d {d:>9d} el: mem - hat = {delta / 2**20:10.3f} MiB ({delta % (1 << 21)} mod 2 MiB): "
              f"median {ts[len(ts) // 2]:8.1f} us")


if __name__ == "__main__":
    main()
