"""Per-kernel times (dispatch-attached events) of the sign / QSGD compress run
back to back on one buffer, optionally after dirtying the Infinity Cache with a
large write (as the previous step's decompress-accumulate does in the bench).

    python tools/codec_loop.py --op qsgd|sign [--dirty] [--lib path]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import _lib, codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="qsgd")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dirty", action="store_true")
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    if a.lib:
        _lib.load(a.lib)
    dev = torch.device("cuda", 0)
    n = a.n or (100_000_000 if a.op == "qsgd" else 345_000_000)
    d = torch.randn(n, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    junk = torch.empty(128 * 2**20, device=dev) if a.dirty else None  # 512 MB
    names = ["qsgd_norm", "qsgd_quantize"] if a.op == "qsgd" else ["sign_pack"]
    codec.profile_enable(True)
    for r in range(a.reps + 3):
        if r == 3:
            codec.profile_reset()
        if junk is not None:
            junk.fill_(1.0)
        if a.op == "qsgd":
            codec.qsgd_compress(d, 4, seed=7, offset=r)
        else:
            codec.sign_compress(d)
    torch.cuda.synchronize()
    out = {nm: codec.profile_read(nm) for nm in names}
    print(a.op, "dirty" if a.dirty else "clean", {k: round(1e3 * v[0] / max(v[1], 1), 1) for k, v in out.items()})


if __name__ == "__main__":
    main()
