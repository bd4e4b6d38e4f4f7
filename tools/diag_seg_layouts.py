"""Diagnostic: QSGD norm / quantize and sign pack times over one 25.6M buffer in different
segment layouts (flat, 2 halves, 161 equal tensors, ResNet-50's 161 tensors), profile hooks."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import _lib, codec  # noqa: E402


def main():
    if len(sys.argv) > 1:
        _lib.load(sys.argv[1])
    with open(os.path.join(ROOT, "tests", "golden", "layouts.json")) as f:
        r50 = json.load(f)["resnet50_imagenet"]
    n = sum(r50)
    h = (n // 2) // 8192 * 8192
    np_ = (n + 31) // 32
    layouts = {"flat": [n], "halves": [n // 2, n - n // 2], "halves_tile_aligned": [h, n - h],
               "rows32": [np_] * 31 + [n - 31 * np_],
               "equal161": [n // 161] * 160 + [n - 160 * (n // 161)],
               "equal161_tile_aligned": [19 * 8192] * 160 + [n - 160 * 19 * 8192], "resnet50": r50}
    dev = torch.device("cuda", 0)
    d = torch.randn(n, device=dev)
    for name, lens in layouts.items():
        nseg = len(lens)
        seg_off = torch.tensor([0] + list(torch.tensor(lens).cumsum(0).tolist()), dtype=torch.int64, device=dev) \
            if nseg > 1 else None
        kw = {"seg_off": seg_off, "nseg": nseg} if nseg > 1 else {}
        for _ in range(3):
            codec.qsgd_compress(d, 4, seed=1, **kw)
            codec.sign_compress(d, **kw)
        torch.cuda.synchronize()
        codec.profile_reset()
        codec.profile_enable(True)
        reps = 20
        for i in range(reps):
            codec.qsgd_compress(d, 4, seed=1, offset=i, **kw)
            codec.sign_compress(d, **kw)
        torch.cuda.synchronize()
        codec.profile_enable(False)
        out = {}
        for k in ("qsgd_norm", "qsgd_quantize", "sign_pack"):
            t, c = codec.profile_read(k)
            out[k] = round(t / c * 1e3, 2) if c else None
        print(name, nseg, out, flush=True)


if __name__ == "__main__":
    main()
