"""Diagnostic: the segmented deferred sign receive's per-segment L1 norms against the unfused
pack and the oracle (ResNet-20 layout and tiny segments); prints the segments that differ."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from chocosgd_amd import codec  # noqa: E402
from conftest import golden_json  # noqa: E402
from oracle import choco_oracle as O  # noqa: E402

DEV = "cuda"


def main():
    for name, lens in (("resnet20", golden_json("layouts.json")["resnet20_cifar10"]),
                       ("tiny", [1 + (i * 7) % 13 for i in range(300)] + [65_536, 3, 200_001])):
        n = sum(lens)
        seg_off = torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int64, device=DEV)
        nseg = len(lens)
        g = torch.Generator(device=DEV).manual_seed(7)
        msgs = [codec.sign_compress(torch.randn(n, generator=g, device=DEV), seg_off=seg_off, nseg=nseg)
                for _ in range(3)]
        x = torch.randn(n, generator=g, device=DEV)
        h = torch.randn(n, generator=g, device=DEV) * 0.3
        m = torch.randn(n, generator=g, device=DEV) * 0.1
        xa, ha, ma = x.clone(), h.clone(), m.clone()
        w = [0.3, 0.4, 0.3]
        codec.sign_accumulate(msgs, w, 1, n, ma, xhat_self=ha, seg_off=seg_off, nseg=nseg)
        pa, na = codec.sign_compress(xa, xhat=ha, seg_off=seg_off, nseg=nseg, gossip=(ma, 0.5))
        pb, nb = codec.sign_recv_gossip_compress(msgs, w, 1, x, m, h, 0.5, seg_off=seg_off, nseg=nseg)
        torch.cuda.synchronize()
        d = (x - h).cpu().numpy()
        exact = O.l1_norms(d, lens)
        na, nb = na.cpu().numpy(), nb.cpu().numpy()
        print(name, "n", n, "nseg", nseg, "words equal", bool(torch.equal(pa, pb)),
              "x equal", bool(torch.equal(xa, x)), flush=True)
        offs = np.concatenate([[0], np.cumsum(lens)])
        for s in range(nseg):
            if not np.isclose(nb[s], exact[s], rtol=1e-6, atol=0) or not np.isclose(na[s], exact[s], rtol=1e-6, atol=0):
                print(f"  seg {s} [{offs[s]}, {offs[s + 1]}) len {lens[s]}: recv {nb[s]!r} pack {na[s]!r} "
                      f"exact {exact[s]!r} ratio {nb[s] / exact[s]:.6f}", flush=True)


if __name__ == "__main__":
    main()
