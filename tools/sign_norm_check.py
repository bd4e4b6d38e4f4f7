"""Per-segment L1 norms of the sign pack vs the fp64 oracle on the golden layouts
(diagnostic for the multi-segment pack's norm path)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from chocosgd_amd import codec  # noqa: E402
from conftest import golden  # noqa: E402
from oracle import choco_oracle as O  # noqa: E402

g = golden("deepsqueeze_sign_mini")
lens = g["layout"].tolist()
offs = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int64, device="cuda")
for r in range(3):
    x = torch.from_numpy(g["mem"][r].copy()).cuda()
    _, nm = codec.sign_compress(x, seg_off=offs, nseg=len(lens))
    a = nm.cpu().numpy()
    b = O.l1_norms(g["mem"][r], lens)
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
    print(r, "max rel", rel.max(), "seg", int(np.argmax(rel)), "len", lens[int(np.argmax(rel))], a[:6], b[:6])
    _, nm2 = codec.sign_compress(x, xhat=torch.zeros_like(x), seg_off=offs, nseg=len(lens))
    print("   with xhat", np.abs(nm2.cpu().numpy() - b).max())
