"""Parity of a segmented top-k library variant (tools/build_variants.py) against the oracle:
python tools/seg_variant_check.py chocosgd_amd/lib/variants/lib_seg5.so

Cold + warm calls (with and without x_hat, with the fused gossip step) on the ResNet-50
layout and an edge layout; exits non-zero on the first mismatch.  Diagnostic: the GPU
suite covers the product library."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(path):
    from chocosgd_amd import _lib, codec
    from oracle import choco_oracle as O
    _lib.load(path)
    dev = torch.device("cuda")
    with open(os.path.join(ROOT, "tests", "golden", "layouts.json")) as f:
        r50 = json.load(f)["resnet50_imagenet"]
    layouts = {"r50": r50, "edges": [20479, 20480, 20481, 1, 3, 700_001, 24576, 24577, 2_500_007, 16383, 16385]}
    for name, lens in layouts.items():
        n = sum(lens)
        plan = codec.SegmentPlan(lens, 0.99, dev)
        g = torch.Generator(device=dev).manual_seed(3)
        for call in range(4):
            x = torch.randn(n, generator=g, device=dev)
            xh = 0.1 * torch.randn(n, generator=g, device=dev) if call % 2 else None
            d = (x - xh).cpu().numpy() if xh is not None else x.cpu().numpy()
            v, i = codec.topk_segmented(x, plan, xhat=xh)
            ov, oi, _ = O.topk_segmented(d, lens, 0.99)
            ok = np.array_equal(i.cpu().numpy().astype(np.int64), oi) and np.array_equal(v.cpu().numpy(), ov)
            print(f"{name} call {call} xhat={xh is not None}: {'ok' if ok else 'MISMATCH'}", flush=True)
            if not ok:
                return 1
        # the fused gossip step (warm)
        x = torch.randn(n, generator=g, device=dev)
        xh = x + 0.1 * torch.randn(n, generator=g, device=dev)
        mem = xh + 0.05 * torch.randn(n, generator=g, device=dev)
        xa = O.gossip_step(x.cpu().numpy(), mem.cpu().numpy(), xh.cpu().numpy(), 0.9)
        v, i = codec.topk_segmented(x, plan, xhat=xh, gossip=(mem, 0.9))
        ov, oi, _ = O.topk_segmented((xa - xh.cpu().numpy()).astype(np.float32), lens, 0.99)
        ok = (np.array_equal(x.cpu().numpy().view(np.uint32), xa.view(np.uint32))
              and np.array_equal(i.cpu().numpy().astype(np.int64), oi) and np.array_equal(v.cpu().numpy(), ov))
        print(f"{name} gossip: {'ok' if ok else 'MISMATCH'}", flush=True)
        if not ok:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
