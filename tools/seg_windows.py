"""Warm-path state of the segmented top-k after a few calls (csrc/topk_seg.hip): per
segment the mode S3a set (0 select, 1 window missed -> exact fallback, 2 every
element) and the window (lo, sh).  python tools/seg_windows.py [--layout resnet50_imagenet]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import codec  # noqa: E402


def align(v, a=256):
    return (v + a - 1) // a * a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="resnet50_imagenet")
    ap.add_argument("--calls", type=int, default=6)
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "layouts.json")) as f:
        lens = json.load(f)[a.layout]
    dev = torch.device("cuda", 0)
    plan = codec.SegmentPlan(lens, 0.99, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    ds = [torch.randn(sum(lens), generator=g, device=dev) for _ in range(4)]
    for i in range(a.calls):
        codec.topk_segmented(ds[i % 4], plan)
    torch.cuda.synchronize()
    ws = plan.workspace(dev).cpu().numpy()
    nseg, ntile = plan.nseg, plan.ntile
    o = 256
    o += align(nseg * 2048 * 4) * 2 + align(nseg * 512 * 4)
    info = ws[o:o + nseg * 32].view(np.uint32).reshape(nseg, 8)
    o += align(nseg * 32) + align(ntile * 4) + align(ntile * 8) + 2 * align(ntile * 16384 * 4)
    win = ws[o:o + nseg * 16].view(np.uint32).reshape(nseg, 4)
    modes = info[:, 6]
    print(f"{nseg} segments, modes: select {int((modes == 0).sum())} missed {int((modes == 1).sum())} "
          f"all {int((modes == 2).sum())}")
    for s in np.nonzero(modes == 1)[0][:20]:
        print(f"  missed seg {s}: len {lens[s]} k {plan.k_per_seg[s]} window lo {win[s, 0]:#x} sh {win[s, 1]}")
    print("window sh histogram:", np.bincount(win[:, 1], minlength=10).tolist())


if __name__ == "__main__":
    main()
