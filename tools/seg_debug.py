"""Diagnose a segmented top-k mismatch: per-segment diff against the oracle and the
device's per-segment select state (b1, kb, T) read back from the workspace.

    python tools/seg_debug.py [--layout resnet50_imagenet] [--ratio 0.99]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import codec  # noqa: E402
from oracle import choco_oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="resnet50_imagenet")
    ap.add_argument("--ratio", type=float, default=0.99)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    lens = json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))[a.layout]
    n = sum(lens)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(n, generator=g, device=dev)
    g2 = torch.Generator(device=dev).manual_seed(12)
    xh = torch.randn(n, generator=g2, device=dev) * 0.5
    plan = codec.SegmentPlan(lens, a.ratio, dev)
    d = x.cpu().numpy() - xh.cpu().numpy()
    ov, oi, ks = O.topk_segmented(d, lens, a.ratio)
    for rep in range(a.reps):
        vals, idx = codec.topk_segmented(x, plan, xhat=xh)
        gi = idx.cpu().numpy().astype(np.int64)
        ws = next(iter(plan._ws.values()))
        nseg = len(lens)
        h = (nseg * 2048 * 4 + 255) // 256 * 256
        info = ws[2 * h: 2 * h + nseg * 16].cpu().numpy().view(np.uint32).reshape(nseg, 4)
        bad = 0
        off = 0
        for s, (m, k) in enumerate(zip(lens, ks)):
            a0 = plan.k_per_seg[:s]
            o0 = sum(a0)
            gs, os_ = gi[o0:o0 + k], oi[o0:o0 + k]
            if not np.array_equal(gs, os_):
                bad += 1
                keys = O.keys(d[off:off + m]).astype(np.int64)
                T = np.partition(keys, m - k)[m - k]
                print(f"rep {rep} seg {s} len {m} k {k}: oracle T {T:#x} (b1 {T >> 20}, b2 {(T >> 9) & 2047}); "
                      f"device b1 {info[s, 0]} kb {info[s, 1]} T {info[s, 2]:#x}; "
                      f"#diff {np.setxor1d(gs, os_).size} gpu-only {np.setdiff1d(gs, os_)[:5]} "
                      f"oracle-only {np.setdiff1d(os_, gs)[:5]} sorted {bool(np.all(np.diff(gs) > 0))}")
            off += m
        print(f"rep {rep}: {bad} bad segments of {nseg}")


if __name__ == "__main__":
    main()
