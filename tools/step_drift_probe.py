"""How far the k-th key of the bench's realistic CHOCO step (bench.py step_topk /
step_topk_r50: apply_gradient + fused consensus step + compress + ring-3 loopback receive)
moves between calls, in units of k: for step t's exact threshold T_t, the next call's delta
holds k (1 + e) keys >= T_t; a carried window of margin m (in k) hits when |e| < m.
Warm start off, so every call samples (the drift is measured, not the warm path).
    python tools/step_drift_probe.py [step_topk|step_topk_r50] [steps] [extra bench args...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "step_topk"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
args = bench.parse(["--workload", wl, "--ring3-loopback"] + sys.argv[3:])
dev = torch.device("cuda", 0)
from chocosgd_amd import codec  # noqa: E402

codec.lib().choco_topk_set_warm_start(0)
w = bench.Worker(args, 0, 1, dev)
if w.plan is not None:
    ks = [int(v) for v in w.plan.k_per_seg]
    offs = torch.tensor([0] + list(torch.tensor(ks).cumsum(0)), dtype=torch.int64)
for t in range(steps):
    w.step()
    vals = w.msg[:w.k].view(torch.float32)
    # the next call's delta, formed as the fused pass will form it
    xx = w.x.clone()
    if w.grads is not None:  # the next step's draw, from a copy of the generator's state
        gs = w.grad_gen.get_state()
        g = torch.empty_like(xx).normal_(0.0, w.grad_scale, generator=w.grad_gen)
        w.grad_gen.set_state(gs)
        xx.add_(g, alpha=-w.grad_lr)
    xx = xx + bench.GAMMA * (w.mem - w.hat)
    d = (xx - w.hat).abs()
    if w.plan is None:
        T = vals.abs().min()
        e = float((d >= T).sum()) / w.k - 1.0
        print(f"{t:3d} T {float(T):.6g}  next-call e = {e:+.4f} k", flush=True)
    else:
        es = []
        lo = 0
        for s, (ks_, ln) in enumerate(zip(ks, w.plan.seg_lens)):
            v = vals[int(offs[s]):int(offs[s + 1])]
            Ts = v.abs().min()
            c = float((d[lo:lo + ln] >= Ts).sum())
            es.append(c / ks_ - 1.0)
            lo += ln
        es_t = torch.tensor(es)
        big = [i for i, ln in enumerate(w.plan.seg_lens) if ln >= 16384 * 2]
        eb = es_t[big]
        print(f"{t:3d} segments {len(es)}: e median {float(es_t.median()):+.4f} k, multi-tile segments |e| max "
              f"{float(eb.abs().max()):.4f} median {float(eb.abs().median()):.4f}", flush=True)
