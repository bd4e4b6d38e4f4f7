"""Per-call warm / cold / miss trace of the top-k on the bench's realistic step (bench.py
step_topk_r50 / step_topk --ring3-loopback: apply_gradient + fused consensus step +
compress + ring-3 receive), over a long run: one character per call --
  segmented: W warm, M warm with a window miss (S4w's shared exact select), C cold (S1 + S2),
             c cold whose shadow check missed (the window the previous call prepared would
             not have held this call's k-th key);
  flat:      W warm, F exact fallback (the carried window missed), S sampled window (a cold
             run's K1 launch or K2 prologue sample).
Every call is synchronised (the counters are read after it), so the host sees a miss flag
at the very next call; the bench's unsynchronised steps see it later.
    python tools/seg_warm_trace.py [steps] [step_topk_r50|step_topk] [extra bench args...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 600
wl = sys.argv[2] if len(sys.argv) > 2 else "step_topk_r50"
args = bench.parse(["--workload", wl, "--ring3-loopback"] + sys.argv[3:])
dev = torch.device("cuda", 0)
from chocosgd_amd import codec, _lib  # noqa: E402

w = bench.Worker(args, 0, 1, dev)
SHADOW = 64  # topk_seg.hip kSegShadowOffset: (misses << 32) | checks


def counters():
    if w.plan is None:
        return (codec.launch_count("topk_bounds") + codec.topk_workspace_word(_lib.TOPK_K2_SAMPLES_OFFSET),
                codec.topk_workspace_word(_lib.TOPK_FALLBACKS_OFFSET), 0)
    return (codec.launch_count("topk_seg_hist"), codec.topk_workspace_word(_lib.TOPK_FALLBACKS_OFFSET, plan=w.plan),
            codec.topk_workspace_word(SHADOW + 4, plan=w.plan))


line = []
prev = counters()
for t in range(steps):
    w.step()
    cur = counters()
    cold = cur[0] > prev[0]
    if w.plan is None:
        line.append("F" if cur[1] > prev[1] else ("S" if cold else "W"))
    elif cold:
        line.append("c" if cur[2] > prev[2] else "C")
    else:
        line.append("M" if cur[1] > prev[1] else "W")
    prev = cur
    if len(line) == 100:
        print(f"{t - 99:5d} {''.join(line)}", flush=True)
        line = []
if line:
    print(f"{steps - len(line):5d} {''.join(line)}", flush=True)
