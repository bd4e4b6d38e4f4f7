"""The top-k status word reaches the host at the very next call.

Run with the `poll1` diagnostic build (tools/build_variants.py poll1: every bounded wait
of the exact fallback gives up at once), so a call that takes the exact fallback flags its
output invalid:
    CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_poll1.so python tools/status_probe.py
Call 1 (an all-equal delta: the sampled window cannot separate the k-th key, the exact
fallback runs) gives up; the stream is synchronised once (the call has run on the GPU);
call 2 must raise RuntimeError before it launches anything -- the check reads the pinned
host mirror the device wrote (choco_topk_host_status), no copy, no synchronisation.
Exit 0 when call 2 raised, 1 otherwise.  Run it once.  (First the same for a segmented
workspace whose missed windows run S4w's shared exact select.)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import codec  # noqa: E402


def segmented(dev):
    """The same through the segmented path: a warm call whose windows miss runs the shared
    exact select of the missed segments (csrc/wide.h) in S4w, which gives up in this build."""
    lens = [1_000_000, 300_000, 50_000]
    plan = codec.SegmentPlan(lens, 0.99, dev)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(sum(lens), generator=g, device=dev)
    codec.topk_segmented(x, plan)        # cold
    codec.topk_segmented(x, plan)        # warm, the windows hold
    codec.topk_segmented(x * 100, plan)  # warm, the windows miss: the shared select gives up
    torch.cuda.synchronize()
    misses = codec.topk_fallback_count(plan=plan)
    try:
        codec.topk_segmented(x, plan)    # must raise before launching
    except RuntimeError as e:
        print(f"segmented: the call after the miss raised (misses counted: {misses}): {e}")
        return 0
    print(f"segmented: the call after the miss did NOT raise (misses counted: {misses})")
    return 1


def main():
    dev = torch.device("cuda", 0)
    if segmented(dev):
        return 1
    n = 4_000_000
    k = codec.topk_k(n, 0.99)
    x = torch.full((n,), 0.5, device=dev)
    codec.topk(x, k)                 # call 1: exact fallback, gives up (poll1 build)
    torch.cuda.synchronize()
    fallbacks = codec.topk_fallback_count()
    try:
        codec.topk(x, k)             # call 2: must raise before launching
    except RuntimeError as e:
        print(f"call 2 raised (fallbacks counted: {fallbacks}): {e}")
        # the status was cleared by the raise: call 3 runs (and gives up again in this build)
        codec.topk(x, k)
        torch.cuda.synchronize()
        return 0
    print(f"call 2 did NOT raise (fallbacks counted: {fallbacks})")
    return 1


if __name__ == "__main__":
    sys.exit(main())
