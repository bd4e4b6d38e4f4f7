"""The top-k status word reaches the host at the very next call.

Run with the `poll1` diagnostic build (tools/build_variants.py poll1: every bounded wait
of the exact fallback gives up at once), so a call that takes the exact fallback flags its
output invalid:
    CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_poll1.so python tools/status_probe.py
Call 1 (an all-equal delta: the sampled window cannot separate the k-th key, the exact
fallback runs) gives up; the stream is synchronised once (the call has run on the GPU);
call 2 must raise RuntimeError before it launches anything -- the check reads the pinned
host mirror the device wrote (choco_topk_host_status), no copy, no synchronisation.
Exit 0 when call 2 raised, 1 otherwise.  Run it once.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import codec  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
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
