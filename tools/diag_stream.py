"""GPU diagnostic: per-kernel HBM rate of the codec's streaming kernels, hot
(back-to-back launches) and cold (a 1 GiB READ between launches evicts the
256 MiB Infinity Cache without leaving dirty lines to write back), next to torch reductions and copies on the same data.

    python tools/diag_stream.py [--n 100000000]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import codec  # noqa: E402


def ev_time(fn, reps, flush=None):
    ts = []
    for _ in range(reps):
        if flush is not None:
            flush()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1e3  # median, us


def prof_time(fn, names, reps, flush=None):
    codec.profile_reset()
    codec.profile_enable(True)
    for _ in range(reps):
        if flush is not None:
            flush()
        fn()
    torch.cuda.synchronize()
    codec.profile_enable(False)
    out = {}
    for nm in names:
        t, c = codec.profile_read(nm)
        out[nm] = t / max(c, 1) * 1e3
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default=None, help="diagnostic variant .so (tools/build_variants.py)")
    ap.add_argument("--only", default=None, help="comma list of rows to run (topk,qsgd,sign,torch)")
    ap.add_argument("--modes", default="hot,cold")
    ap.add_argument("--ratios", default="0.99", help="top-k compression ratios (k = n * (1 - ratio))")
    a = ap.parse_args()
    if a.lib:
        from chocosgd_amd import _lib
        _lib.load(a.lib)
    only = set(a.only.split(",")) if a.only else {"topk", "qsgd", "sign", "torch"}
    n, reps = a.n, a.reps
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    d = torch.randn(n, generator=g, device=dev)
    junk = torch.empty(256 * 1024 * 1024, device=dev)  # 1 GiB
    y = torch.empty_like(d)
    codec.lib()

    junk.fill_(1.0)
    sink = torch.empty(1, device=dev)

    def flush():
        torch.sum(junk, dim=0, keepdim=True, out=sink)

    GB = 4 * n / 1e9
    rows = []
    for mode, fl in (("hot", None), ("cold", flush)):
        if mode not in a.modes.split(","):
            continue
        if "torch" in only:
            t = ev_time(lambda: torch.sum(d), reps, fl); rows.append((mode, "torch.sum", t, GB))
            t = ev_time(lambda: torch.linalg.vector_norm(d), reps, fl); rows.append((mode, "torch.norm", t, GB))
            t = ev_time(lambda: y.copy_(d), reps, fl); rows.append((mode, "torch.copy", t, 2 * GB))
        if "topk" in only:
            for ratio in [float(v) for v in a.ratios.split(",")]:
                k = codec.topk_k(n, ratio)
                r = prof_time(lambda: codec.topk(d, k), ["topk_stream"], reps, fl)
                rows.append((mode, f"topk_stream@{ratio}", r["topk_stream"], GB))
                if not a.lib:
                    t = ev_time(lambda: codec.topk(d, k), reps, fl)
                    rows.append((mode, f"topk(all)@{ratio}", t, GB))
        if "qsgd" in only:
            r = prof_time(lambda: codec.qsgd_compress(d, 4, seed=1, offset=0), ["qsgd_norm", "qsgd_quantize"],
                          reps, fl)
            rows.append((mode, "qsgd_norm", r["qsgd_norm"], GB))
            rows.append((mode, "qsgd_quantize", r["qsgd_quantize"], GB * 1.125))
        if "sign" in only:
            r = prof_time(lambda: codec.sign_compress(d), ["sign_pack"], reps, fl)
            rows.append((mode, "sign_pack", r["sign_pack"], GB * (1 + 1 / 32)))
    for mode, nm, us, gb in rows:
        print(f"{os.path.basename(a.lib or 'product'):28s} {mode:4s} {nm:22s} {us:9.1f} us  {gb / (us * 1e-6):8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
