"""Is the bench step host-bound?  Enqueue time of K steps (no sync) against their GPU
time, for a bench workload, with and without the in-region kernel events.

    python tools/host_overhead.py [--workload topk] [--steps 20]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="topk")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from chocosgd_amd import codec
    sys.argv = [sys.argv[0], "--workload", a.workload]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    w = bench.Worker(args, 0, 1, dev)
    comp_k, _ = bench.STAGES[w.op]
    for ev in (False, True):
        codec.profile_reset()
        codec.profile_filter(comp_k)
        codec.profile_enable(ev)
        for _ in range(5):
            w.step()
        torch.cuda.synchronize()
        for rep in range(3):
            t0 = time.perf_counter()
            for _ in range(a.steps):
                w.step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"events={ev} enqueue {(t1 - t0) / a.steps * 1e6:7.1f} us/step  "
                  f"gpu-bound total {(t2 - t0) / a.steps * 1e6:7.1f} us/step")
        codec.profile_enable(False)
        codec.profile_reset()
    # host cost of the pieces of one step
    torch.cuda.synchronize()
    for name, fn in (("compress", w.compress), ("decompress", w.decompress)):
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"{name:10s} enqueue {(t1 - t0) / a.steps * 1e6:7.1f} us")


if __name__ == "__main__":
    main()
