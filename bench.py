"""CHOCO compressor-path benchmark on MI355X.

One "step" = one CHOCO gossip round of the compressor path for every worker
(reference: CHOCO*Compressor.pipeline, dl_code/pcode/optim/parallel_choco_v.py:220-227):
compress the worker's device-resident delta buffer d, exchange the packed
message with its graph neighbours (RCCL send/recv over xGMI for N > 1), and
decompress-accumulate every received message (self included) into x_hat_i and
memory.  One process per GPU; each worker owns its own buffer (weak scaling).

    python bench.py [--gpus N --steps K --warmup W --workload topk|topk25m|qsgd|sign]

metric (BASELINE.json): compress+decompress GB/s = sum_r 4*n_r / max_r(step time).
roofline: the dominant kernel's algorithmic bytes / its HIP-event-timed duration
on its own stream, against 8 TB/s.  cpu_baseline: the reference's torch-CPU op
sequence (oracle/torch_port.py) on the host cores, rank 0 only, N = 1 only.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "compress+decompress GB/s (device-resident) on flat fp32 buffer, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)

WORKLOADS = {
    # name: (op, n per worker, parameter, dominant kernel)
    "topk": ("topk", 100_000_000, 0.99, "topk_stream"),
    "topk25m": ("topk", 25_000_000, 0.99, "topk_stream"),
    "qsgd": ("qsgd", 100_000_000, 4, "qsgd_quantize"),
    "sign": ("sign", 345_000_000, None, "sign_pack"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--workload", default="topk", choices=sorted(WORKLOADS))
    p.add_argument("--n", type=int, default=0, help="override elements per worker")
    p.add_argument("--nbuf", type=int, default=4, help="delta buffers compressed in rotation (one per step)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--no-e2e", action="store_true", help="skip the host-resident (PCIe-inclusive) leg")
    p.add_argument("--lib", default=None, help=argparse.SUPPRESS)
    p.add_argument("--no-kernel-events", action="store_true", help=argparse.SUPPRESS)  # diagnostic  # diagnostic variant (tools/build_variants.py)
    p.add_argument("--diag-evict", action="store_true", help=argparse.SUPPRESS)  # 1 GiB read after each step
    return p.parse_args()


class Worker:
    """Per-rank buffers and one compress -> exchange -> decompress round."""

    def __init__(self, args, rank, world, dev):
        from chocosgd_amd import codec
        from chocosgd_amd.communication import neighborhood
        self.codec = codec
        self.op, n, self.param, self.kernel = WORKLOADS[args.workload]
        self.n = args.n or n
        self.rank, self.world, self.dev = rank, world, dev
        self.nb = neighborhood(rank, world)
        self.peers = [r for r in self.nb if r != rank]
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        # The worker's delta x - x_hat.  Consecutive steps compress different
        # buffers (args.nbuf, independent draws), so each step selects a new
        # index set and the accumulate dirties new lines, as in training.
        self.ds = [torch.randn(self.n, generator=g, device=dev) for _ in range(max(1, args.nbuf))]
        self.d = self.ds[0]
        self.hat = torch.zeros(self.n, device=dev)
        self.mem = torch.zeros(self.n, device=dev)
        if self.op == "topk":
            self.k = codec.topk_k(self.n, self.param)
            self.msg = torch.empty(2 * self.k, dtype=torch.int32, device=dev)
        elif self.op == "qsgd":
            self.k = None
            nbytes = codec.qsgd_packed_bytes(self.n, self.param)
            self.msg = torch.empty(16 + nbytes, dtype=torch.uint8, device=dev)   # [norm (16 B) | planes]
        else:
            self.k = None
            self.msg = torch.empty(4 + codec.sign_words(self.n), dtype=torch.int32, device=dev)
        self.recv = {r: torch.empty_like(self.msg) for r in self.peers}
        self.step_id = 0

    def compress(self):
        c = self.codec
        self.d = self.ds[self.step_id % len(self.ds)]
        if self.op == "topk":
            c.topk(self.d, self.k, out=(self.msg[:self.k].view(torch.float32), self.msg[self.k:]))
        elif self.op == "qsgd":
            packed, norms, _ = c.qsgd_compress(self.d, self.param, seed=12345 + self.rank, offset=self.step_id)
            self.msg[16:].copy_(packed)
            self.msg[:4].view(torch.float32).copy_(norms)
        else:
            packed, norms = c.sign_compress(self.d)
            self.msg[4:].copy_(packed)
            self.msg[:1].view(torch.float32).copy_(norms)
        self.step_id += 1

    def exchange(self):
        if not self.peers:
            return
        ops = []
        for r in self.peers:
            ops.append(dist.P2POp(dist.isend, self.msg, r))
            ops.append(dist.P2POp(dist.irecv, self.recv[r], r))
        for w in dist.batch_isend_irecv(ops):
            w.wait()

    def decompress(self):
        c = self.codec
        ranks = list(self.nb.keys())
        msgs = [self.msg if r == self.rank else self.recv[r] for r in ranks]
        weights = [self.nb[r] for r in ranks]
        self_slot = ranks.index(self.rank)
        if self.op == "topk":
            for r, m, w in zip(ranks, msgs, weights):
                c.sparse_accumulate(m[:self.k].view(torch.float32), m[self.k:], self.mem, w,
                                    xhat_self=self.hat if r == self.rank else None)
        elif self.op == "qsgd":
            parts = [(m[16:], m[:4].view(torch.float32)) for m in msgs]
            c.qsgd_accumulate(parts, weights, self_slot, self.n, self.param, self.mem, xhat_self=self.hat)
        else:
            parts = [(m[4:], m[:1].view(torch.float32)) for m in msgs]
            c.sign_accumulate(parts, weights, self_slot, self.n, self.mem, xhat_self=self.hat)

    def step(self):
        self.compress()
        self.exchange()
        self.decompress()

    def kernel_bytes(self):
        """Algorithmic HBM bytes of ONE launch of the dominant kernel."""
        n = self.n
        if self.op == "topk":
            return 4 * n + 8 * self.k                    # read d once, write k (fp32 value, int32 index)
        if self.op == "qsgd":
            cw = 1
            while cw < self.param:
                cw <<= 1
            return 4 * n + n * cw // 8 + n // 8          # read d, write level + sign planes
        return 4 * n + 4 * ((n + 31) // 32)              # read d, write packed sign words


def e2e_rate(w, reps=5):
    """Host-resident leg (north star: the path starts and ends in host memory):
    pinned H2D of the worker's buffer -> compress -> D2H of the packed message
    -> H2D of that message (the receiver's copy) -> decompress-accumulate.
    Reported next to, never as, the device-resident value."""
    host_x = w.d.cpu().pin_memory()
    host_msg = torch.empty(w.msg.shape, dtype=w.msg.dtype).pin_memory()
    parts = {"h2d": [], "device": [], "d2h": [], "total": []}
    for i in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w.ds[w.step_id % len(w.ds)].copy_(host_x, non_blocking=True)  # the buffer compress() takes next
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        w.compress()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host_msg.copy_(w.msg, non_blocking=True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        w.msg.copy_(host_msg, non_blocking=True)
        w.decompress()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        if i:  # first round is a warm-up
            parts["h2d"].append(t1 - t0)
            parts["device"].append((t2 - t1) + (t4 - t3))
            parts["d2h"].append(t3 - t2)
            parts["total"].append(t4 - t0)
    med = {k: statistics.median(v) for k, v in parts.items()}
    return {"value": round(4 * w.n / med["total"] / 1e9, 3), "unit": "GB/s",
            "ms": {k: round(v * 1e3, 3) for k, v in med.items()},
            "msg_bytes": w.msg.numel() * w.msg.element_size(),
            "note": "pinned host buffers; H2D x, compress, D2H message, H2D message + decompress; median of "
                    f"{reps}"}


def cpu_baseline(w, threads):
    """Reference torch-CPU op sequence (oracle/torch_port.py) on the host cores."""
    from oracle import torch_port as P
    torch.set_num_threads(threads)
    n = w.n
    if w.op == "topk":
        d = w.d.cpu()
        hat, mem = torch.zeros(n), torch.zeros(n)

        def run():
            v, i = P.topk_compress(d, w.param)
            P.sparse_decompress(hat, mem, v, i, 1.0)
        sample = f"full {n}-element delta, top-k ratio {w.param}, compress + self decompress"
    elif w.op == "qsgd":
        d = w.d.cpu()
        hat, mem = torch.zeros(n), torch.zeros(n)

        def run():
            q = P.qsgd_compress(d, 2 ** w.param - 1)
            P.dense_decompress(hat, mem, q, 1.0)
        sample = f"full {n}-element delta, QSGD q={w.param}, compress + self decompress"
    else:
        m = min(n, 100_000_000)
        d = w.d[:m].cpu()
        hat, mem = torch.zeros(m), torch.zeros(m)

        def run():
            words, norm = P.sign_compress(d)
            P.sign_decompress(hat, mem, words, norm, m, 1.0)
        n = m
        sample = f"first {m} elements of the delta, sign+L1 norm compress + self decompress"
    run()  # warm-up
    ts = []
    budget = time.perf_counter() + 25.0
    while len(ts) < 3 and (not ts or time.perf_counter() < budget):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    return {"value": round(4 * n / med / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{sample}; median of {len(ts)} after 1 warm-up; {med * 1e3:.1f} ms each"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    from chocosgd_amd import _lib, codec
    if args.lib:
        _lib.load(args.lib)
    codec.lib()
    w = Worker(args, rank, world, dev)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    if args.diag_evict:
        junk = torch.ones(256 * 1024 * 1024, device=dev)
        sink = torch.empty(1, device=dev)
        inner = w.step

        def evicting_step():
            inner()
            torch.sum(junk, dim=0, keepdim=True, out=sink)
        w.step = evicting_step
    for _ in range(args.warmup):
        w.step()
    barrier()
    # Only the dominant kernel's launches carry timing events inside the timed
    # region: each event pair costs ~3 us of GPU time per launch (measured: all
    # four kernels timed made the top-k step 13 us slower).
    codec.profile_reset()
    codec.profile_filter(w.kernel)
    codec.profile_enable(not args.no_kernel_events)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        w.step()
    barrier()
    elapsed = time.perf_counter() - t0
    codec.profile_enable(False)
    ktot, kcnt = codec.profile_read(w.kernel)
    # the other kernels of the step: an untimed pass with every launch timed
    codec.profile_reset()
    codec.profile_filter(None)
    codec.profile_enable(True)
    for _ in range(min(args.steps, 10)):
        w.step()
    barrier()
    codec.profile_enable(False)
    kernels = {}
    for name in ("topk_stream", "topk_finish", "sparse_accumulate", "qsgd_norm", "qsgd_quantize", "qsgd_accumulate", "sign_pack",
                 "sign_accumulate"):
        t, c = (ktot, kcnt) if name == w.kernel else codec.profile_read(name)
        if c:
            kernels[name] = round(t / c * 1e3, 2)  # us per launch
    t_max = elapsed
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    ms_per_step = t_max / args.steps * 1e3
    value = world * 4 * w.n * args.steps / t_max / 1e9
    if rank == 0:
        avg_s = ktot / max(kcnt, 1) / 1e3
        achieved = w.kernel_bytes() / avg_s / 1e9 if kcnt else None
        traffic = None
        tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tf):
            entry = json.load(open(tf)).get(f"{args.workload}:{w.n}")
            traffic = int(entry["bytes"]) if entry else None
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": {"topk": "topk_k1pct_per_worker", "topk25m": "topk_k1pct_25M",
                                    "qsgd": "qsgd_q4_per_worker", "sign": "sign_norm_per_worker"}[args.workload],
                       "n_per_worker": w.n, "k_per_worker": w.k,
                       "graph": "self" if world == 1 else ("complete" if world == 2 else "ring"),
                       "step": "compress+exchange+decompress-accumulate", "parallelism": f"gossip{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": traffic, "kernel": w.kernel, "kernel_us": round(avg_s * 1e6, 2),
                         "algorithmic_bytes_per_launch": w.kernel_bytes()},
            "kernels_us": kernels,
            "kernels_note": "dispatch-attached HIP events: the dominant kernel inside the timed region (only its "
                            "launches carry events there), the others in an untimed pass after it",
            "e2e": None,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_e2e:
            out["e2e"] = e2e_rate(w)
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count())
            out["cpu_baseline"] = cpu_baseline(w, threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
