"""CHOCO compressor-path benchmark on MI355X.

One "step" = one CHOCO gossip round of the compressor path for every worker
(reference: CHOCO*Compressor.pipeline, dl_code/pcode/optim/parallel_choco_v.py:220-227):
compress the worker's device-resident delta buffer d, exchange the packed
message with its graph neighbours (RCCL send/recv over xGMI for N > 1), and
decompress-accumulate every received message (self included) into x_hat_i and
memory.  One process per GPU; each worker owns its own buffer (weak scaling).

    python bench.py [--gpus N --steps K --warmup W --workload topk|...]

`--gpus N` without a launcher starts N rank processes itself (before this
process touches the GPU); under torch.distributed.run the ranks come from the
environment.

The step_* workloads run the whole CHOCO step of ParallelCHOCO_V (parallel_choco_v.py:
116-155, after apply_gradient): the consensus step x += gamma (memory - x_hat) FUSED into
the compressor's first pass (include/choco_codec.h), compress of d = x_new - x_hat,
exchange, accumulate; `--unfused` runs the consensus step as its own pass first, as the
reference does (optim/utils.py:67-72), for the A/B.

metric (BASELINE.json): compress+decompress GB/s = sum_r 4*n_r / max_r(step time).
roofline: per STAGE of the step (compress, decompress), algorithmic bytes
 / the stage's kernel time from dispatch-attached HIP events;
`roofline` is the stage that takes the most time (measured, not assumed): its
kernels carry events inside the timed region, the other stage's in an untimed
pass after it.  cpu_baseline: the reference's torch-CPU op sequence
(oracle/torch_port.py) on the host cores, rank 0 only, N = 1 only.
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "compress+decompress GB/s (device-resident) on flat fp32 buffer, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)

# name: op, elements per worker, parameter (ratio or q), config label
WORKLOADS = {
    "topk": ("topk", 100_000_000, 0.99, "topk_k1pct_per_worker"),
    "topk25m": ("topk", 25_000_000, 0.99, "topk_k1pct_25M"),
    "topk_r50": ("topk_seg", 25_557_032, 0.99, "topk_k1pct_resnet50_161seg"),
    "randk": ("randk", 100_000_000, 0.99, "randk_k1pct_per_worker"),
    "qsgd": ("qsgd", 100_000_000, 4, "qsgd_q4_per_worker"),
    "sign": ("sign", 345_000_000, None, "sign_norm_per_worker"),
    "step_topk": ("topk", 100_000_000, 0.99, "choco_step_gossip_topk_k1pct"),
    "step_sign": ("sign", 345_000_000, None, "choco_step_gossip_sign_norm"),
    "step_qsgd": ("qsgd", 100_000_000, 4, "choco_step_gossip_qsgd_q4"),
    # the drop-in's per-tensor layout (ResNet-50's 161 tensors, create_optimizer.py:15-24)
    "step_sign_r50": ("sign", 25_557_032, None, "choco_step_gossip_sign_norm_resnet50_161seg"),
    "step_qsgd_r50": ("qsgd", 25_557_032, 4, "choco_step_gossip_qsgd_q4_resnet50_161seg"),
    "step_topk_r50": ("topk_seg", 25_557_032, 0.99, "choco_step_gossip_topk_k1pct_resnet50_161seg"),
    "sign_r50": ("sign", 25_557_032, None, "sign_norm_resnet50_161seg"),
    "qsgd_r50": ("qsgd", 25_557_032, 4, "qsgd_q4_resnet50_161seg"),
    "randk_r50": ("randk_seg", 25_557_032, 0.99, "randk_k1pct_resnet50_161seg"),
}
GAMMA = 0.9  # consensus_stepsize (parameters.py:126 default)

# kernels (profile names) of each stage
STAGES = {
    "topk": (["topk_bounds", "topk_stream", "topk_finish", "topk_exact", "topk_all"],
             ["sparse_accumulate"]),
    "topk_seg": (["topk_seg_hist", "topk_seg_collect", "topk_seg_fine", "topk_seg_count", "topk_seg_bin",
                  "topk_seg_emit", "topk_bounds", "topk_stream", "topk_finish"], ["sparse_accumulate"]),
    "randk": (["randk_count", "randk_tile"], ["sparse_accumulate"]),
    "randk_seg": (["randk_count", "randk_tile"], ["sparse_accumulate"]),
    "qsgd": (["qsgd_norm", "qsgd_quantize"], ["qsgd_accumulate"]),
    "sign": (["sign_pack"], ["sign_accumulate"]),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--workload", default="topk", choices=sorted(WORKLOADS))
    p.add_argument("--n", type=int, default=0, help="override elements per worker")
    p.add_argument("--nbuf", type=int, default=4, help="delta buffers compressed in rotation (one per step)")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="gloo: messages staged through host memory (comm_device=cpu); lets ranks share a GPU")
    p.add_argument("--unfused", action="store_true",
                   help="step_* workloads: the consensus step as its own pass (the reference's order)")
    p.add_argument("--fold", action="store_true",
                   help="top-k: fold the self message's uncompress (x_hat, and memory when the self rank is first) "
                        "into the compress emission (choco_topk_compress_accumulate)")
    p.add_argument("--ring3-loopback", action="store_true",
                   help="one GPU: each step applies the self message plus two neighbour messages, no exchange -- a "
                        "ring worker's receive (cfg 4).  topk/randk workloads: the neighbours' messages are compressed "
                        "once from other resident deltas; step_* workloads: they are this worker's own messages of "
                        "the two previous steps (same codec, same magnitudes, other index sets)")
    p.add_argument("--grad-lr", type=float, default=0.1,
                   help="step_* workloads: apply_gradient (optim/utils.py:13-47, no momentum / weight decay) "
                        "x -= lr * g at the start of every step; 0 = off (round-5 steps)")
    p.add_argument("--grad-scale", type=float, default=0.01,
                   help="step_* workloads: the synthetic gradient g ~ N(0, scale^2), a fresh seeded draw every step "
                        "(with the gradient on, x_hat and memory start as copies of x, as the reference's do)")
    p.add_argument("--burn-in", type=int, default=None,
                   help="step_* workloads with the gradient on: untimed steps run before the warm-up, so the timed "
                        "steps are those of a running training job, not its first few (default 200; the delta "
                        "starts at 0 and its k-th key moves by large factors over the first ~50 steps)")
    p.add_argument("--defer-receive", action="store_true",
                   help="step_* workloads: apply each step's received messages inside the NEXT step's first pass "
                        "(receive + consensus step + first compress pass in one kernel; same x / x_hat / memory)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the host-resident (PCIe-inclusive) leg")
    p.add_argument("--lib", default=None, help=argparse.SUPPRESS)
    p.add_argument("--no-kernel-events", action="store_true", help=argparse.SUPPRESS)  # diagnostic
    p.add_argument("--dist-timeout", type=float, default=300.0,
                   help="seconds for init_process_group and every collective before a rank gives up")
    p.add_argument("--die-before-exchange", type=int, default=None, help=argparse.SUPPRESS)  # launcher test
    return p.parse_args(argv)


def traffic_key(args):
    """The workload key of profiles/pmc_traffic.json (tools/pmc_traffic.py's 3rd argument;
    scripts/gpu_measure.sh derives it from the same flags)."""
    key = args.workload
    if args.ring3_loopback:
        key += "_ring3"
    if getattr(args, "defer_receive", False):
        key += "_deferred"
    if args.workload.startswith("step_") and getattr(args, "grad_lr", 0.1) <= 0:
        key += "_nograd"
    return key


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_exit_code(rc):
    """A child's return code as this launcher's exit code: 0 only for 0.  Popen reports a
    rank killed by signal s as -s, which max() over return codes would have hidden; it maps
    to 128 + s, as a shell reports it."""
    if rc is None or rc == 0:
        return 0 if rc == 0 else 1
    return 128 - rc if rc < 0 else rc


def wait_ranks(procs, poll_s=0.2):
    """Wait for every rank; on the first one that fails (non-zero exit or a signal),
    terminate its siblings (then kill those that ignore it) so none is left blocked in a
    collective, and return that rank's exit code.  0 when all ranks exit 0."""
    first = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and first == 0:
                first = rank_exit_code(rc)
                print(f"bench.py: rank pid {p.pid} exited with {rc}; stopping {len(live)} sibling rank(s)",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
                deadline = time.time() + 10.0
                for q in live:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
                break
        if live:
            time.sleep(poll_s)
    return first


def spawn_ranks(n, argv=None):
    """`python bench.py --gpus N` with no launcher: one child process per rank, started
    before this process makes any GPU call (it never makes one).  Returns 0 only when every
    rank exits 0; the first failing rank (exit code or signal) stops the others."""
    port = str(_free_port())
    procs = []
    argv = sys.argv[1:] if argv is None else argv
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    return wait_ranks(procs)


class Worker:
    """Per-rank buffers and one compress -> exchange -> decompress round."""

    def __init__(self, args, rank, world, dev):
        import torch
        from chocosgd_amd import codec
        from chocosgd_amd.communication import neighborhood
        self.torch = torch
        self.codec = codec
        self.op, n, self.param, self.label = WORKLOADS[args.workload]
        self.step_mode = args.workload.startswith("step_")
        self.unfused = self.step_mode and args.unfused
        if self.unfused:
            self.label += "_unfused"
        self.defer = self.step_mode and args.defer_receive and not self.unfused
        if args.defer_receive and not self.defer:
            raise SystemExit("--defer-receive: step_* workloads without --unfused only")
        if self.defer:
            if self.op not in ("qsgd", "sign"):
                raise SystemExit("--defer-receive: step_qsgd / step_sign only")
            self.label += "_deferred_receive"
        self.pending = None  # (messages, weights, self slot) the next step's first pass applies
        self.backend = args.backend
        self.rank, self.world, self.dev = rank, world, dev
        self.nb = neighborhood(rank, world)
        self.ranks = list(self.nb.keys())
        self.peers = [r for r in self.ranks if r != rank]
        self.weights = [self.nb[r] for r in self.ranks]
        self.self_slot = self.ranks.index(rank)
        # self-message fold (top-k): x_hat always; memory only when the self message is the
        # first one applied to it (ascending rank order, parallel_choco_v.py:291-310)
        self.fold = bool(args.fold) and self.op == "topk"
        self.fold_mem = self.fold and self.self_slot == 0
        self.plan = None
        self.seg_off, self.nseg = None, 1  # per-tensor layout of the dense codecs (_r50 workloads)
        if self.op in ("topk_seg", "randk_seg") or args.workload.endswith("_r50"):
            with open(os.path.join(ROOT, "tests", "golden", "layouts.json")) as f:
                lens = json.load(f)["resnet50_imagenet"]
            n = sum(lens)
            if self.op in ("topk_seg", "randk_seg"):
                self.plan = codec.SegmentPlan(lens, self.param, dev)
            else:
                if args.n:
                    raise SystemExit("--n: not with a per-tensor layout")
                self.seg_off = torch.tensor([0] + [int(v) for v in torch.tensor(lens).cumsum(0)], dtype=torch.int64,
                                            device=dev)
                self.nseg = len(lens)
        self.n = args.n or n
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        # The worker's delta x - x_hat.  Consecutive steps compress different
        # buffers (args.nbuf, independent draws), so each step selects a new
        # index set and the accumulate dirties new lines, as in training.
        if self.step_mode:
            # x, x_hat, memory resident; x moves every step (the consensus step), so every
            # step selects a new index set
            self.x = torch.randn(self.n, generator=g, device=dev)
            if args.grad_lr > 0:
                # the reference's start: x_hat_i and memory are copies of the parameters
                # (parallel_choco_v.py:94-97); the gradient then drives the delta
                self.hat = self.x.clone()
                self.mem = self.x.clone()
            else:
                # round 5's synthetic state (no gradient: the delta would stay 0)
                self.hat = self.x + 0.1 * torch.randn(self.n, generator=g, device=dev)
                self.mem = self.hat + 0.05 * torch.randn(self.n, generator=g, device=dev)
            self.ds = [self.x]
        else:
            self.ds = [torch.randn(self.n, generator=g, device=dev) for _ in range(max(1, args.nbuf))]
            self.hat = torch.zeros(self.n, device=dev)
            self.mem = torch.zeros(self.n, device=dev)
        self.d = self.ds[0]
        self.k = None
        if self.op in ("topk", "randk"):
            self.k = codec.topk_k(self.n, self.param)
            self.msg = torch.empty(2 * self.k, dtype=torch.int32, device=dev)
        elif self.op in ("topk_seg", "randk_seg"):
            self.k = self.plan.k_total
            self.msg = torch.empty(2 * self.k, dtype=torch.int32, device=dev)
        elif self.op == "qsgd":  # [norms (16-B padded) | planes]; compress writes in place
            self.msg, self.wire = codec.qsgd_wire(self.n, self.param, self.nseg, dev)
        else:  # [norms (16-B padded) | words]
            self.msg, self.wire = codec.sign_wire(self.n, self.nseg, dev)
        self.recv = {r: torch.empty_like(self.msg) for r in self.peers}
        # deferred sign receive: this step's words are packed in the pass that reads the previous
        # step's (own) message, so the own message alternates between two buffers
        self.msg_pp = [self.msg, torch.zeros_like(self.msg)] if (self.defer and self.op == "sign") else None
        self.loop_sets = None
        self.ring_msgs = None
        if args.ring3_loopback and self.step_mode:
            if world != 1:
                raise SystemExit("--ring3-loopback: --gpus 1 only")
            # a ring worker's neighbourhood {r-1, r, r+1} (weights 1/3, the self message second);
            # the neighbours' messages are this worker's own of steps t-1 and t-2: four message
            # buffers in rotation (the deferred receive still reads step t-1's while step t writes)
            self.ranks, self.self_slot = ["left", rank, "right"], 1
            self.weights = [1.0 / 3] * 3
            self.fold, self.fold_mem = False, False
            self.ring_msgs = [self.msg] + [torch.zeros_like(self.msg) for _ in range(3)]
            self.msg_pp = None
            self.recv = {"left": self.ring_msgs[3], "right": self.ring_msgs[2]}
            self.label += "_ring3_loopback"
        elif args.ring3_loopback:
            if self.op not in ("topk", "topk_seg", "randk") or world != 1:
                raise SystemExit("--ring3-loopback: sparse workloads (or step_*) at --gpus 1 only")
            # a ring worker's neighbourhood {r-1, r, r+1} (weights 1/3, the self message second):
            # the two neighbour messages come from other deltas, compressed once per rotation slot
            self.ranks, self.self_slot = ["left", rank, "right"], 1
            self.weights = [1.0 / 3] * 3
            self.fold_mem = False
            self.loop_sets = []
            for j in range(len(self.ds)):
                pair = {}
                for side, sd in (("left", 5000 + 2 * j), ("right", 5001 + 2 * j)):
                    gj = torch.Generator(device=dev).manual_seed(sd)
                    dj = torch.randn(self.n, generator=gj, device=dev)
                    m = torch.empty_like(self.msg)
                    vv, ii = m[:self.k].view(torch.float32), m[self.k:]
                    if self.op == "topk":
                        codec.topk(dj, self.k, out=(vv, ii))
                    elif self.op == "topk_seg":
                        codec.topk_segmented(dj, self.plan, out=(vv, ii))
                    else:
                        codec.randk(dj, self.k, seed=777 + sd, offset=0, out=(vv, ii))
                    pair[side] = m
                    del dj
                self.loop_sets.append(pair)
            self.recv = self.loop_sets[0]
            self.label += "_ring3_loopback"
        # apply_gradient (optim/utils.py:13-47; momentum and weight decay 0): x -= lr * g at the
        # start of every step, g a FRESH seeded draw N(0, scale^2) each step
        self.grads, self.grad_lr, self.grad_scale, self.grad_events = None, 0.0, 0.0, None
        if self.step_mode and args.grad_lr > 0:
            self.grad_gen = torch.Generator(device=dev).manual_seed(3000 + rank)
            self.grads = torch.empty(self.n, device=dev)
            self.grad_lr, self.grad_scale = args.grad_lr, args.grad_scale
            self.label += f"_grad_lr{args.grad_lr:g}_scale{args.grad_scale:g}"
        if self.backend == "gloo":
            self.msg_h = torch.empty(self.msg.shape, dtype=self.msg.dtype).pin_memory()
            self.recv_h = {r: torch.empty_like(self.msg_h).pin_memory() for r in self.peers}
        self.step_id = 0

    def compress(self):
        c = self.codec
        torch = self.torch
        self.d = self.ds[self.step_id % len(self.ds)]
        if self.loop_sets:
            self.recv = self.loop_sets[self.step_id % len(self.loop_sets)]
        if self.ring_msgs:
            t = self.step_id
            self.msg = self.ring_msgs[t % 4]
            if self.op in ("qsgd", "sign"):
                self.wire = self._parts(self.msg)
            self.recv = {"left": self.ring_msgs[(t - 1) % 4], "right": self.ring_msgs[(t - 2) % 4]}
        if self.step_mode:
            if self.grads is not None:
                ev = None
                if self.grad_events is not None:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record()
                self.grads.normal_(0.0, self.grad_scale, generator=self.grad_gen)
                self.x.add_(self.grads, alpha=-self.grad_lr)
                if ev:
                    ev[1].record()
                    self.grad_events.append(ev)
            self.compress_step()
        elif self.op == "topk":
            c.topk(self.d, self.k, out=(self.msg[:self.k].view(torch.float32), self.msg[self.k:]),
                   fold=self._fold_args())
        elif self.op == "topk_seg":
            c.topk_segmented(self.d, self.plan, out=(self.msg[:self.k].view(torch.float32), self.msg[self.k:]))
        elif self.op == "randk_seg":
            c.randk_segmented(self.d, self.plan, seed=12345 + self.rank, offset=self.step_id,
                              out=(self.msg[:self.k].view(torch.float32), self.msg[self.k:]))
        elif self.op == "randk":
            # one seed per worker, the step number as the stream offset (include/choco_codec.h)
            c.randk(self.d, self.k, seed=12345 + self.rank, offset=self.step_id,
                    out=(self.msg[:self.k].view(torch.float32), self.msg[self.k:]))
        elif self.op == "qsgd":
            c.qsgd_compress(self.d, self.param, seed=12345 + self.rank, offset=self.step_id, out=self.wire,
                            **self._seg())
        else:
            c.sign_compress(self.d, out=self.wire, **self._seg())
        self.step_id += 1

    def compress_step(self):
        """consensus step (fused, or its own pass with --unfused) + compress of x - x_hat"""
        c, torch = self.codec, self.torch
        g = (self.mem, GAMMA)
        if self.unfused:
            c.gossip_step(self.x, self.mem, self.hat, GAMMA)
            g = None
        if self.op == "topk":
            c.topk(self.x, self.k, xhat=self.hat, out=(self.msg[:self.k].view(torch.float32), self.msg[self.k:]),
                   gossip=g, fold=self._fold_args())
        elif self.op == "topk_seg":
            c.topk_segmented(self.x, self.plan, xhat=self.hat,
                             out=(self.msg[:self.k].view(torch.float32), self.msg[self.k:]), gossip=g)
        elif self.op == "qsgd" and self.pending is not None:
            # the previous step's receive + this step's consensus step + norm pass, one kernel
            parts, weights, slot = self.pending
            self.pending = None
            c.qsgd_recv_gossip_norms(parts, weights, slot, self.x, self.mem, self.hat, GAMMA, self.param,
                                     out=self.wire[1], **self._seg())
            c.qsgd_compress(self.x, self.param, xhat=self.hat, norm_in=self.wire[1], seed=12345 + self.rank,
                            offset=self.step_id, out=self.wire, **self._seg())
        elif self.op == "qsgd":
            c.qsgd_compress(self.x, self.param, xhat=self.hat, seed=12345 + self.rank, offset=self.step_id,
                            gossip=g, out=self.wire, **self._seg())
        elif self.pending is not None:  # sign: receive + consensus step + pack, one kernel
            parts, weights, slot = self.pending
            self.pending = None
            if self.msg_pp:
                self.msg = self.msg_pp[self.step_id % 2]
                self.wire = self._parts(self.msg)
            c.sign_recv_gossip_compress(parts, weights, slot, self.x, self.mem, self.hat, GAMMA, out=self.wire,
                                        **self._seg())
        else:
            c.sign_compress(self.x, xhat=self.hat, gossip=g, out=self.wire, **self._seg())

    def _seg(self):
        return {"seg_off": self.seg_off, "nseg": self.nseg} if self.nseg > 1 else {}

    def _parts(self, m):
        """(payload, norms) views of a dense codec's wire message (codec.sign_wire / qsgd_wire)."""
        hw = self.codec.wire_header_words(self.nseg)
        if self.op == "qsgd":
            return m[4 * hw:], m[:4 * hw].view(self.torch.float32)[:self.nseg]
        return m[hw:], m[:hw].view(self.torch.float32)[:self.nseg]

    def _fold_args(self):
        if not self.fold:
            return None
        return (self.hat, self.mem if self.fold_mem else None, self.weights[self.self_slot])

    def exchange(self):
        self.exchange_finish(self.exchange_start())

    def exchange_start(self):
        """Post the grouped sends/recvs; returns the works (None without peers)."""
        if not self.peers:
            return None
        import torch.distributed as dist
        if self.backend == "gloo":  # comm_device=cpu: pinned host staging (parallel_choco_v.py:271-272)
            self.msg_h.copy_(self.msg)
            src, dst = self.msg_h, self.recv_h
        else:
            src, dst = self.msg, self.recv
        ops = []
        for r in self.peers:
            ops.append(dist.P2POp(dist.isend, src, r))
            ops.append(dist.P2POp(dist.irecv, dst[r], r))
        return dist.batch_isend_irecv(ops)

    def exchange_finish(self, works):
        if works is None:
            return
        for w in works:
            w.wait()
        if self.backend == "gloo":
            for r in self.peers:
                self.recv[r].copy_(self.recv_h[r], non_blocking=True)

    def hat_self_update(self):
        """x_hat += own message (sparse codecs): it needs no remote message, so with peers
        it runs while the exchange is in flight (bit-identical: x_hat takes only the
        local message; memory's updates stay in neighbour order, parallel_choco_v.py:307-310)."""
        torch = self.torch
        self.codec.sparse_accumulate(self.msg[:self.k].view(torch.float32), self.msg[self.k:], self.hat, 1.0)

    def decompress(self, hat_done=False):
        c = self.codec
        torch = self.torch
        msgs = [self.msg if r == self.rank else self.recv[r] for r in self.ranks]
        if self.op in ("topk", "topk_seg", "randk", "randk_seg"):
            # the self message's memory update is skipped when the fold applied it; x_hat takes
            # it here unless the overlap (hat_done) or the fold did
            items = [(r, m, w) for r, m, w in zip(self.ranks, msgs, self.weights)
                     if not (r == self.rank and self.fold_mem)]
            want_hat = not (hat_done or self.fold)
            slot = next((i for i, (r, _, _) in enumerate(items) if r == self.rank), -1) if want_hat else -1
            c.sparse_accumulate_multi([(m[:self.k].view(torch.float32), m[self.k:]) for _, m, _ in items],
                                      [w for _, _, w in items], self.mem, self_slot=slot,
                                      xhat_self=self.hat if slot >= 0 else None)
        elif self.op == "qsgd":
            parts = [self._parts(m) for m in msgs]
            if self.defer:  # applied by the next step's first pass
                self.pending = (parts, list(self.weights), self.self_slot)
                return
            c.qsgd_accumulate(parts, self.weights, self.self_slot, self.n, self.param, self.mem, xhat_self=self.hat,
                              **self._seg())
        else:
            parts = [self._parts(m) for m in msgs]
            if self.defer:  # applied by the next step's pass
                self.pending = (parts, list(self.weights), self.self_slot)
                return
            c.sign_accumulate(parts, self.weights, self.self_slot, self.n, self.mem, xhat_self=self.hat,
                              **self._seg())

    def step(self):
        self.compress()
        works = self.exchange_start()
        overlap = works is not None and self.op in ("topk", "topk_seg", "randk", "randk_seg") and not self.fold
        if overlap:
            self.hat_self_update()
        self.exchange_finish(works)
        self.decompress(hat_done=overlap)

    def warm_counters(self):
        """Counters behind the warm-start hit rate (top-k): sample launches, K2 prologue
        samples, exact fallbacks / segment window misses, calls.  None for other codecs."""
        c = self.codec
        from chocosgd_amd import _lib
        if self.op == "topk":
            return {"calls": c.launch_count("topk_stream"), "k1_sample_launches": c.launch_count("topk_bounds"),
                    "k2_prologue_samples": c.topk_workspace_word(_lib.TOPK_K2_SAMPLES_OFFSET),
                    "exact_fallbacks": c.topk_workspace_word(_lib.TOPK_FALLBACKS_OFFSET)}
        if self.op == "topk_seg":
            return {"calls": c.launch_count("topk_seg_collect"), "s1_cold_passes": c.launch_count("topk_seg_hist"),
                    "segment_window_misses": c.topk_workspace_word(_lib.TOPK_FALLBACKS_OFFSET, plan=self.plan)}
        return None

    def warm_rates(self, before, steps):
        """Per-step rates of warm_counters() over the timed region, and the warm-call share."""
        if before is None:
            return None
        after = self.warm_counters()
        d = {k: after[k] - before[k] for k in after}
        calls = max(d["calls"], 1)
        if self.op == "topk":
            cold = d["k1_sample_launches"] + d["k2_prologue_samples"] + d["exact_fallbacks"]
            note = ("warm = took the previous call's window without a fallback; cold = a K1 sample launch, a K2 "
                    "prologue sample (cold run after a warm miss) or an exact fallback")
        else:
            cold = d["s1_cold_passes"]
            note = ("warm = one read against the segments' carried windows (W2); cold = the S1 + S2 sequence "
                    "(cold run after a window miss); segment_window_misses counts segments, not calls")
        r = {k + "_per_step": round(v / steps, 3) for k, v in d.items()}
        r["warm_call_share"] = round(max(0.0, 1.0 - cold / calls), 3)
        r["note"] = note
        return r

    def stage_bytes(self):
        """Algorithmic HBM bytes per step of each stage, and the
        notes that say how they are counted."""
        n, nm = self.n, len(self.ranks)
        if self.step_mode:
            comp, dec, note = self._codec_bytes(n, nm)
            # the consensus step reads x, memory, x_hat and writes x (16n) in place of the
            # 4n read of a resident delta: the compulsory bytes of the fused pass
            if self.defer:
                # the receive runs inside the next step's first pass: one stage whose compulsory
                # bytes are x, x_hat, memory read and written once (24n), every message read, and
                # this step's message written
                wire = comp - 4 * n
                return 24 * n + nm * (wire - 4) + wire, 0, (
                    "deferred receive: x, x_hat, memory read + written once (24n) + each received message + "
                    "this step's message (QSGD: the quantize pass's second read of x, x_hat is not counted)")
            return comp + 12 * n, dec, "consensus step + compress 16n + codec output; " + note
        return self._codec_bytes(n, nm)

    def _codec_bytes(self, n, nm):
        if self.op in ("topk", "topk_seg"):
            comp = 4 * n + 8 * self.k                    # read d once, write k (fp32 value, int32 index)
            dec = 8 * self.k * nm + 8 * self.k * (nm + 1)  # read each message; RMW mem per msg + x_hat (self)
            if self.fold:
                s = 1 if self.fold_mem else 0
                comp += 8 * self.k * (1 + s)            # the self message's RMW of x_hat (+ memory) in the emission
                dec = 8 * self.k * (nm - s) * 2           # the other messages: read + memory RMW
                return comp, dec, ("compress 4n + 8k + 8k RMW of x_hat (+ 8k of memory when the self rank is "
                                   "first: the fold); decompress 8k read + 8k memory RMW per other message")
            return comp, dec, "compress 4n + 8k; decompress 8k read per message + 8k RMW per touched buffer"
        if self.op in ("randk", "randk_seg"):
            comp = 4 * self.k + 8 * self.k                # gather k values + write k pairs (the sampler reads none)
            dec = 8 * self.k * nm + 8 * self.k * (nm + 1)
            return comp, dec, "compress 4k gather + 8k; decompress as top-k"
        if self.op == "qsgd":
            cw = 1
            while cw < self.param:
                cw <<= 1
            wire = n * cw // 8 + n // 8
            comp = 4 * n + wire + 4                       # read d, write level + sign planes + norm
            dec = nm * wire + 8 * n + 8 * n               # read each message, RMW memory and x_hat
            return comp, dec, "compress 4n + n(cw+1)/8 (the norm pass's second read of d is not counted); " \
                              "decompress wire per message + 8n RMW memory + 8n RMW x_hat"
        words = 4 * ((n + 31) // 32)
        return 4 * n + words + 4, nm * words + 16 * n, "compress 4n + n/8; decompress n/8 per message + 16n RMW"

    def granule_bytes_decompress(self):
        """Sparse accumulate at HBM access granularity: every touched 64-B segment of
        x_hat / memory is read and written whole (the bound a scattered RMW really pays)."""
        if self.op not in ("topk", "topk_seg", "randk", "randk_seg"):
            return None
        torch = self.torch
        ms = [self.msg] + [self.recv[r] for r in self.ranks if r != self.rank]
        own = int(torch.unique(self.msg[self.k:].long() // 16).numel())  # x_hat: the self message's lines
        segs = sum(int(torch.unique(m[self.k:].long() // 16).numel()) for m in ms)
        return 8 * self.k * len(self.ranks) + 128 * (segs + own)


def e2e_rate(w, reps=5):
    """Host-resident leg (north star: the path starts and ends in host memory):
    pinned H2D of the worker's buffer -> compress -> D2H of the packed message
    -> H2D of that message (the receiver's copy) -> decompress-accumulate.
    Reported next to, never as, the device-resident value."""
    import torch
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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cpus():
    """CPUs this process may actually use: the affinity mask, capped by a cgroup v2/v1
    CPU quota (a GPU box grants a 16-CPU share of a machine whose os.cpu_count() is far
    larger; oversubscribing that share only slows torch down)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts and parts[0] != "max":
                n = min(n, max(1, int(int(parts[0]) / int(parts[1]))))
            elif path.endswith("quota_us") and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    n = min(n, max(1, int(int(parts[0]) / int(f.read()))))
            break
        except (OSError, ValueError, IndexError):
            continue
    return n


def cpu_baseline(w):
    """Reference torch-CPU op sequence (oracle/torch_port.py) on the host cores: the
    process's usable CPUs (affinity and cgroup quota), one thread, and os.cpu_count()
    threads."""
    import torch
    from oracle import torch_port as P

    def make(m):
        if w.step_mode:  # the reference's step: consensus step, then compress x - x_hat
            x0, hat, mem = w.x[:m].cpu(), w.hat[:m].cpu(), w.mem[:m].cpu()
            codec_run = make_codec(m, hat, mem, None)

            def run():
                x = x0.clone()  # (the copy is outside the reference's work but cheap next to it)
                P.gossip_step(x, mem, hat, GAMMA)
                codec_run(x - hat)
            return run
        return make_codec(m, torch.zeros(m), torch.zeros(m), w.d[:m].cpu())

    def make_codec(m, hat, mem, d_fixed):
        def wrap(f):
            return (lambda: f(d_fixed)) if d_fixed is not None else f
        if w.op in ("topk", "topk_seg", "randk", "randk_seg"):
            if w.op in ("randk", "randk_seg"):
                return wrap(lambda d: P.sparse_decompress(hat, mem, *P.randk_compress(d, w.param), 1.0))
            return wrap(lambda d: P.sparse_decompress(hat, mem, *P.topk_compress(d, w.param), 1.0))
        if w.op == "qsgd":
            return wrap(lambda d: P.dense_decompress(hat, mem, P.qsgd_compress(d, 2 ** w.param - 1), 1.0))
        return wrap(lambda d: P.sign_decompress(hat, mem, *P.sign_compress(d), m, 1.0))

    what = {"topk": "top-k (torch.topk) compress + self decompress",
            "topk_seg": "top-k (torch.topk, flat) compress + self decompress",
            "randk": "random-k (np.random.choice) compress + self decompress",
            "randk_seg": "random-k (np.random.choice, flat) compress + self decompress",
            "qsgd": f"QSGD q={w.param} compress + self decompress",
            "sign": "sign + L1 norm compress + self decompress"}[w.op]
    if w.step_mode:
        what = "consensus step x += gamma (memory - x_hat) + " + what

    def timed(threads, m, reps, budget_s):
        torch.set_num_threads(threads)
        run = make(m)
        run()  # warm-up
        ts = []
        stop = time.perf_counter() + budget_s
        while len(ts) < reps and (not ts or time.perf_counter() < stop):
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        med = statistics.median(ts)
        return {"threads": threads, "n": m, "value": round(4 * m / med / 1e9, 4), "ms": round(med * 1e3, 1),
                "reps": len(ts)}

    usable = usable_cpus()
    big = min(w.n, 100_000_000)
    small = min(w.n, 25_000_000)
    rows = [timed(usable, big, 3, 20.0), timed(1, small, 2, 10.0)]
    if (os.cpu_count() or usable) != usable:
        rows.append(timed(os.cpu_count(), small, 2, 10.0))
    main = rows[0]
    return {"value": main["value"], "unit": "GB/s", "cores": usable, "kind": "port",
            "sample": f"first {big} elements of the delta, {what}; median of {main['reps']} after 1 warm-up, "
                      f"{main['ms']} ms each; rows: 1 thread and os.cpu_count() threads on {small} elements",
            "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(), "usable_cpus": usable, "rows": rows}


def _bench_device(torch, local):
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise SystemExit("bench.py: no GPU visible (the codec has no CPU path)")
    torch.cuda.set_device(local % ndev)
    return torch.device("cuda", local % ndev)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = None
    if world > 1:
        import datetime
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # bounded: a rank that never arrives (or dies) fails the others instead of hanging them
        tmo = datetime.timedelta(seconds=args.dist_timeout)
        if args.backend == "nccl":
            dev = _bench_device(torch, local)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, timeout=tmo)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=tmo)
        if args.die_before_exchange is not None:
            # launcher test (tests/test_bench_launcher.py): one rank aborts, the others block in
            # the first collective, as a rank killed before the exchange leaves them
            if rank == args.die_before_exchange:
                import signal
                os.kill(os.getpid(), signal.SIGABRT)
            dist.barrier()
            raise SystemExit("bench.py: --die-before-exchange: the barrier returned")
    if dev is None:
        dev = _bench_device(torch, local)
    from chocosgd_amd import _lib, codec
    if args.lib:
        _lib.load(args.lib)
    codec.lib()
    w = Worker(args, rank, world, dev)
    comp_k, dec_k = STAGES[w.op]
    if w.step_mode:
        comp_k = comp_k + ["gossip_step", "qsgd_recv_norm", "sign_recv_pack", "sign_planes"]

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def stage_times(steps):
        out = {}
        for name in comp_k + dec_k:
            t, c = codec.profile_read(name)
            if c:
                out[name] = (t / steps * 1e3, t / c * 1e3, c / steps)  # us per step, us per launch, launches/step
        return out

    burn = args.burn_in if args.burn_in is not None else (200 if (w.step_mode and w.grads is not None) else 0)
    for _ in range(burn):  # untimed: the steady state of a training run (step_* workloads)
        w.step()
    # warm-up; its last steps time every kernel to find the dominant stage
    codec.profile_reset()
    for i in range(args.warmup):
        codec.profile_enable(i >= args.warmup // 2)
        w.step()
    barrier()
    codec.profile_enable(False)
    nw = args.warmup - args.warmup // 2
    pre = stage_times(max(nw, 1))
    t_comp = sum(pre[k][0] for k in comp_k if k in pre)
    t_dec = sum(pre[k][0] for k in dec_k if k in pre)
    dom_name, dom_k = ("decompress", dec_k) if t_dec > t_comp else ("compress", comp_k)

    # timed region: only the dominant stage's longest kernel carries events (a
    # dispatch-attached event pair costs ~4 us of GPU time: three pairs on the top-k
    # compress made the step 176 -> 189 us, tools/host_overhead.py); the stage's other
    # kernels are timed in the untimed pass below
    dom_kernel = max((k for k in dom_k if k in pre), key=lambda k: pre[k][0], default=None)
    codec.profile_reset()
    codec.profile_filter([dom_kernel] if dom_kernel else dom_k)
    warm0 = w.warm_counters()  # (synchronises: before the timed region)
    codec.profile_enable(not args.no_kernel_events)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        w.step()
    barrier()
    elapsed = time.perf_counter() - t0
    codec.profile_enable(False)
    timed = stage_times(args.steps)
    # calls that took the exact fallback so far (top-k: the flat workspace's counter)
    fallbacks = codec.topk_fallback_count() if w.op == "topk" else None
    warm_start = w.warm_rates(warm0, args.steps)

    # untimed pass: every kernel, plus the exchange on its own events
    codec.profile_reset()
    codec.profile_filter(None)
    codec.profile_enable(True)
    npass = min(args.steps, 10)
    ex_ms = []
    if w.grads is not None:
        w.grad_events = []
    for _ in range(npass):
        w.compress()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        w.exchange()
        e1.record()
        w.decompress()
        ex_ms.append((e0, e1))
    barrier()
    codec.profile_enable(False)
    untimed = stage_times(npass)
    exchange_us = statistics.median(a.elapsed_time(b) * 1e3 for a, b in ex_ms) if w.peers else 0.0
    grad_us = None
    if w.grad_events:
        grad_us = statistics.median(a.elapsed_time(b) * 1e3 for a, b in w.grad_events)
        w.grad_events = None
    # top-k: the same compress with the warm start off (every call samples its window
    # in K1 / reads twice in the segmented path), beside the warm numbers above
    cold = None
    if w.op in ("topk", "topk_seg"):
        lib = codec.lib()
        lib.choco_topk_set_warm_start(0)
        codec.profile_reset()
        codec.profile_enable(True)
        for _ in range(npass):
            w.compress()
        barrier()
        codec.profile_enable(False)
        lib.choco_topk_set_warm_start(1)
        cold = stage_times(npass)
    granule = w.granule_bytes_decompress()

    t_max = elapsed
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    ms_per_step = t_max / args.steps * 1e3
    value = world * 4 * w.n * args.steps / t_max / 1e9
    if rank == 0:
        comp_b, dec_b, bytes_note = w.stage_bytes()

        def stage_entry(name, kernels, nbytes, src):
            us = sum(src[k][0] for k in kernels if k in src)
            if us <= 0:
                return None
            ach = nbytes / (us * 1e-6) / 1e9
            e = {"stage": name, "kernels": {k: {"us_per_launch": round(src[k][1], 2),
                                                "launches_per_step": round(src[k][2], 2)}
                                            for k in kernels if k in src},
                 "us_per_step": round(us, 2), "algorithmic_bytes": nbytes, "achieved": round(ach, 1),
                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}
            return e

        in_timed = {k: timed[k] for k in dom_k if k in timed}
        src_dom = {**untimed, **in_timed}  # the timed kernel's own numbers, the rest untimed
        src_comp = src_dom if dom_name == "compress" else untimed
        src_dec = src_dom if dom_name == "decompress" else untimed
        stages = [stage_entry("compress", comp_k, comp_b, src_comp), stage_entry("decompress", dec_k, dec_b, src_dec)]
        stages = [s for s in stages if s]
        if granule and len(stages) > 1:
            s = stages[-1]
            s["granule_bytes"] = granule
            s["granule_achieved"] = round(granule / (s["us_per_step"] * 1e-6) / 1e9, 1)
            s["granule_note"] = "every touched 64-B segment of x_hat / memory read + written whole, + messages"
            # what a scattered RMW really pays: HBM line transactions per second (a read and a
            # write-back per touched 64-B line).  Reported as a rate only: no ceiling is claimed
            # (a separate probe's best rate was beaten by this kernel in round 2).
            tx = (granule - 8 * w.k * len(w.ranks)) / 64
            s["line_tx_rate"] = round(tx / (s["us_per_step"] * 1e-6) / 1e9, 2)
            s["line_tx_unit"] = "G line-transactions/s"
        cold_entry = None
        if cold:
            ce = stage_entry("compress", comp_k, comp_b, cold)
            if ce:
                cold_entry = {"compress_us": ce["us_per_step"], "achieved": ce["achieved"], "frac": ce["frac"],
                              "kernels_us": {k: v["us_per_launch"] for k, v in ce["kernels"].items()},
                              "note": "warm start off (choco_topk_set_warm_start(0)): every call takes its window "
                                      "from the K1 sample / the segmented path reads twice; same data, untimed pass"}
        dom = next((s for s in stages if s["stage"] == dom_name), stages[0] if stages else None)
        traffic = None
        tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tf) and dom:
            with open(tf) as f:
                tab = json.load(f)
            ks = [f"{k}:{traffic_key(args)}:{w.n}" for k in dom["kernels"]]
            if all(k in tab for k in ks):
                traffic = int(sum(tab[k]["bytes"] for k in ks))
        roofline = None
        if dom:
            roofline = {"bound": "hbm", "achieved": dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": dom["frac"], "traffic": traffic, "stage": dom["stage"],
                        "kernels": sorted(dom["kernels"]), "kernel_us": dom["us_per_step"],
                        "algorithmic_bytes_per_launch": dom["algorithmic_bytes"],
                        "dominant_kernel": dom_kernel,
                        "timed_in": (f"{dom_kernel}: timed region (dispatch-attached events); the stage's other "
                                     f"kernels: untimed pass right after" if in_timed else "untimed pass")}
        # top-k: the measured floor of a single pass that is GIVEN the k-th key (tools/probe_floor.hip)
        if roofline and w.op == "topk" and not w.fold and not w.step_mode and dom and dom["stage"] == "compress":
            ff = os.path.join(ROOT, "profiles", "probe_floor.json")
            if os.path.exists(ff):
                with open(ff) as f:
                    fl = json.load(f).get(f"topk:{w.n}:{w.k}")
                if fl:
                    roofline["known_t_floor"] = {
                        "us": fl["known_t_floor_us"], "frac_of_peak": round(dom["algorithmic_bytes"] / (
                            fl["known_t_floor_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                        "compress_vs_floor": round(fl["known_t_floor_us"] / dom["us_per_step"], 4),
                        "source": fl["source"]}
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": w.label + ("_fold" if w.fold else ""), "n_per_worker": w.n, "k_per_worker": w.k,
                       "graph": ("ring3_loopback" if w.loop_sets else "self") if world == 1 else (
                           "complete" if world == 2 else "ring"),
                       "messages_per_step": len(w.ranks), "backend": args.backend if world > 1 else None,
                       "step": "compress+exchange+decompress-accumulate", "parallelism": f"gossip{world}"},
            "roofline": roofline,
            "stages": stages,
            "stage_bytes_note": bytes_note,
            "kernels_us": {k: round(v[1], 2) for k, v in untimed.items()},
            "exchange_us": round(exchange_us, 1),
            "topk_fallbacks": fallbacks,
            "warm_start": warm_start,
            "burn_in_steps": burn,
            "apply_gradient": None if grad_us is None else {
                "us": round(grad_us, 1), "lr": args.grad_lr, "scale": args.grad_scale,
                "note": "g ~ N(0, scale^2) drawn fresh each step, then x -= lr * g (optim/utils.py:13-47, no "
                        "momentum / weight decay): torch ops inside the timed step (ms_per_step includes them); not "
                        "part of the codec stages"},
            "cold_start": cold_entry,
            "e2e": None,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_e2e and not w.step_mode:
            out["e2e"] = e2e_rate(w)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(w)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
