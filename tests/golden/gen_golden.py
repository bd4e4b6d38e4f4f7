"""Golden-vector generator for the CHOCO compressor path.

Runs ONLY in the authoring container, where the upstream reference is mounted
read-only at /root/reference.  It imports the reference's own compressor code
(`dl_code/pcode/utils/sparsification.py`, `dl_code/pcode/optim/parallel_choco_v.py`,
`dl_code/pcode/optim/utils.py`, `dl_code/pcode/utils/tensor_buffer.py`) and
records inputs + outputs as small .npz fixtures next to this script.  Nothing
from the reference is copied: the fixtures are data only.

`bit2byte` (the reference's unvendored C++/CUDA packing extension,
tvogels/signSGD-with-Majority-Vote, unpinned commit) is not available, so a stub
implementing this repo's documented convention (row r of the (32, N') view ->
bit r of word j, LSB first; bit set <=> value == -1; unpack writes v = 2*bit so
the reference's `1 - v` decode yields -1/+1) is injected.  Sign fixtures
therefore pin the wrapper semantics (sign, pad-to-32, (32, N') split, decode
rule, per-tensor L1 norms, accumulate), while the bit position inside a word
is this repo's convention ("parity unpinned" at that one boundary).

Usage:  python tests/golden/gen_golden.py [generator ...]   (no argument: all)
"""
import importlib
import json
import os
import sys
import types

sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference

import numpy as np  # noqa: E402
import torch  # noqa: E402

REF = "/root/reference/dl_code"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# bit2byte stub (this repo's convention; see module docstring)
# --------------------------------------------------------------------------
def _stub_packing(src):
    # src: int32 [32, N'] with values in {-1, 0, 1}
    src = src.view(32, -1)
    bits = (src == -1).to(torch.int64)
    shifts = torch.arange(32, dtype=torch.int64).view(32, 1)
    words = (bits << shifts).sum(dim=0)  # < 2**32
    words = torch.where(words >= 2**31, words - 2**32, words)
    return words.to(torch.int32)


def _stub_unpacking(src, dst):
    w = src.to(torch.int64) & 0xFFFFFFFF
    shifts = torch.arange(32, dtype=torch.int64).view(32, 1)
    bits = (w.view(1, -1) >> shifts) & 1
    dst.copy_((2 * bits).to(dst.dtype).view_as(dst))
    return dst


b2b = types.ModuleType("bit2byte")
b2b.packing = _stub_packing
b2b.unpacking = _stub_unpacking
sys.modules["bit2byte"] = b2b
sys.path.insert(0, REF)

import pcode.utils.sparsification as ref_sp  # noqa: E402
import pcode.optim.parallel_choco_v as ref_pcv  # noqa: E402
import pcode.optim.utils as ref_ou  # noqa: E402
from pcode.utils.tensor_buffer import TensorBuffer  # noqa: E402


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {name}.npz ({os.path.getsize(path)} B)")


def randn(n, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, generator=g) * scale).float()


# --------------------------------------------------------------------------
# k rule (sparsification.py:22,45) -- double rounding table
# --------------------------------------------------------------------------
def gen_k_table():
    rows = []
    for n in [1, 2, 7, 10, 50, 99, 100, 640, 1000, 4096, 65536, 272474, 1000003,
              25_000_000, 100_000_000, 345_000_000, 2**24 + 5]:
        for ratio in [0.0, 0.5, 0.9, 0.95, 0.99, 0.999, 0.9999]:
            x = torch.zeros(1)  # shape irrelevant: replicate the exact expression
            k = max(1, int(n * (1 - ratio)))
            rows.append([n, ratio, k])
    # cross-check the expression against the reference function on real tensors
    c = ref_sp.SparsificationCompressor()
    for n, ratio in [(640, 0.9), (1000, 0.9), (50, 0.99), (4096, 0.99)]:
        v, i = c.get_top_k(torch.arange(n, dtype=torch.float32), ratio)
        assert len(i) == max(1, int(n * (1 - ratio)))
    with open(os.path.join(OUT, "k_table.json"), "w") as f:
        json.dump(rows, f)
    print("wrote k_table.json")


# --------------------------------------------------------------------------
# top-k  (sparsification.py:18-31)
# --------------------------------------------------------------------------
def gen_topk():
    c = ref_sp.SparsificationCompressor()
    cases = []
    # (name, x, xhat_or_None, ratio)
    cases.append(("topk_n1000_r09", randn(1000, 11), None, 0.9))
    cases.append(("topk_n65536_r099", randn(65536, 12), randn(65536, 13, 0.5), 0.99))
    cases.append(("topk_n262144_r099", randn(262144, 14), None, 0.99))
    cases.append(("topk_n30011_r09", randn(30011, 15), randn(30011, 16), 0.9))
    cases.append(("topk_n50_k1", randn(50, 17), None, 0.99))
    # k==1 tie on the max magnitude: torch.max returns the first index
    t = torch.tensor([0.5, -3.0, 1.0, 3.0, -3.0, 2.0], dtype=torch.float32)
    cases.append(("topk_k1_tie", t, None, 0.9))
    # ties at the k-th magnitude (round(randn*8)/8): set semantics only
    g = torch.Generator().manual_seed(3)
    tq = (torch.round(torch.randn(4096, generator=g) * 8) / 8).float()
    cases.append(("topk_ties_n4096_r09", tq, None, 0.9))
    for name, x, xhat, ratio in cases:
        d = x - xhat if xhat is not None else x
        vals, idx = c.get_top_k(d, ratio)
        extra = {} if xhat is None else {"xhat": xhat.numpy()}
        save(name, x=x.numpy(), ratio=np.float64(ratio), values=vals.numpy(),
             indices=idx.numpy().astype(np.int64),
             k=np.int64(max(1, int(d.numel() * (1 - ratio)))), **extra)


# --------------------------------------------------------------------------
# random-k (sparsification.py:40-54): gather-given-indices is bit-exact
# --------------------------------------------------------------------------
def gen_randk():
    c = ref_sp.SparsificationCompressor()
    x = randn(20000, 21)
    np.random.seed(5)
    vals_b, idx_b = c.get_random_k(x, 0.95)  # as compress() calls it: biased
    np.random.seed(6)
    vals_u, idx_u = c.get_random_k(x, 0.95, is_biased=False)
    save("randk_n20000_r095", x=x.numpy(), ratio=np.float64(0.95),
         idx_biased=idx_b.numpy(), vals_biased=vals_b.numpy(),
         idx_unbiased=idx_u.numpy(), vals_unbiased=vals_u.numpy())


# --------------------------------------------------------------------------
# QSGD (sparsification.py:87-98,114-123); rand_like captured
# --------------------------------------------------------------------------
class RandCapture:
    def __init__(self):
        self.draws = []
        self._orig = torch.rand_like

    def __enter__(self):
        def rl(*a, **k):
            r = self._orig(*a, **k)
            self.draws.append(r.clone())
            return r
        torch.rand_like = rl
        return self

    def __exit__(self, *exc):
        torch.rand_like = self._orig


def gen_qsgd():
    qc = ref_sp.QuantizationCompressor()
    for name, n, q, biased, seed, scale in [
        ("qsgd_n32771_q4", 32771, 4, False, 31, 1.0),
        ("qsgd_n32771_q4_biased", 32771, 4, True, 32, 1.0),
        ("qsgd_n4099_q2", 4099, 2, False, 33, 1.0),
        ("qsgd_n4099_q8", 4099, 8, False, 34, 1.0),
        ("qsgd_n257_q4_small", 257, 4, False, 35, 1.0),
    ]:
        x = randn(n, seed, scale)
        torch.manual_seed(1000 + seed)
        with RandCapture() as cap:
            out = qc.compress(x, "quantize_qsgd", q, biased)
        assert len(cap.draws) == 1
        norm = x.norm(p=2)
        save(name, x=x.numpy(), u=cap.draws[0].numpy(), norm_ref=norm.numpy(),
             norm_f64=np.float64(np.sqrt(np.sum(x.numpy().astype(np.float64) ** 2))),
             out=out.numpy(), q=np.int64(q), biased=np.int64(biased))
    # all-zero tensor -> NaN (0/0 at sparsification.py:88-89)
    x = torch.zeros(64)
    torch.manual_seed(7)
    with RandCapture() as cap:
        out = qc.compress(x, "quantize_qsgd", 4, False)
    save("qsgd_zeros", x=x.numpy(), u=cap.draws[0].numpy(), out=out.numpy())
    # quantize_level == 32 -> passthrough
    x = randn(100, 36)
    out = qc.compress(x, "quantize_qsgd", 32, False)
    save("qsgd_q32_passthrough", x=x.numpy(), out=out.numpy())


# --------------------------------------------------------------------------
# sign pack / unpack (sparsification.py:129-163) with the stubbed bit2byte
# --------------------------------------------------------------------------
def gen_sign():
    sc = ref_sp.SignCompressor()
    for name, n, seed in [("sign_n4096", 4096, 41), ("sign_n40003_pad", 40003, 42),
                          ("sign_n31", 31, 43)]:
        x = randn(n, seed)
        if n == 4096:  # exact zeros and -0.0 encode as "positive"
            x[::97] = 0.0
            x[1::89] = -0.0
        packed, size = sc.compress(x)
        dec = sc.uncompress(packed, size)
        save(name, x=x.numpy(), packed=packed.numpy(), decoded=dec.numpy())


# --------------------------------------------------------------------------
# CHOCO round trips (parallel_choco_v.py:229-558, optim/utils.py:67-72)
# --------------------------------------------------------------------------
MINI_LAYOUT = [432, 16, 16, 2304, 16, 16, 2304, 16, 16, 4608, 32, 32, 9216,
               32, 32, 512, 32, 32, 640, 10, 1, 3]


class CaptureAgg:
    def __init__(self):
        self.sent = []

    def _agg(self, data, op, force_wait=False):
        assert op == "get_raw_sync_data" and force_wait is False
        self.sent.append(data.clone())
        return [], {}

    def complete_wait(self, reqs):
        pass


class ReplayAgg:
    def __init__(self, per_call):
        self.per_call = list(per_call)

    def _agg(self, data, op, force_wait=False):
        return [], self.per_call.pop(0)

    def complete_wait(self, reqs):
        pass


def make_comp(cls, comm_op, ratio=0.9, qlevel=4, biased=False):
    comp = object.__new__(cls)  # skip the torch.cuda stream in __init__
    comp.aggregator_fn = None
    comp.comm_op = comm_op
    comp.comm_device = "gpu"
    comp.compress_ratio = ratio
    comp.quantize_level = qlevel
    comp.is_biased = biased
    comp.backend = "nccl"
    comp.use_ipc = False
    comp.kargs = {}
    comp.compressor_fn = {
        ref_pcv.CHOCOSparsificationCompressor: ref_sp.SparsificationCompressor,
        ref_pcv.CHOCOQuantizationCompressor: ref_sp.QuantizationCompressor,
        ref_pcv.CHOCOSignCompressor: ref_sp.SignCompressor,
    }[cls]()
    return comp


def split(flat, layout):
    out, p = [], 0
    for m in layout:
        out.append(flat[p:p + m].clone())
        p += m
    return out


def gen_choco(kind, name, layout, comm_op, **kw):
    cls = {"topk": ref_pcv.CHOCOSparsificationCompressor,
           "qsgd": ref_pcv.CHOCOQuantizationCompressor,
           "sign": ref_pcv.CHOCOSignCompressor}[kind]
    n = sum(layout)
    shapes = [(torch.Size([m]), m) for m in layout]
    W = 3  # ring of 3: every worker sees {0,1,2} with weight 1/3
    self_rank = 1
    neighbors_info = {0: 1.0 / 3, 1: 1.0 / 3, 2: 1.0 / 3}
    xs = [randn(n, 500 + 10 * r) for r in range(W)]
    xhats = [xs[r] + randn(n, 501 + 10 * r, 0.1) for r in range(W)]
    sent, sbs, draws = [], [], []
    for r in range(W):
        comp = make_comp(cls, comm_op, **kw)
        sb = {"original_shapes": shapes,
              "flatten_params": TensorBuffer(split(xs[r], layout)),
              "flatten_hat_params": TensorBuffer(split(xhats[r], layout))}
        torch.manual_seed(900 + r)
        with RandCapture() as cap:
            comp.compress(sb)
        draws.append(torch.cat(cap.draws) if cap.draws else torch.zeros(0))
        comp.aggregator_fn = CaptureAgg()
        comp.sync(sb)
        sent.append(comp.aggregator_fn.sent)
        sbs.append((comp, sb))
    # receiver = worker 1, with non-trivial initial x_hat_i and memory
    comp, sb = sbs[self_rank]
    hat0 = randn(n, 777, 0.3)
    mem0 = randn(n, 778, 0.3)
    nhp = {self_rank: TensorBuffer(split(hat0, layout)),
           "memory": TensorBuffer(split(mem0, layout))}
    ncalls = len(sent[0])
    comp.aggregator_fn = ReplayAgg([{r: sent[r][c] for r in range(W)} for c in range(ncalls)])
    comp.sync(sb)
    comp.uncompress(sb, nhp, neighbors_info)
    hat1 = nhp[self_rank].buffer.clone()
    mem1 = nhp["memory"].buffer.clone()
    # consensus step x += gamma (memory - x_hat)   (optim/utils.py:67-72)
    fp = TensorBuffer(split(xs[self_rank], layout))
    ref_ou.update_params_from_neighbor(nhp, fp, 0.9, self_rank)
    arrays = dict(layout=np.array(layout, dtype=np.int64),
                  x=np.stack([x.numpy() for x in xs]),
                  xhat=np.stack([x.numpy() for x in xhats]),
                  hat0=hat0.numpy(), mem0=mem0.numpy(), hat1=hat1.numpy(), mem1=mem1.numpy(),
                  x_after_gossip=fp.buffer.numpy(), gamma=np.float64(0.9),
                  weights=np.array([neighbors_info[r] for r in range(W)]),
                  self_rank=np.int64(self_rank), n_bits=np.float64(sb["n_bits"]))
    if kind == "topk":
        arrays["selected_shapes"] = np.array(sb["selected_shapes"], dtype=np.int64)
        for r in range(W):
            arrays[f"msg{r}"] = sent[r][0].numpy()
    if kind == "qsgd":
        arrays["u"] = np.stack([d.numpy() for d in draws])
        arrays["norms_ref"] = np.stack(
            [np.array([s.norm(p=2).item() for s in split(xs[r] - xhats[r], layout)],
                      dtype=np.float32) for r in range(W)])
        for r in range(W):
            arrays[f"msg{r}"] = sent[r][0].numpy()
    if kind == "sign":
        for r in range(W):
            arrays[f"norms{r}"] = sent[r][0].numpy()
            arrays[f"signs{r}"] = sent[r][1].numpy()
    save(name, **arrays)


def gen_choco_step(kind, name, layout, comm_op, **kw):
    """ParallelCHOCO_V.step after apply_gradient (parallel_choco_v.py:116-155) for a ring
    of 3: every worker r runs update_params_from_neighbor (optim/utils.py:67-72) on its
    own x_r, x_hat_r, memory_r, then compress + sync; worker 1 replays the three
    messages through uncompress.  Pins the fused gossip + compress entry points."""
    cls = {"topk": ref_pcv.CHOCOSparsificationCompressor,
           "sign": ref_pcv.CHOCOSignCompressor}[kind]
    n = sum(layout)
    shapes = [(torch.Size([m]), m) for m in layout]
    W, self_rank, gamma = 3, 1, 0.9
    neighbors_info = {0: 1.0 / 3, 1: 1.0 / 3, 2: 1.0 / 3}
    xs = [randn(n, 1500 + 10 * r) for r in range(W)]
    hats = [xs[r] + randn(n, 1501 + 10 * r, 0.1) for r in range(W)]
    mems = [hats[r] + randn(n, 1502 + 10 * r, 0.05) for r in range(W)]
    sent, sbs, x_after = [], [], []
    for r in range(W):
        comp = make_comp(cls, comm_op, **kw)
        nhp = {r: TensorBuffer(split(hats[r], layout)), "memory": TensorBuffer(split(mems[r], layout))}
        fp = TensorBuffer(split(xs[r], layout))
        ref_ou.update_params_from_neighbor(nhp, fp, gamma, r)
        x_after.append(fp.buffer.clone())
        sb = {"original_shapes": shapes, "flatten_params": fp,
              "flatten_hat_params": TensorBuffer(split(hats[r], layout))}
        comp.compress(sb)
        comp.aggregator_fn = CaptureAgg()
        comp.sync(sb)
        sent.append(comp.aggregator_fn.sent)
        sbs.append((comp, sb, nhp))
    comp, sb, nhp = sbs[self_rank]
    ncalls = len(sent[0])
    comp.aggregator_fn = ReplayAgg([{r: sent[r][c] for r in range(W)} for c in range(ncalls)])
    comp.sync(sb)
    comp.uncompress(sb, nhp, neighbors_info)
    save(name, layout=np.array(layout, dtype=np.int64), gamma=np.float64(gamma),
         x=np.stack([x.numpy() for x in xs]), xhat=np.stack([h.numpy() for h in hats]),
         mem=np.stack([m.numpy() for m in mems]), x_after_gossip=np.stack([x.numpy() for x in x_after]),
         hat1=nhp[self_rank].buffer.numpy(), mem1=nhp["memory"].buffer.numpy(),
         weights=np.array([neighbors_info[r] for r in range(W)]), self_rank=np.int64(self_rank),
         n_bits=np.float64(sb["n_bits"]))


def gen_gossip():
    x, mem, hat = randn(10007, 61), randn(10007, 62), randn(10007, 63)
    fp = TensorBuffer([x.clone()])
    nhp = {0: TensorBuffer([hat.clone()]), "memory": TensorBuffer([mem.clone()])}
    ref_ou.update_params_from_neighbor(nhp, fp, 0.9, 0)
    save("gossip_n10007", x=x.numpy(), mem=mem.numpy(), hat=hat.numpy(),
         gamma=np.float64(0.9), out=fp.buffer.numpy())


def gen_layouts():
    """Per-tensor segmentation of the reference's own models (create_optimizer.py:15-24)."""
    import importlib
    rn = importlib.import_module("pcode.models.resnet")
    rn = sys.modules["pcode.models.resnet"]
    res = {}
    for nm, ds, size in [("resnet20_cifar10", "cifar10", 20)]:
        m = rn.ResNet_cifar(dataset=ds, resnet_size=size)
        res[nm] = [p.nelement() for _, p in m.named_parameters()]
    m = rn.ResNet_imagenet(dataset="imagenet", resnet_size=50)
    res["resnet50_imagenet"] = [p.nelement() for _, p in m.named_parameters()]
    with open(os.path.join(OUT, "layouts.json"), "w") as f:
        json.dump(res, f)
    print("wrote layouts.json", {k: (len(v), sum(v)) for k, v in res.items()})


def _consumer(cls, comm_op, ratio=0.9, qlevel=4, biased=False, **extra):
    """A reference DCD / DeepSqueeze compressor (its __init__ only stores arguments)."""
    return cls(aggregator=None, comm_op=comm_op, comm_device="gpu", compress_ratio=ratio,
               quantize_level=qlevel, is_biased=biased, backend="nccl", use_ipc=False, **extra)


class SyncCapture:
    """force_wait=True aggregator: returns {rank: data}; records what was sent."""

    def __init__(self, rank):
        self.rank, self.sent = rank, []

    def _agg(self, data, op, force_wait=True):
        assert op == "get_raw_sync_data" and force_wait is True
        self.sent.append(data.clone())
        return {self.rank: data}


class SyncReplay:
    def __init__(self, per_call):
        self.per_call = list(per_call)

    def _agg(self, data, op, force_wait=True):
        return self.per_call.pop(0)


def gen_dcd(kind, name, layout, comm_op, **kw):
    """DCD_PSGD's compressor (dcd_psgd.py:150-446) for a ring of 3: worker r compresses
    d = half_r - x_r; worker 1 replays the three messages into its replicas of every
    neighbour's model (neighbor_hat_params, one per rank)."""
    import pcode.optim.dcd_psgd as ref_dcd
    cls = {"topk": ref_dcd.DCDSparsificationCompressor, "qsgd": ref_dcd.DCDQuantizationCompressor,
           "sign": ref_dcd.DCDSignCompressor}[kind]
    n = sum(layout)
    shapes = [(torch.Size([m]), m) for m in layout]
    W, self_rank = 3, 1
    xs = [randn(n, 2500 + 10 * r) for r in range(W)]
    halfs = [xs[r] + randn(n, 2501 + 10 * r, 0.1) for r in range(W)]
    sent, draws, last = [], [], None
    for r in range(W):
        comp = _consumer(cls, comm_op, **kw)
        sb = {"original_shapes": shapes, "flatten_half_params": TensorBuffer(split(halfs[r], layout)),
              "flatten_params": TensorBuffer(split(xs[r], layout))}
        torch.manual_seed(2900 + r)
        with RandCapture() as cap:
            comp.compress(sb)
        draws.append(torch.cat(cap.draws) if cap.draws else torch.zeros(0))
        comp.aggregator_fn = SyncCapture(r)
        comp.sync(sb)
        sent.append(comp.aggregator_fn.sent)
        if r == self_rank:
            last = (comp, sb)
    comp, sb = last
    hats0 = [randn(n, 2600 + r, 0.5) for r in range(W)]
    nhp = {r: TensorBuffer(split(hats0[r], layout)) for r in range(W)}
    comp.aggregator_fn = SyncReplay([{r: sent[r][c] for r in range(W)} for c in range(len(sent[0]))])
    comp.sync(sb)
    comp.uncompress(sb, nhp)
    arrays = dict(layout=np.array(layout, dtype=np.int64), x=np.stack([x.numpy() for x in xs]),
                  half=np.stack([h.numpy() for h in halfs]), hats0=np.stack([h.numpy() for h in hats0]),
                  hats1=np.stack([nhp[r].buffer.numpy() for r in range(W)]), self_rank=np.int64(self_rank),
                  n_bits=np.float64(sb["n_bits"]))
    if kind == "qsgd":
        arrays["u"] = np.stack([d.numpy() for d in draws])
        for r in range(W):
            arrays[f"msg{r}"] = sent[r][0].numpy()
    save(name, **arrays)


def gen_deepsqueeze(kind, name, layout, comm_op, **kw):
    """DeepSqueeze's compressor (deep_squeeze.py:133-489) for a ring of 3: worker r
    compresses its error-compensated memory_r and returns the local compressed copy;
    worker 1 aggregates consensus_stepsize * (w_r - [r == 1]) * decode(msg_r)."""
    import pcode.optim.deep_squeeze as ref_ds
    cls = {"topk": ref_ds.DeepSqueezeSparsificationCompressor, "qsgd": ref_ds.DeepSqueezeQuantizationCompressor,
           "sign": ref_ds.DeepSqueezeSignCompressor}[kind]
    n = sum(layout)
    shapes = [(torch.Size([m]), m) for m in layout]
    W, self_rank, gamma = 3, 1, 0.5
    neighbors_info = {0: 1.0 / 3, 1: 1.0 / 3, 2: 1.0 / 3}
    mems = [randn(n, 3500 + 10 * r) for r in range(W)]
    if kind == "sign":
        for m in mems:
            m[::101] = 0.0  # torch.sign(0) = 0 in the local copy, "+" on the wire
    sent, draws, local, last = [], [], [], None
    for r in range(W):
        comp = _consumer(cls, comm_op, rank=r, consensus_stepsize=gamma, **kw)
        sb = {"original_shapes": shapes, "params_tb": TensorBuffer(split(mems[r], layout))}
        torch.manual_seed(3900 + r)
        with RandCapture() as cap:
            lc = comp.compress(sb)
        draws.append(torch.cat(cap.draws) if cap.draws else torch.zeros(0))
        local.append(lc.buffer.clone())
        comp.aggregator_fn = SyncCapture(r)
        comp.sync(sb)
        sent.append(comp.aggregator_fn.sent)
        if r == self_rank:
            last = (comp, sb)
    comp, sb = last
    comp.aggregator_fn = SyncReplay([{r: sent[r][c] for r in range(W)} for c in range(len(sent[0]))])
    comp.sync(sb)
    agg = comp.uncompress(sb, neighbors_info)
    arrays = dict(layout=np.array(layout, dtype=np.int64), mem=np.stack([m.numpy() for m in mems]),
                  local=np.stack([m.numpy() for m in local]), agg=agg.buffer.numpy(), gamma=np.float64(gamma),
                  weights=np.array([neighbors_info[r] for r in range(W)]), self_rank=np.int64(self_rank),
                  n_bits=np.float64(sb["n_bits"]))
    if kind == "qsgd":
        arrays["u"] = np.stack([d.numpy() for d in draws])
        for r in range(W):
            arrays[f"msg{r}"] = sent[r][0].numpy()
    if kind == "sign":
        for r in range(W):
            arrays[f"norms{r}"] = sent[r][0].numpy()
    save(name, **arrays)


def gen_ecd(kind, name, layout, comm_op, local_index=5, **kw):
    """ECD_PSGD's compressor (ecd_psgd.py:186-455) for a ring of 3: worker r compresses
    its extrapolated model z_r; worker 1 extrapolates its replica of every neighbour,
    hat <- (1 - 2/t) hat + (2/t) q, t = local_index."""
    import pcode.optim.ecd_psgd as ref_ecd
    cls = {"topk": ref_ecd.ECDSparsificationCompressor, "qsgd": ref_ecd.ECDQuantizationCompressor,
           "sign": ref_ecd.ECDSignCompressor}[kind]
    n = sum(layout)
    shapes = [(torch.Size([m]), m) for m in layout]
    W, self_rank = 3, 1
    zs = [randn(n, 4500 + 10 * r) for r in range(W)]
    sent, draws, last = [], [], None
    for r in range(W):
        comp = _consumer(cls, comm_op, **kw)
        sb = {"original_shapes": shapes, "flatten_updated_params": TensorBuffer(split(zs[r], layout))}
        torch.manual_seed(4900 + r)
        with RandCapture() as cap:
            comp.compress(sb)
        draws.append(torch.cat(cap.draws) if cap.draws else torch.zeros(0))
        comp.aggregator_fn = SyncCapture(r)
        comp.sync(sb)
        sent.append(comp.aggregator_fn.sent)
        if r == self_rank:
            last = (comp, sb)
    comp, sb = last
    hats0 = [randn(n, 4600 + r, 0.5) for r in range(W)]
    nhp = {r: TensorBuffer(split(hats0[r], layout)) for r in range(W)}
    comp.aggregator_fn = SyncReplay([{r: sent[r][c] for r in range(W)} for c in range(len(sent[0]))])
    comp.sync(sb)
    comp.uncompress(sb, nhp, local_index)
    arrays = dict(layout=np.array(layout, dtype=np.int64), z=np.stack([z.numpy() for z in zs]),
                  hats0=np.stack([h.numpy() for h in hats0]),
                  hats1=np.stack([nhp[r].buffer.numpy() for r in range(W)]), local_index=np.int64(local_index),
                  self_rank=np.int64(self_rank), n_bits=np.float64(sb["n_bits"]))
    if kind == "qsgd":
        arrays["u"] = np.stack([d.numpy() for d in draws])
        for r in range(W):
            arrays[f"msg{r}"] = sent[r][0].numpy()
    if kind == "sign":
        for r in range(W):
            arrays[f"norms{r}"] = sent[r][0].numpy()
    save(name, **arrays)


class GatherCapture:
    """centralized all-gather aggregator over W simulated ranks: returns the list of
    every rank's data (filled in from the recorded messages)."""

    def __init__(self, msgs):
        self.msgs = msgs  # per call: list over ranks

    def _agg(self, data, op=None, communication_scheme="all_gather", **kw):
        return self.msgs.pop(0)


def gen_ef_sign(name, layout):
    """EFSignCompressor (ef_sign_sgd.py:126-219) for 3 ranks: rank 1 decompresses."""
    import pcode.optim.ef_sign_sgd as ref_ef
    W, me = 3, 1
    n = sum(layout)
    grads = [randn(n, 5500 + r) for r in range(W)]
    grads[0][::97] = 0.0
    bufs, sent = [], []
    for r in range(W):
        comp = ref_ef.EFSignCompressor(rank=r, world_size=W, aggregator=None, comm_op="sign", comm_device="gpu",
                                       use_ipc=False)
        sb = comp.compress(TensorBuffer(split(grads[r], layout)))
        bufs.append((comp, sb))
        sent.append((sb["grad_norms_tb"].buffer.clone(), sb["signs"].clone()))
    comp, sb = bufs[me]
    local = sb["synced_grads_tb"].buffer.clone()
    comp.aggregator_fn = GatherCapture([[s[0] for s in sent], [s[1] for s in sent]])
    comp.sync(sb)
    out = comp.decompress(sb)
    save(name, layout=np.array(layout, dtype=np.int64), grads=np.stack([g.numpy() for g in grads]),
         local=local.numpy(), out=out.buffer.numpy(), norms=np.stack([s[0].numpy() for s in sent]),
         rank=np.int64(me), n_bits=np.float64(sb["n_bits"]))


def gen_dgc(name, layout, ratio=0.9):
    """DGC._compress / _sync / _recover_info (dgc.py:153-252) with top-k, 3 ranks."""
    import pcode.optim.dgc as ref_dgc
    W, me, lr = 3, 1, 0.1
    n = sum(layout)
    names = [f"p{i}" for i in range(len(layout))]
    grads = [randn(n, 6500 + r) for r in range(W)]
    mems = [randn(n, 6600 + r, 0.3) for r in range(W)]
    msgs, outs = [], {}
    for r in range(W):
        opt = object.__new__(ref_dgc.DGC)
        opt.param_names = list(enumerate(names))
        opt.memory_of_grads = {nm: m.clone() for nm, m in zip(names, split(mems[r], layout))}
        opt._get_compress_ratio = lambda: ratio
        opt.comm_op = "compress_top_k"
        opt.compressor_fn = ref_sp.SparsificationCompressor()
        opt.quantize_level = 32
        opt.is_biased = False
        opt.is_compress_op = True
        opt.mask_momentum = False
        opt.comm_device = "gpu"
        vals, idx, n_bits = opt._compress(split(grads[r], layout))
        msgs.append(torch.cat([vals, idx]))
        outs[r] = (opt, vals, idx, n_bits, torch.cat([opt.memory_of_grads[nm] for nm in names]))
    opt, vals, idx, n_bits, mem_after = outs[me]
    opt.world_aggregator = GatherCapture([list(msgs)])
    synced, size = opt._sync(vals, idx)
    opt.n_nodes = W
    opt.param_groups = [{"lr": lr}]
    params = randn(n, 6700, 1.0)
    shapes = [(torch.Size([m]), m) for m in layout]
    upd = opt._recover_info(params, synced, size, opt.selected_shapes, shapes)
    save(name, layout=np.array(layout, dtype=np.int64), grads=np.stack([g.numpy() for g in grads]),
         mems=np.stack([m.numpy() for m in mems]),
         mems_after=np.stack([outs[r][4].numpy() for r in range(W)]), params=params.numpy(),
         params_after=upd.numpy(), lr=np.float64(lr), ratio=np.float64(ratio), rank=np.int64(me),
         n_bits=np.float64(n_bits))


def gen_consumers():
    gen_dcd("topk", "dcd_topk_mini_r09", MINI_LAYOUT, "compress_top_k", ratio=0.9)
    gen_dcd("qsgd", "dcd_qsgd_mini_q4", MINI_LAYOUT, "quantize_qsgd", qlevel=4)
    gen_dcd("sign", "dcd_sign_mini", MINI_LAYOUT, "sign")
    gen_deepsqueeze("topk", "deepsqueeze_topk_mini_r09", MINI_LAYOUT, "compress_top_k", ratio=0.9)
    gen_deepsqueeze("qsgd", "deepsqueeze_qsgd_mini_q4", MINI_LAYOUT, "quantize_qsgd", qlevel=4)
    gen_deepsqueeze("sign", "deepsqueeze_sign_mini", MINI_LAYOUT, "sign")
    gen_ecd_all()
    gen_central()


def gen_central():
    gen_ef_sign("efsign_mini", MINI_LAYOUT)
    gen_dgc("dgc_topk_mini_r09", MINI_LAYOUT)


def gen_ecd_all():
    gen_ecd("topk", "ecd_topk_mini_r09", MINI_LAYOUT, "compress_top_k", ratio=0.9)
    gen_ecd("qsgd", "ecd_qsgd_mini_q4", MINI_LAYOUT, "quantize_qsgd", qlevel=4)
    gen_ecd("sign", "ecd_sign_mini", MINI_LAYOUT, "sign")


def ref_neighborhood(world, rank):
    """neighbors_info as the reference's graphs give it: RingGraph for world > 2
    (topology.py:186-202 mixing matrix, :295-299 get_neighborhood), CompleteGraph for
    world 2 (topology.py:127,156-162); the constructors' process-group setup is skipped."""
    topo = importlib.import_module("pcode.utils.topology")
    if world == 2:
        g = object.__new__(topo.CompleteGraph)
        g._mixing_matrix = np.ones((world, world)) / world
    else:
        g = object.__new__(topo.RingGraph)
        g._mixing_matrix, g._rho = g._compute_mixing_matrix_and_rho(world)
    g._rank = rank
    return {int(r): float(w) for r, w in g.get_neighborhood().items()}


def gen_ring():
    """A ring of 8 CHOCO workers through the reference (parallel_choco_v.py:229-332 top-k,
    :476-558 sign): every worker compresses, then every worker uncompresses the messages of
    ITS neighbourhood only (a strict subset of the world from rank 0's {0, 1, 7} on), so the
    fixture pins the per-rank neighbour selection and order of a ring larger than 3.
    Inputs come from tests/_ring.py (seeded); only the outputs are stored."""
    sys.path.insert(0, os.path.dirname(OUT))
    import _ring as R
    nbs = {str(w): [[[r, wt] for r, wt in ref_neighborhood(w, q).items()] for q in range(w)]
           for w in range(2, 9)}
    with open(os.path.join(OUT, "ring_neighborhoods.json"), "w") as f:
        json.dump(nbs, f)
    print("wrote ring_neighborhoods.json")
    W, lens = R.RING_WORLD, R.RING_LAYOUT
    shapes = [(torch.Size([m]), m) for m in lens]
    ins = [R.ring_inputs(r) for r in range(W)]
    for kind, name, cls, op in (("topk", "choco_ring8_topk_r09", ref_pcv.CHOCOSparsificationCompressor,
                                 "compress_top_k"),
                                ("sign", "choco_ring8_sign", ref_pcv.CHOCOSignCompressor, "sign")):
        sent, sbs = [], []
        for r in range(W):
            x, xh, _, _ = (torch.from_numpy(a) for a in ins[r])
            comp = make_comp(cls, op, ratio=R.RING_RATIO)
            sb = {"original_shapes": shapes, "flatten_params": TensorBuffer(split(x, lens)),
                  "flatten_hat_params": TensorBuffer(split(xh, lens))}
            comp.compress(sb)
            comp.aggregator_fn = CaptureAgg()
            comp.sync(sb)
            sent.append(comp.aggregator_fn.sent)
            sbs.append((comp, sb))
        hat1, mem1 = [], []
        for r in range(W):
            nb = ref_neighborhood(W, r)
            comp, sb = sbs[r]
            nhp = {r: TensorBuffer(split(torch.from_numpy(ins[r][2]), lens)),
                   "memory": TensorBuffer(split(torch.from_numpy(ins[r][3]), lens))}
            comp.aggregator_fn = ReplayAgg([{q: sent[q][c] for q in nb} for c in range(len(sent[0]))])
            comp.sync(sb)
            comp.uncompress(sb, nhp, nb)
            hat1.append(nhp[r].buffer.numpy().copy())
            mem1.append(nhp["memory"].buffer.numpy().copy())
        extra = {}
        if kind == "sign":  # the reference's fp32 CPU L1 norms (SURVEY 0.4d drift), per worker
            extra["norms"] = np.stack([sent[r][0].numpy() for r in range(W)])
        save(name, layout=np.array(lens, dtype=np.int64), hat1=np.stack(hat1), mem1=np.stack(mem1), **extra)


STEP_LAYOUT = MINI_LAYOUT + [1029, 3]


def gen_choco_steps():
    gen_choco_step("topk", "choco_step_topk_r099", STEP_LAYOUT, "compress_top_k", ratio=0.99)
    gen_choco_step("sign", "choco_step_sign", STEP_LAYOUT, "sign")


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if len(sys.argv) > 1:  # only the named generators, e.g. gen_choco_steps
        for nm in sys.argv[1:]:
            globals()[nm]()
        sys.exit(0)
    gen_k_table()
    gen_topk()
    gen_randk()
    gen_qsgd()
    gen_sign()
    gen_choco("topk", "choco_topk_mini_r09", MINI_LAYOUT, "compress_top_k", ratio=0.9)
    gen_choco("topk", "choco_topk_mini_r099", MINI_LAYOUT, "compress_top_k", ratio=0.99)
    gen_choco("qsgd", "choco_qsgd_mini_q4", MINI_LAYOUT, "quantize_qsgd", qlevel=4)
    gen_choco("sign", "choco_sign_mini", MINI_LAYOUT, "sign")
    gen_gossip()
    gen_choco_steps()
    gen_consumers()
    gen_layouts()
