"""The other consumers of the codec through their drop-ins:
DCD (chocosgd_amd/dcd.py, reference dcd_psgd.py:150-446), DeepSqueeze
(chocosgd_amd/deep_squeeze.py, reference deep_squeeze.py:133-489) and ECD
(chocosgd_amd/ecd.py, reference ecd_psgd.py:186-455), driven on the GPU with
capturing / replaying aggregators against the reference's own round trips
(tests/golden/gen_golden.py gen_dcd, gen_deepsqueeze, gen_ecd).

Top-k: bit-exact.  Sign: the device L1 norms are fp64 sums (the reference's fp32 CPU
norms drift ~1e-6), so results agree to 1e-5 and are bit-exact against the oracle fed
the device norms.  QSGD: the device draws its own uniforms, so every message is checked
against the oracle with the device's norms and uniforms, then the receiver bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import golden, same_bits
from oracle import choco_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED0 = 5000  # torch.manual_seed(SEED0 + rank) before each rank's compress


def drawn_seed(r):
    """The seed sparsification._draw_seed takes from torch's generator after manual_seed(SEED0 + r)."""
    torch.manual_seed(SEED0 + r)
    return int(torch.randint(0, 2**62, (1,)).item())


def randk_expected(d, lens, ratio, r):
    """(values, global indices) the device sampler draws for rank r (oracle restatement)."""
    return O.randk_segmented(np.asarray(d, dtype=np.float32), lens, ratio, drawn_seed(r), is_biased=True)


def wire(vals, idx):
    return np.concatenate([np.asarray(vals, dtype=np.float32).view(np.int32), np.asarray(idx).astype(np.int32)])


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    return t.cpu().numpy()


def _split(flat, lens):
    out, p = [], 0
    for m in lens:
        out.append(flat[p:p + m].clone())
        p += m
    return out


class _Capture:
    def __init__(self, rank):
        self.rank, self.sent = rank, []

    def _agg(self, data, op, force_wait=True):
        assert op == "get_raw_sync_data" and force_wait is True
        self.sent.append(data.clone())
        return {self.rank: data}


class _Replay:
    def __init__(self, per_call):
        self.per_call = list(per_call)

    def _agg(self, data, op, force_wait=True):
        return self.per_call.pop(0)


def _args(comm_op, **kw):
    return dict(aggregator=None, comm_op=comm_op, comm_device="gpu", compress_ratio=kw.get("ratio", 0.9),
                quantize_level=kw.get("q", 4), is_biased=False, backend="nccl", use_ipc=False)


# ------------------------------------------------------------------------------ DCD
def run_dcd(g, comm_op, **kw):
    from chocosgd_amd.dcd import DCDCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer
    lens = g["layout"].tolist()
    shapes = [(torch.Size([m]), m) for m in lens]
    s = int(g["self_rank"])
    sent, mine = [], None
    for r in range(3):
        comp = DCDCompressor(**_args(comm_op, **kw))
        sb = {"original_shapes": shapes, "flatten_half_params": TensorBuffer(_split(dev(g["half"][r]), lens)),
              "flatten_params": TensorBuffer(_split(dev(g["x"][r]), lens))}
        torch.manual_seed(SEED0 + r)  # the random-k sampler's seed (sparsification._draw_seed)
        comp.compress(sb)
        comp.compressor_fn.aggregator_fn = _Capture(r)
        comp.sync(sb)
        sent.append(comp.compressor_fn.aggregator_fn.sent)
        if r == s:
            mine = (comp, sb)
    comp, sb = mine
    nhp = {r: TensorBuffer(_split(dev(g["hats0"][r]), lens)) for r in range(3)}
    comp.compressor_fn.aggregator_fn = _Replay([{r: sent[r][c] for r in range(3)} for c in range(len(sent[0]))])
    comp.sync(sb)
    comp.uncompress(sb, nhp)
    return sb, nhp, sent


def test_dcd_topk_golden():
    g = golden("dcd_topk_mini_r09")
    sb, nhp, _ = run_dcd(g, "compress_top_k", ratio=0.9)
    for r in range(3):
        assert same_bits(host(nhp[r].buffer), g["hats1"][r]), f"replica {r}"
    assert sb["n_bits"] == float(g["n_bits"])


def test_dcd_sign_golden():
    g = golden("dcd_sign_mini")
    lens = g["layout"].tolist()
    sb, nhp, sent = run_dcd(g, "sign")
    hw = (len(lens) + 3) // 4 * 4
    for r in range(3):
        assert np.allclose(host(nhp[r].buffer), g["hats1"][r], rtol=1e-5, atol=1e-6)
        m = host(sent[r][0])
        hat = g["hats0"][r].copy()
        O.sign_axpy(hat, m[hw:], m[:hw].view(np.float32)[:len(lens)], lens, 1.0, two_roundings=False)
        assert same_bits(host(nhp[r].buffer), hat)
    assert sb["n_bits"] == float(g["n_bits"])


def _qsgd_decoded(msg, lens, q=4):
    n = sum(lens)
    hb = 4 * ((len(lens) + 3) // 4 * 4)
    norms = msg[:hb].view(np.float32)[:len(lens)]
    levels, neg = O.qsgd_unpack(msg[hb:], n, q)
    off, parts = 0, []
    for si, m in enumerate(lens):
        parts.append(O.qsgd_decode(levels[off:off + m], neg[off:off + m], norms[si], 2 ** q - 1, m))
        off += m
    return np.concatenate(parts)


def test_dcd_qsgd_consistent():
    g = golden("dcd_qsgd_mini_q4")
    lens = g["layout"].tolist()
    sb, nhp, sent = run_dcd(g, "quantize_qsgd", q=4)
    for r in range(3):
        dec = _qsgd_decoded(host(sent[r][0]), lens)
        assert same_bits(host(nhp[r].buffer), (g["hats0"][r] + dec).astype(np.float32))
        d = (g["half"][r] - g["x"][r]).astype(np.float64)
        assert np.corrcoef(dec, d)[0, 1] > 0.3  # an unbiased quantization of the delta
    assert sb["n_bits"] == float(g["n_bits"])


# ------------------------------------------------------------------------------ DeepSqueeze
def run_deepsqueeze(g, comm_op, **kw):
    from chocosgd_amd.deep_squeeze import DeepSqueezeCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer
    lens = g["layout"].tolist()
    shapes = [(torch.Size([m]), m) for m in lens]
    s = int(g["self_rank"])
    neighbors_info = {r: float(w) for r, w in enumerate(g["weights"])}
    sent, local, mine = [], [], None
    for r in range(3):
        comp = DeepSqueezeCompressor(rank=r, consensus_stepsize=float(g["gamma"]), **_args(comm_op, **kw))
        sb = {"original_shapes": shapes, "params_tb": TensorBuffer(_split(dev(g["mem"][r]), lens))}
        torch.manual_seed(SEED0 + r)
        local.append(host(comp.compress(sb).buffer))
        comp.compressor_fn.aggregator_fn = _Capture(r)
        comp.sync(sb)
        sent.append(comp.compressor_fn.aggregator_fn.sent)
        if r == s:
            mine = (comp, sb)
    comp, sb = mine
    comp.compressor_fn.aggregator_fn = _Replay([{r: sent[r][c] for r in range(3)} for c in range(len(sent[0]))])
    comp.sync(sb)
    agg = host(comp.uncompress(sb, neighbors_info).buffer)
    return sb, local, agg, sent


def test_deepsqueeze_topk_golden():
    g = golden("deepsqueeze_topk_mini_r09")
    sb, local, agg, _ = run_deepsqueeze(g, "compress_top_k", ratio=0.9)
    for r in range(3):
        assert same_bits(local[r], g["local"][r]), f"local {r}"
    assert same_bits(agg, g["agg"])
    assert sb["n_bits"] == float(g["n_bits"])


def test_deepsqueeze_sign_golden():
    g = golden("deepsqueeze_sign_mini")
    lens = g["layout"].tolist()
    s = int(g["self_rank"])
    sb, local, agg, sent = run_deepsqueeze(g, "sign")
    hw = (len(lens) + 3) // 4 * 4
    want = np.zeros_like(g["agg"])
    for r in range(3):
        m = host(sent[r][0])
        norms = m[:hw].view(np.float32)[:len(lens)]
        assert np.allclose(norms, g[f"norms{r}"], rtol=1e-5, atol=0)
        assert np.array_equal(m[hw:], O.sign_pack(g["mem"][r]))
        assert same_bits(local[r], O.sign_local(g["mem"][r], norms, lens))  # sign(0) = 0 kept
        assert np.allclose(local[r], g["local"][r], rtol=1e-5, atol=1e-7)
        c = O.deepsqueeze_weight(float(g["gamma"]), float(g["weights"][r]), r == s)
        O.sign_axpy(want, m[hw:], norms, lens, c, two_roundings=True)
    assert same_bits(agg, want)
    # the aggregate sums terms of both signs (c_self < 0): absolute tolerance at the terms' scale
    assert np.allclose(agg, g["agg"], rtol=1e-5, atol=1e-6)


def test_deepsqueeze_qsgd_consistent():
    g = golden("deepsqueeze_qsgd_mini_q4")
    lens = g["layout"].tolist()
    s = int(g["self_rank"])
    sb, local, agg, sent = run_deepsqueeze(g, "quantize_qsgd", q=4)
    want = np.zeros_like(g["agg"])
    for r in range(3):
        dec = _qsgd_decoded(host(sent[r][0]), lens)
        assert same_bits(local[r], dec)  # the local copy is the decoded message
        c = O.deepsqueeze_weight(float(g["gamma"]), float(g["weights"][r]), r == s)
        want = (want + (c * dec).astype(np.float32)).astype(np.float32)
    assert same_bits(agg, want)
    assert sb["n_bits"] == float(g["n_bits"])


# ------------------------------------------------------------------------------ ECD
def run_ecd(g, comm_op, **kw):
    from chocosgd_amd.ecd import ECDCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer
    lens = g["layout"].tolist()
    shapes = [(torch.Size([m]), m) for m in lens]
    s = int(g["self_rank"])
    sent, mine = [], None
    for r in range(3):
        comp = ECDCompressor(**_args(comm_op, **kw))
        sb = {"original_shapes": shapes, "flatten_updated_params": TensorBuffer(_split(dev(g["z"][r]), lens))}
        torch.manual_seed(SEED0 + r)
        comp.compress(sb)
        comp.compressor_fn.aggregator_fn = _Capture(r)
        comp.sync(sb)
        sent.append(comp.compressor_fn.aggregator_fn.sent)
        if r == s:
            mine = (comp, sb)
    comp, sb = mine
    nhp = {r: TensorBuffer(_split(dev(g["hats0"][r]), lens)) for r in range(3)}
    comp.compressor_fn.aggregator_fn = _Replay([{r: sent[r][c] for r in range(3)} for c in range(len(sent[0]))])
    comp.sync(sb)
    comp.uncompress(sb, nhp, int(g["local_index"]))
    return sb, nhp, sent


def test_ecd_topk_golden():
    g = golden("ecd_topk_mini_r09")
    sb, nhp, _ = run_ecd(g, "compress_top_k", ratio=0.9)
    for r in range(3):
        assert same_bits(host(nhp[r].buffer), g["hats1"][r]), f"replica {r}"
    assert sb["n_bits"] == float(g["n_bits"])


def test_ecd_sign_golden():
    g = golden("ecd_sign_mini")
    lens = g["layout"].tolist()
    t = int(g["local_index"])
    sb, nhp, sent = run_ecd(g, "sign")
    hw = (len(lens) + 3) // 4 * 4
    for r in range(3):
        m = host(sent[r][0])
        want = O.ecd_sign_extrapolate(g["hats0"][r], m[hw:], m[:hw].view(np.float32)[:len(lens)], lens, t)
        assert same_bits(host(nhp[r].buffer), want)
        assert np.allclose(host(nhp[r].buffer), g["hats1"][r], rtol=1e-5, atol=1e-6)


def test_ecd_qsgd_consistent():
    g = golden("ecd_qsgd_mini_q4")
    lens = g["layout"].tolist()
    t = int(g["local_index"])
    sb, nhp, sent = run_ecd(g, "quantize_qsgd", q=4)
    for r in range(3):
        dec = _qsgd_decoded(host(sent[r][0]), lens)
        assert same_bits(host(nhp[r].buffer), O.ecd_extrapolate(g["hats0"][r], dec, t))
    assert sb["n_bits"] == float(g["n_bits"])


# ------------------------------------------------------------------------------ EF-sign, DGC
class _Gather:
    """all-gather stand-in: every rank's message, in rank order, per call."""

    def __init__(self, per_call):
        self.per_call = list(per_call)

    def _agg(self, data, op=None, communication_scheme="all_gather", **kw):
        return self.per_call.pop(0)


def test_ef_sign_golden():
    from chocosgd_amd.ef_sign import EFSignCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer
    g = golden("efsign_mini")
    lens = g["layout"].tolist()
    me = int(g["rank"])
    hw = (len(lens) + 3) // 4 * 4
    msgs, bufs = [], []
    for r in range(3):
        comp = EFSignCompressor(rank=r, world_size=3, aggregator=None, comm_op="sign", comm_device="gpu",
                                use_ipc=False)
        sb = comp.compress(TensorBuffer(_split(dev(g["grads"][r]), lens)))
        bufs.append((comp, sb))
        norms = sb["grad_norms_tb"].buffer
        header = torch.zeros(hw, dtype=torch.float32, device=DEV)
        header[:len(lens)] = norms
        msgs.append(torch.cat([header.view(torch.int32), sb["signs"]]))
    comp, sb = bufs[me]
    nm_me = host(sb["grad_norms_tb"].buffer)
    assert np.allclose(nm_me, g["norms"][me], rtol=1e-5, atol=0)
    local = host(sb["synced_grads_tb"].buffer)
    assert same_bits(local, O.sign_local(g["grads"][me], nm_me, lens))
    comp.aggregator_fn = _Gather([msgs])
    comp.sync(sb)
    out = host(comp.decompress(sb).buffer)
    want = local.copy()
    for r in range(3):
        if r != me:
            m = host(msgs[r])
            O.sign_axpy(want, m[hw:], m[:hw].view(np.float32)[:len(lens)], lens, 1.0, two_roundings=False)
    assert same_bits(out, (want / np.float32(3.0)).astype(np.float32))
    assert np.allclose(out, g["out"], rtol=1e-5, atol=1e-6)
    assert sb["n_bits"] == float(g["n_bits"])


def test_dgc_topk():
    """strict_reference=False: the intended memory update (selected entries zeroed, what `~`
    on a ByteTensor gave in PyTorch <= 1.1); the selection and the recovered parameters
    bit-exact against the reference's fixture."""
    from chocosgd_amd.dgc import DGCCodec
    from chocosgd_amd.tensor_buffer import TensorBuffer
    g = golden("dgc_topk_mini_r09")
    lens = g["layout"].tolist()
    me = int(g["rank"])
    ratio = float(g["ratio"])
    msgs, mine = [], None
    for r in range(3):
        codec_r = DGCCodec(world_aggregator=None, comm_op="compress_top_k", comm_device="gpu", n_nodes=3,
                           strict_reference=False)
        mem = TensorBuffer(_split(dev(g["mems"][r]), lens))
        grads = _split(dev(g["grads"][r]), lens)
        vals, idx, n_bits = codec_r.compress(grads, mem, ratio)
        x = (g["grads"][r] + g["mems"][r]).astype(np.float32)
        ov, oi, _ = O.topk_segmented(x, lens, ratio)
        assert np.array_equal(host(idx).astype(np.int64), oi) and same_bits(host(vals), ov)
        x[oi] = 0.0
        assert same_bits(host(mem.buffer), x)
        msgs.append(torch.cat([vals.view(torch.int32), idx]))
        if r == me:
            mine = (codec_r, vals, idx, n_bits)
    codec_r, vals, idx, n_bits = mine
    assert n_bits == float(g["n_bits"])
    codec_r.world_aggregator = _Gather([msgs])
    synced, size = codec_r.sync(vals, idx)
    out = codec_r.recover_info(dev(g["params"]), synced, size, float(g["lr"]))
    assert same_bits(host(out), g["params_after"])


# ------------------------------------------------------------------------------ random-k consumers
def test_dcd_random_k():
    """DCDSparsificationCompressor with random_k (dcd_psgd.py:150-275): each rank's message is
    the device sampler's draw (oracle restatement of the seeded hash, seed from torch's
    generator) of half - x, and every replica gets hat[idx] += v."""
    g = golden("dcd_topk_mini_r09")
    lens = g["layout"].tolist()
    sb, nhp, sent = run_dcd(g, "compress_random_k", ratio=0.9)
    for r in range(3):
        ov, oi = randk_expected((g["half"][r] - g["x"][r]).astype(np.float32), lens, 0.9, r)
        assert np.array_equal(host(sent[r][0]), wire(ov, oi)), f"message {r}"
        want = g["hats0"][r].copy()
        want[oi] = (want[oi] + ov).astype(np.float32)
        assert same_bits(host(nhp[r].buffer), want), f"replica {r}"


def test_ecd_random_k():
    """ECDSparsificationCompressor with random_k (ecd_psgd.py:211-303): messages of z, every
    replica extrapolated hat[idx] = fmaf(2/t, v, hat[idx] * (1 - 2/t))."""
    g = golden("ecd_topk_mini_r09")
    lens = g["layout"].tolist()
    t = int(g["local_index"])
    a, b = O.ecd_coeffs(t)
    sb, nhp, sent = run_ecd(g, "compress_random_k", ratio=0.9)
    for r in range(3):
        ov, oi = randk_expected(g["z"][r], lens, 0.9, r)
        assert np.array_equal(host(sent[r][0]), wire(ov, oi)), f"message {r}"
        want = g["hats0"][r].copy()
        want[oi] = O.fma32(b, ov, (want[oi] * a).astype(np.float32))
        assert same_bits(host(nhp[r].buffer), want), f"replica {r}"


def test_deepsqueeze_random_k():
    """DeepSqueezeSparsificationCompressor with random_k (deep_squeeze.py:158-279): the local
    copy holds the drawn values, the aggregate sums c_r * v in neighbour order."""
    g = golden("deepsqueeze_topk_mini_r09")
    lens = g["layout"].tolist()
    s = int(g["self_rank"])
    sb, local, agg, sent = run_deepsqueeze(g, "compress_random_k", ratio=0.9)
    want = np.zeros_like(g["agg"])
    for r in range(3):
        ov, oi = randk_expected(g["mem"][r], lens, 0.9, r)
        assert np.array_equal(host(sent[r][0]), wire(ov, oi)), f"message {r}"
        loc = np.zeros_like(g["mem"][r])
        loc[oi] = ov
        assert same_bits(local[r], loc)
        c = O.deepsqueeze_weight(float(g["gamma"]), float(g["weights"][r]), r == s)
        want[oi] = (want[oi] + (c * ov).astype(np.float32)).astype(np.float32)
    assert same_bits(agg, want)


# ------------------------------------------------------------------------------ DGC: strict / intended / quantize
def test_dgc_topk_strict_reference_memory():
    """strict_reference=True (the default): memory <- _grad * nmask with the reference's
    nmask = (~mask.byte()).float() = 255 / 254 (dgc.py:174-176, sparsification.py:33-38),
    bit-exact against the reference's own fixture; get_mask agrees."""
    from chocosgd_amd.dgc import DGCCodec
    from chocosgd_amd.sparsification import SparsificationCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer
    g = golden("dgc_topk_mini_r09")
    lens = g["layout"].tolist()
    ratio = float(g["ratio"])
    for r in range(3):
        c = DGCCodec(world_aggregator=None, comm_op="compress_top_k", comm_device="gpu", n_nodes=3)
        assert c.strict_reference
        mem = TensorBuffer(_split(dev(g["mems"][r]), lens))
        vals, idx, _ = c.compress(_split(dev(g["grads"][r]), lens), mem, ratio)
        assert same_bits(host(mem.buffer), g["mems_after"][r])
        x = dev((g["grads"][r] + g["mems"][r]).astype(np.float32))
        _, nmask = SparsificationCompressor().get_mask(x, idx.long())
        assert same_bits(host(x * nmask), g["mems_after"][r])


@pytest.mark.parametrize("q", [32, 4])
def test_dgc_quantize_multistep(q):
    """DGC's quantize branch (dgc.py:183-185, 336-340) over three steps: the memory is left
    alone (the reference's `pass`), the message is QSGD of grad + memory (q = 32: the floats
    themselves), and recover_info applies params - lr * sum / n_nodes."""
    from chocosgd_amd.dgc import DGCCodec
    from chocosgd_amd.tensor_buffer import TensorBuffer
    g = golden("dgc_topk_mini_r09")
    lens = g["layout"].tolist()
    n = sum(lens)
    c = DGCCodec(world_aggregator=None, comm_op="quantize_qsgd", comm_device="gpu", n_nodes=3, quantize_level=q)
    mem0 = g["mems"][0]
    mem = TensorBuffer(_split(dev(mem0), lens))
    params = g["params"].copy()
    for step in range(3):
        grads = (g["grads"][step] * np.float32(0.5 + step)).astype(np.float32)
        seed = drawn_seed(step)
        torch.manual_seed(SEED0 + step)
        dense, idx, n_bits = c.compress(_split(dev(grads), lens), mem, None)
        assert idx is None
        assert same_bits(host(mem.buffer), mem0), "memory must keep its value"
        x = (grads + mem0).astype(np.float32)
        if q == 32:
            want = x
        else:
            s = 2 ** q - 1
            u = O.qsgd_uniforms(n, seed, 0)
            off, parts = 0, []
            for si, m in enumerate(lens):
                nd = np.float32(np.sqrt(np.sum(x[off:off + m].astype(np.float64) ** 2)))
                parts.append(O.qsgd_dense(x[off:off + m], s, u[off:off + m], nd))
                off += m
            want = np.concatenate(parts)
        assert same_bits(host(dense), want)
        others = [dense, dense * 2, dense * 3]
        summed = others[0] + others[1] + others[2]
        c.world_aggregator = _Gather([summed])
        synced, size = c.sync(dense, None)
        out = c.recover_info(dev(params), synced, size, 0.1)
        upd = (host(summed) / np.float32(3)).astype(np.float32)
        params_next = O.fma32(np.float32(-0.1), upd, params)
        assert same_bits(host(out), params_next)
        params = params_next
