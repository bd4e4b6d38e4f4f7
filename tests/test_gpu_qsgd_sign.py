"""GPU parity: QSGD, sign(+norm), gossip step through the C ABI vs the oracle and the
reference's golden vectors.  Run on an MI355X with `pytest -m gpu`."""
import numpy as np
import pytest
import torch

from conftest import golden, golden_json, same_bits
from oracle import choco_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    return t.cpu().numpy()


def randn(n, seed, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(n, generator=g, device=DEV) * scale


def seg_table(lens):
    return dev(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)) if len(lens) > 1 else None


# ------------------------------------------------------------------------------------ QSGD
QCASES = [("qsgd_n32771_q4", 4, False), ("qsgd_n32771_q4_biased", 4, True), ("qsgd_n4099_q2", 2, False),
          ("qsgd_n4099_q8", 8, False), ("qsgd_n257_q4_small", 4, False)]


@pytest.mark.parametrize("name,q,biased", QCASES)
def test_qsgd_golden_pinned(name, q, biased):
    """Given the reference's uniforms and norm: dense output bit-exact, wire bit-exact vs
    the oracle packer, decode(wire) == reference output."""
    from chocosgd_amd import codec
    g = golden(name)
    x = dev(g["x"])
    norm = dev(np.array([g["norm_ref"]], dtype=np.float32))
    packed, norms, dense = codec.qsgd_compress(x, q, is_biased=biased, norm_in=norm, u_in=dev(g["u"]),
                                               want_dense=True)
    assert same_bits(host(dense), g["out"])
    s = 2 ** q - 1
    lvl = O.qsgd_levels(g["x"], s, g["u"], g["norm_ref"])
    assert np.array_equal(host(packed), O.qsgd_pack(lvl, g["x"], q))
    dec = codec.qsgd_decode(packed, norm, x.numel(), q, is_biased=biased)
    assert same_bits(host(dec), g["out"])


@pytest.mark.parametrize("n", [257, 100003, 4_000_001, 100_000_000])
def test_qsgd_device_norm_vs_fp64(n):
    from chocosgd_amd import codec
    x = randn(n, 7)
    _, norms, _ = codec.qsgd_compress(x, 4, seed=1)
    exact = float(np.sqrt(np.sum(host(x).astype(np.float64) ** 2)))
    assert abs(float(host(norms)[0]) - exact) <= 1e-6 * exact


@pytest.mark.parametrize("q", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("n", [1000, 262147])
def test_qsgd_device_rng_matches_oracle(q, n):
    from chocosgd_amd import codec
    x = randn(n, 100 + q)
    seed, offset = 0x1234_5678_9ABC, 77
    packed, norms, dense = codec.qsgd_compress(x, q, seed=seed, offset=offset, want_dense=True)
    u = O.qsgd_uniforms(n, seed, offset)
    s = 2 ** q - 1
    nrm = host(norms)[0]
    assert same_bits(host(dense), O.qsgd_dense(host(x), s, u, nrm))
    assert np.array_equal(host(packed), O.qsgd_pack(O.qsgd_levels(host(x), s, u, nrm), host(x), q))


def test_qsgd_looping_quantize_and_ranges():
    """The looping quantize kernel (single-segment buffers without x_hat: 1024 resident
    workgroups walk the tiles backward with a one-tile prefetch) at a size where every
    workgroup takes more than one tile plus a partial tail, whole-buffer and as chunked
    ranges (range starts aligned to 8192, the last range ending in the partial tile):
    bit-exact against the oracle."""
    from chocosgd_amd import codec
    n = 8192 * 1100 + 333
    q, seed, offset = 4, 0x2468_ACE0, 3
    x = randn(n, 515)
    packed, norms, dense = codec.qsgd_compress(x, q, seed=seed, offset=offset, want_dense=True)
    u = O.qsgd_uniforms(n, seed, offset)
    s = 2 ** q - 1
    nrm = host(norms)[0]
    lvl = O.qsgd_levels(host(x), s, u, nrm)
    assert same_bits(host(dense), O.qsgd_dense(host(x), s, u, nrm))
    assert np.array_equal(host(packed), O.qsgd_pack(lvl, host(x), q))
    for e0, e1 in codec.qsgd_chunks(n, 3):
        part = torch.empty(codec.qsgd_packed_bytes(e1 - e0, q), dtype=torch.uint8, device=DEV)
        codec.qsgd_quantize_range(x, q, norms, e0, e1, part, seed=seed, offset=offset)
        assert np.array_equal(host(part), O.qsgd_pack(lvl[e0:e1], host(x)[e0:e1], q)), (e0, e1)


def test_qsgd_quantize_many_units_per_wave():
    """A size where every resident wave of the ring quantize (CHOCO_QQ_RING builds: loads
    through LDS, waits counted by hand) walks ~8 units, so its steady-state waits run, with
    and without the dense output (4 or 8 stores per unit in the count): the whole wire
    and the dense values bit-exact against the oracle.  (Default builds: the one-tile
    kernel at a 3000-tile size.)"""
    from chocosgd_amd import codec
    n = 8192 * 3000 + 333
    q, seed, offset = 4, 0x1357_9BDF, 11
    x = randn(n, 516)
    packed_d, norms, dense = codec.qsgd_compress(x, q, seed=seed, offset=offset, want_dense=True)
    packed, norms2, _ = codec.qsgd_compress(x, q, seed=seed, offset=offset)
    u = O.qsgd_uniforms(n, seed, offset)
    s = 2 ** q - 1
    nrm = host(norms)[0]
    assert host(norms2)[0] == nrm
    xh = host(x)
    lvl = O.qsgd_levels(xh, s, u, nrm)
    want = O.qsgd_pack(lvl, xh, q)
    assert np.array_equal(host(packed), want)
    assert np.array_equal(host(packed_d), want)
    assert same_bits(host(dense), O.qsgd_dense(xh, s, u, nrm))


def test_qsgd_zero_segment_nan():
    from chocosgd_amd import codec
    x = torch.zeros(64, device=DEV)
    packed, norms, dense = codec.qsgd_compress(x, 4, seed=3, want_dense=True)
    assert host(norms)[0] == 0 and np.all(np.isnan(host(dense)))
    assert np.all(np.isnan(host(codec.qsgd_decode(packed, norms, 64, 4))))


def test_choco_qsgd_round_trip_golden():
    """Per-tensor QSGD of 3 workers (reference uniforms + norms pinned) -> fused accumulate."""
    from chocosgd_amd import codec
    g = golden("choco_qsgd_mini_q4")
    lens = g["layout"].tolist()
    so = seg_table(lens)
    msgs = []
    for r in range(3):
        packed, _, dense = codec.qsgd_compress(dev(g["x"][r]), 4, xhat=dev(g["xhat"][r]), seg_off=so,
                                               nseg=len(lens), norm_in=dev(g["norms_ref"][r]),
                                               u_in=dev(g["u"][r]), want_dense=True)
        assert same_bits(host(dense), g[f"msg{r}"])
        msgs.append((packed, dev(g["norms_ref"][r])))
    hat, mem = dev(g["hat0"]), dev(g["mem0"])
    codec.qsgd_accumulate(msgs, g["weights"].tolist(), int(g["self_rank"]), sum(lens), 4, mem, xhat_self=hat,
                          seg_off=so, nseg=len(lens))
    assert same_bits(host(hat), g["hat1"])
    assert same_bits(host(mem), g["mem1"])


@pytest.mark.parametrize("layout,biased", [("resnet20_cifar10", False), ("resnet50_imagenet", False),
                                           ("tiny", False), ("tiny", True), ("many", False)])
def test_qsgd_segmented_layout_norms_and_levels(layout, biased):
    """Per-tensor QSGD against the oracle: norms, levels (dense output) and the decode.  "tiny":
    300 tensors of 1-13 elements between larger ones, so that 8-element groups and 8192-element
    tiles straddle boundaries (the quantize's per-group and per-element segment parameters);
    biased: the per-tensor scale too."""
    from chocosgd_amd import codec
    if layout == "tiny":
        lens = [20_000] + [1 + (i * 7) % 13 for i in range(300)] + [9_000, 3, 70_001]
    elif layout == "many":  # more tensors than the kernels' LDS tables hold (their global fallbacks)
        lens = np.random.default_rng(5).integers(1, 40, size=1500).tolist() + [50_000]
    else:
        lens = golden_json("layouts.json")[layout]
    n = sum(lens)
    x, xh = randn(n, 21), randn(n, 22, 0.3)
    so = seg_table(lens)
    packed, norms, dense = codec.qsgd_compress(x, 4, is_biased=biased, xhat=xh, seg_off=so, nseg=len(lens), seed=9,
                                               offset=1, want_dense=True)
    d = host(x) - host(xh)
    ref = O.l2_norms(d, lens)
    assert np.allclose(host(norms), ref, rtol=1e-6, atol=0)
    u = O.qsgd_uniforms(n, 9, 1)
    off, outs = 0, []
    for s, m in enumerate(lens):
        outs.append(O.qsgd_dense(d[off:off + m], 15, u[off:off + m], host(norms)[s], is_biased=biased))
        off += m
    assert same_bits(host(dense), np.concatenate(outs))
    dec = codec.qsgd_decode(packed, norms, n, 4, is_biased=biased, seg_off=so, nseg=len(lens))
    levels, neg = O.qsgd_unpack(host(packed), n, 4)  # the oracle's decode of the wire itself
    off, want = 0, []
    for s, m in enumerate(lens):
        want.append(O.qsgd_decode(levels[off:off + m], neg[off:off + m], host(norms)[s], 15, m, is_biased=biased))
        off += m
    assert same_bits(host(dec), np.concatenate(want))
    assert same_bits(host(dense), np.concatenate(want))


# ------------------------------------------------------------------------------------ sign
@pytest.mark.parametrize("name", ["sign_n4096", "sign_n40003_pad", "sign_n31"])
def test_sign_golden(name):
    from chocosgd_amd import codec
    g = golden(name)
    packed, _ = codec.sign_compress(dev(g["x"]), want_norms=False)
    assert np.array_equal(host(packed), g["packed"])
    out = codec.sign_unpack(packed, g["x"].size)
    assert same_bits(host(out), g["decoded"])


@pytest.mark.parametrize("n", [1, 5, 32, 33, 127, 1000, 4096 * 32 + 3, 1_000_000, 1_000_007, 10_781_250 * 4 + 1])
def test_sign_random_sizes(n):
    from chocosgd_amd import codec
    x = randn(n, n % 1009)
    xh = randn(n, 5, 0.5)
    packed, norms = codec.sign_compress(x, xhat=xh)
    d = host(x) - host(xh)
    assert np.array_equal(host(packed), O.sign_pack(d))
    assert host(norms)[0] == O.l1_norms(d, [n])[0] or np.isclose(host(norms)[0], O.l1_norms(d, [n])[0],
                                                                  rtol=1e-7)
    assert same_bits(host(codec.sign_unpack(packed, n)), O.sign_unpack(O.sign_pack(d), n))


@pytest.mark.parametrize("layout", ["resnet20_cifar10", "resnet50_imagenet", "tiny_segments"])
def test_sign_segmented_norms(layout):
    from chocosgd_amd import codec
    if layout == "tiny_segments":
        rng = np.random.default_rng(0)
        lens = rng.integers(1, 40, size=3000).tolist()
    else:
        lens = golden_json("layouts.json")[layout]
    n = sum(lens)
    x = randn(n, 31)
    packed, norms = codec.sign_compress(x, seg_off=seg_table(lens), nseg=len(lens))
    assert np.array_equal(host(packed), O.sign_pack(host(x)))
    assert np.allclose(host(norms), O.l1_norms(host(x), lens), rtol=1e-7, atol=0)


@pytest.mark.parametrize("layout", ["one_segment", "resnet20_cifar10", "tiny_segments"])
@pytest.mark.parametrize("chunks", [2, 3, 7])
@pytest.mark.parametrize("fused", [False, True])
def test_sign_compress_ranges(layout, chunks, fused):
    """The chunked pack (choco_sign_compress_range, exchange_chunks): words bit-exact and
    norms as the oracle's, x_new (fused consensus step) bit-identical to the whole-buffer
    call; the finishing range leaves the accumulators clear for the next message."""
    from chocosgd_amd import codec
    if layout == "one_segment":
        lens = [1_000_007]
    elif layout == "tiny_segments":
        lens = np.random.default_rng(1).integers(1, 3000, size=700).tolist()
    else:
        lens = golden_json("layouts.json")[layout]
    n, nseg, so = sum(lens), len(lens), seg_table(lens)
    x, xh, mem = randn(n, 41), randn(n, 42, 0.5), randn(n, 43)
    gamma = 0.37
    x_whole = x.clone()
    if fused:
        codec.gossip_step(x_whole, mem, xh, gamma)
    d = host(x_whole) - host(xh)
    ranges = codec.sign_chunks(n, chunks)
    assert ranges[0][0] == 0 and ranges[-1][1] == codec.sign_words(n)
    for rep in range(2):
        xr = x.clone()
        packed = torch.full((codec.sign_words(n),), -1, dtype=torch.int32, device=DEV)
        norms = torch.full((nseg,), -1.0, device=DEV)
        for i, (w0, w1) in enumerate(ranges):
            codec.sign_compress_range(xr, w0, w1, i == len(ranges) - 1, xhat=xh, seg_off=so, nseg=nseg,
                                      gossip=(mem, gamma) if fused else None, out=(packed, norms))
        assert np.array_equal(host(packed), O.sign_pack(d)), rep
        assert np.allclose(host(norms), O.l1_norms(d, lens), rtol=1e-7, atol=0), rep
        if fused:
            assert same_bits(host(xr), host(x_whole)), rep
    with pytest.raises(RuntimeError, match="word range"):
        codec.sign_compress_range(x, 512, codec.sign_words(n), True, xhat=xh, seg_off=so, nseg=nseg,
                                  out=(packed, norms))


def test_sign_chunked_pack_interrupted_leaves_norms_clean():
    """A chunked sign pack interrupted after its first range (the exchange raises) must not
    leave per-segment L1 sums in the stream's accumulator: the next message's norms are the
    oracle's (CHOCOSignCompressor drops the workspace on failure)."""
    from chocosgd_amd import codec
    from chocosgd_amd.parallel_choco import CHOCOCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer
    lens = [70_001, 5, 1_100_003, 300]
    n, nseg, so = sum(lens), len(lens), seg_table(lens)

    class _FailingAgg:
        rank, neighbor_ranks = 0, [1]

        def __init__(self):
            self.calls = 0

        def _agg(self, data, op, force_wait=True, out=None):
            self.calls += 1
            raise RuntimeError("exchange failed")

    comp = CHOCOCompressor(aggregator=_FailingAgg(), comm_op="sign", comm_device="gpu", compress_ratio=0.0,
                           quantize_level=32, is_biased=False, backend="nccl", use_ipc=False, exchange_chunks=4)
    x, xh = randn(n, 51), randn(n, 52, 0.5)

    def split(t):
        out, p = [], 0
        for m in lens:
            out.append(t[p:p + m].clone())
            p += m
        return out
    sb = {"original_shapes": [(torch.Size([m]), m) for m in lens],
          "flatten_params": TensorBuffer(split(x)), "flatten_hat_params": TensorBuffer(split(xh))}
    with pytest.raises(RuntimeError, match="exchange failed"):
        comp.compress(sb)
    assert comp.compressor_fn.aggregator_fn.calls == 1  # the first range was packed, then the send failed
    x2, xh2 = randn(n, 53), randn(n, 54, 0.5)
    packed, norms = codec.sign_compress(x2, xhat=xh2, seg_off=so, nseg=nseg)
    d2 = host(x2) - host(xh2)
    assert np.array_equal(host(packed), O.sign_pack(d2))
    assert np.allclose(host(norms), O.l1_norms(d2, lens), rtol=1e-7, atol=0)


def test_choco_sign_round_trip_golden():
    from chocosgd_amd import codec
    g = golden("choco_sign_mini")
    lens = g["layout"].tolist()
    so = seg_table(lens)
    msgs = []
    for r in range(3):
        packed, norms = codec.sign_compress(dev(g["x"][r]), xhat=dev(g["xhat"][r]), seg_off=so, nseg=len(lens))
        assert np.array_equal(host(packed), g[f"signs{r}"])
        assert np.allclose(host(norms), g[f"norms{r}"], rtol=1e-5, atol=0)
        msgs.append((dev(g[f"signs{r}"]), dev(g[f"norms{r}"])))  # reference norms pinned
    hat, mem = dev(g["hat0"]), dev(g["mem0"])
    codec.sign_accumulate(msgs, g["weights"].tolist(), int(g["self_rank"]), sum(lens), mem, xhat_self=hat,
                          seg_off=so, nseg=len(lens))
    assert same_bits(host(hat), g["hat1"])
    assert same_bits(host(mem), g["mem1"])


@pytest.mark.parametrize("n,nseg", [(1_000_003, 1), (2_000_000, 7), (65, 3)])
def test_sign_accumulate_vs_oracle(n, nseg):
    from chocosgd_amd import codec
    rng = np.random.default_rng(n)
    cuts = np.sort(rng.choice(np.arange(1, n), size=nseg - 1, replace=False)) if nseg > 1 else np.array([])
    lens = np.diff(np.concatenate([[0], cuts, [n]])).astype(np.int64).tolist()
    so = seg_table(lens)
    msgs_d, msgs_h = [], []
    for r in range(3):
        x = randn(n, 50 + r)
        packed, norms = codec.sign_compress(x, seg_off=so, nseg=len(lens))
        msgs_d.append((packed, norms))
        msgs_h.append((host(packed), host(norms)))
    hat, mem = randn(n, 60), randn(n, 61)
    h0, m0 = host(hat), host(mem)
    w = [1 / 3, 1 / 3, 1 / 3]
    codec.sign_accumulate(msgs_d, w, 1, n, mem, xhat_self=hat, seg_off=so, nseg=len(lens))
    O.sign_accumulate(h0, m0, msgs_h, w, 1, lens)
    assert same_bits(host(hat), h0)
    assert same_bits(host(mem), m0)


# ------------------------------------------------------------------------------------ gossip
def test_gossip_golden():
    from chocosgd_amd import codec
    g = golden("gossip_n10007")
    x = dev(g["x"])
    codec.gossip_step(x, dev(g["mem"]), dev(g["hat"]), float(g["gamma"]))
    assert same_bits(host(x), g["out"])


def test_primitives_accept_host_tensors():
    """BASELINE cfg 1 runs the reference's SignCompressor on CPU tensors: the drop-in
    primitives accept host tensors (staged to the device, computed by the same kernels)
    and return host tensors, equal to the oracle."""
    from chocosgd_amd.sparsification import QuantizationCompressor, SignCompressor, SparsificationCompressor
    n = 1_000_000
    x = torch.from_numpy(np.random.default_rng(5).standard_normal(n).astype(np.float32))
    sc = SignCompressor()
    packed, size = sc.compress(x)
    assert packed.device.type == "cpu" and size == x.size()
    assert np.array_equal(packed.numpy(), O.sign_pack(x.numpy()))
    dec = sc.uncompress(packed, size)
    assert dec.device.type == "cpu"
    assert np.array_equal(dec.numpy(), np.where(x.numpy() < 0, -1.0, 1.0).astype(np.float32))
    vals, idx = SparsificationCompressor().get_top_k(x, 0.99)
    assert vals.device.type == "cpu" and idx.device.type == "cpu"
    ov, oi = O.topk(x.numpy(), O.topk_k(n, 0.99))
    assert np.array_equal(idx.numpy(), oi) and same_bits(vals.numpy(), ov)
    out = QuantizationCompressor().compress(x[:4099].clone(), "quantize_qsgd", 4, False)
    assert out.device.type == "cpu" and out.shape == (4099,)
