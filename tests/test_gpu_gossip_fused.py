"""The fused CHOCO step: update_params_from_neighbor (optim/utils.py:67-72) inside the
compressor's first pass (include/choco_codec.h "fused gossip step").

Golden: ParallelCHOCO_V.step for a ring of 3 run by the reference itself
(tests/golden/gen_golden.py gen_choco_step) -- x after the consensus step, the
messages and the receiver's x_hat / memory.  Oracle: every entry point at sizes that
take each device path (flat K1/K2 stream, small-n / k = n standalone step, batched
segments, > 16M segments, random-k, one- and multi-segment sign, QSGD).
"""
import numpy as np
import pytest
import torch

from conftest import golden, same_bits
from oracle import choco_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
GAMMA = 0.9


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    return t.cpu().numpy()


def _inputs(n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    return x, mem, hat


def _expected(x, mem, hat):
    xa = O.gossip_step(host(x), host(mem), host(hat), GAMMA)
    return xa, (xa - host(hat)).astype(np.float32)


def _split(flat, lens):
    out, p = [], 0
    for m in lens:
        out.append(flat[p:p + m].clone())
        p += m
    return out


class _Capture:
    def __init__(self):
        self.sent = []

    def _agg(self, data, op, force_wait=False):
        self.sent.append(data.clone())
        return [], {}

    def complete_wait(self, reqs):
        pass


class _Replay:
    def __init__(self, per_call):
        self.per_call = list(per_call)

    def _agg(self, data, op, force_wait=False):
        return [], self.per_call.pop(0)

    def complete_wait(self, reqs):
        pass


def _run_step(g, comm_op, ratio=0.9):
    """utils.fused_step's sequence per worker: compress with sync_buffer['gossip'],
    capture; worker self_rank replays the three messages through uncompress."""
    from chocosgd_amd.parallel_choco import CHOCOCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer
    lens = g["layout"].tolist()
    shapes = [(torch.Size([m]), m) for m in lens]
    s = int(g["self_rank"])
    args = dict(aggregator=None, comm_op=comm_op, comm_device="gpu", compress_ratio=ratio, quantize_level=4,
                is_biased=False, backend="nccl", use_ipc=False)
    sent, state = [], []
    for r in range(3):
        comp = CHOCOCompressor(**args)
        nhp = {r: TensorBuffer(_split(dev(g["xhat"][r]), lens)), "memory": TensorBuffer(_split(dev(g["mem"][r]), lens))}
        sb = {"original_shapes": shapes, "flatten_params": TensorBuffer(_split(dev(g["x"][r]), lens)),
              "flatten_hat_params": TensorBuffer(_split(dev(g["xhat"][r]), lens)),
              "gossip": (nhp["memory"].buffer, float(g["gamma"]))}
        comp.compress(sb)
        comp.compressor_fn.aggregator_fn = _Capture()
        comp.sync(sb)
        sent.append(comp.compressor_fn.aggregator_fn.sent)
        state.append((comp, sb, nhp))
    comp, sb, nhp = state[s]
    comp.compressor_fn.aggregator_fn = _Replay([{r: sent[r][c] for r in range(3)} for c in range(len(sent[0]))])
    comp.sync(sb)
    comp.uncompress(sb, nhp, {r: float(w) for r, w in enumerate(g["weights"])})
    return state, s


def test_fused_step_topk_golden():
    g = golden("choco_step_topk_r099")
    state, s = _run_step(g, "compress_top_k", ratio=0.99)
    for r, (_, sb, _) in enumerate(state):
        assert same_bits(host(sb["flatten_params"].buffer), g["x_after_gossip"][r]), f"worker {r} x"
    _, sb, nhp = state[s]
    assert same_bits(host(nhp[s].buffer), g["hat1"])
    assert same_bits(host(nhp["memory"].buffer), g["mem1"])
    assert sb["n_bits"] == float(g["n_bits"])


def test_fused_step_sign_golden():
    """x after the step bit-exact; the accumulate within the device-fp64-norm tolerance
    of test_gpu_choco_api.test_choco_sign_api_close."""
    g = golden("choco_step_sign")
    state, s = _run_step(g, "sign")
    for r, (_, sb, _) in enumerate(state):
        assert same_bits(host(sb["flatten_params"].buffer), g["x_after_gossip"][r]), f"worker {r} x"
    _, sb, nhp = state[s]
    assert np.allclose(host(nhp[s].buffer), g["hat1"], rtol=1e-5, atol=1e-6)
    assert np.allclose(host(nhp["memory"].buffer), g["mem1"], rtol=1e-5, atol=1e-6)


def test_fused_step_helper_updates_model():
    """utils.fused_step end to end on a tiny model: params hold x_new afterwards."""
    from chocosgd_amd import utils
    from chocosgd_amd.parallel_choco import CHOCOCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer

    class Agg:
        def _agg(self, data, op, force_wait=False):
            return [], {0: data}

        def complete_wait(self, reqs):
            pass

    lens = [37, 4096, 5]
    params = [torch.randn(m, device=DEV) for m in lens]
    groups = [{"params": [p], "name": f"p{i}"} for i, p in enumerate(params)]
    names = list(enumerate(g["name"] for g in groups))
    shapes = [(torch.Size([m]), m) for m in lens]
    hat = torch.randn(sum(lens), device=DEV)
    mem = torch.randn(sum(lens), device=DEV)
    nhp = {0: TensorBuffer(_split(hat, lens)), "memory": TensorBuffer(_split(mem, lens))}
    x0 = torch.cat([p.detach().clone() for p in params])
    want = O.gossip_step(host(x0), host(mem), host(hat), GAMMA)
    comp = CHOCOCompressor(aggregator=Agg(), comm_op="compress_top_k", comm_device="gpu", compress_ratio=0.9,
                           quantize_level=4, is_biased=False, backend="nccl", use_ipc=False)
    sb = utils.fused_step(comp, groups, names, shapes, nhp, {0: 1.0}, GAMMA, 0)
    assert same_bits(host(torch.cat([p.detach() for p in params])), want)
    d = (want - host(hat)).astype(np.float32)
    ov, oi, _ = O.topk_segmented(d, lens, 0.9)
    assert same_bits(host(sb["flatten_selected_values"].buffer), ov)


@pytest.mark.parametrize("n,ratio", [(3_000_017, 0.99), (1_000_000, 0.9), (40_000, 0.99), (70_001, 0.0)])
def test_gossip_topk_flat(n, ratio):
    """K1 sample + K2 stream with the step fused (n > 64K, k < n); the standalone step
    otherwise (small n, k = n)."""
    from chocosgd_amd import codec
    x, mem, hat = _inputs(n, n)
    xa, d = _expected(x, mem, hat)
    k = O.topk_k(n, ratio)
    v, i = codec.topk(x, k, xhat=hat, gossip=(mem, GAMMA))
    assert same_bits(host(x), xa)
    ov, oi = O.topk(d, k)
    assert np.array_equal(host(i).astype(np.int64), oi)
    assert same_bits(host(v), ov)


@pytest.mark.parametrize("lens", [[3, 70_001, 5, 1_200_003, 17, 300], [5, 16_777_300, 11]])
def test_gossip_topk_segmented(lens):
    """S1 with the step fused (every batched tile), the flat pipeline's fused stream for
    a segment over 16M (its memory pointer offset by the segment start)."""
    from chocosgd_amd import codec
    n = sum(lens)
    x, mem, hat = _inputs(n, 7)
    xa, d = _expected(x, mem, hat)
    plan = codec.SegmentPlan(lens, 0.99, x.device)
    v, i = codec.topk_segmented(x, plan, xhat=hat, gossip=(mem, GAMMA))
    assert same_bits(host(x), xa)
    ov, oi, _ = O.topk_segmented(d, lens, 0.99)
    assert np.array_equal(host(i).astype(np.int64), oi)
    assert same_bits(host(v), ov)


def test_gossip_randk_segmented():
    from chocosgd_amd import codec
    lens = [3, 70_001, 5, 1_200_003]
    n = sum(lens)
    x, mem, hat = _inputs(n, 8)
    xa, d = _expected(x, mem, hat)
    plan = codec.SegmentPlan(lens, 0.95, x.device)
    v, i = codec.randk_segmented(x, plan, 1234, xhat=hat, gossip=(mem, GAMMA))
    assert same_bits(host(x), xa)
    ov, oi = O.randk_segmented(d, lens, 0.95, 1234)
    assert np.array_equal(host(i).astype(np.int64), oi)
    assert same_bits(host(v), ov)


MANY = np.random.default_rng(6).integers(1, 40, size=1500).tolist() + [300_000]  # past the LDS tables


@pytest.mark.parametrize("lens", [[1_000_003], [4_194_304], [3, 70_001, 5, 1_200_003, 17, 301], [33, 31, 2_000_000],
                                  MANY], ids=["flat", "flat4m", "ragged", "small_first", "many"])
def test_gossip_sign(lens):
    """The one-pass pack with the step fused, one segment and per-tensor norms (small grids: rows
    split over two waves; "many": more tensors than its LDS tables hold)."""
    from chocosgd_amd import codec
    n = sum(lens)
    x, mem, hat = _inputs(n, 9)
    xa, d = _expected(x, mem, hat)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    seg_off = dev(offs) if len(lens) > 1 else None
    packed, norms = codec.sign_compress(x, xhat=hat, seg_off=seg_off, nseg=len(lens), gossip=(mem, GAMMA))
    assert same_bits(host(x), xa)
    assert np.array_equal(host(packed), O.sign_pack(d))
    assert np.allclose(host(norms), O.l1_norms(d, lens), rtol=1e-6, atol=0)


@pytest.mark.parametrize("lens", [[2_000_003], [3, 70_001, 5, 1_200_003], MANY], ids=["flat", "ragged", "many"])
def test_gossip_qsgd(lens):
    """The norm pass with the step fused; levels and signs on the wire vs the oracle with
    the device norms and the device uniforms (SplitMix64)."""
    from chocosgd_amd import codec
    n = sum(lens)
    x, mem, hat = _inputs(n, 10)
    xa, d = _expected(x, mem, hat)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    seg_off = dev(offs) if len(lens) > 1 else None
    packed, norms, _ = codec.qsgd_compress(x, 4, xhat=hat, seg_off=seg_off, nseg=len(lens), seed=77, offset=5,
                                           gossip=(mem, GAMMA))
    assert same_bits(host(x), xa)
    nm = host(norms)
    assert np.allclose(nm, O.l2_norms(d, lens), rtol=1e-6, atol=0)
    u = O.qsgd_uniforms(n, 77, 5)
    lvl, off = [], 0
    for si, m in enumerate(lens):
        lvl.append(O.qsgd_levels(d[off:off + m], 15, u[off:off + m], nm[si]))
        off += m
    assert np.array_equal(host(packed), O.qsgd_pack(np.concatenate(lvl), d, 4))
