"""GPU parity: the deferred receive fused into the next step's first pass (QSGD, sign).

ParallelCHOCO_V.step (parallel_choco_v.py:104-155) joins the previous step's gossip --
whose uncompress applied the neighbours' messages to x_hat / memory (:430-433 QSGD) --
and then runs update_params_from_neighbor (optim/utils.py:67-72) and compress.  The fused
kernels apply the previous messages, the consensus step and this step's first compress
pass in ONE pass; x, x_hat, memory must equal the sequence bit for bit (and the oracle's),
and the norms must be the exact fp64 norms rounded once."""
import numpy as np
import pytest
import torch

from conftest import golden_json, same_bits
from oracle import choco_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
GAMMA = 0.9


def host(t):
    return t.cpu().numpy()


def _state(n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    return x, hat, mem


def _seg(lens):
    if lens is None:
        return None, 1
    return torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int64, device=DEV), len(lens)


@pytest.mark.parametrize("case", ["flat", "ragged", "resnet20", "ten_messages", "no_self"])
def test_qsgd_recv_gossip_norms_matches_sequence(case):
    from chocosgd_amd import codec
    lens = {"flat": None, "ragged": [3, 70_001, 5, 1_200_003, 17, 300],
            "resnet20": golden_json("layouts.json")["resnet20_cifar10"],
            "ten_messages": None, "no_self": [1000, 2_000_001]}[case]
    n = sum(lens) if lens else (1_000_003 if case == "flat" else 262_147)
    seg_off, nseg = _seg(lens)
    q, nmsg = 4, (10 if case == "ten_messages" else 3)
    self_slot = -1 if case == "no_self" else 1
    weights = [1.0 / nmsg] * nmsg
    # the previous step's messages (compressed from other deltas on the device)
    msgs = []
    for r in range(nmsg):
        d = torch.randn(n, generator=torch.Generator(device=DEV).manual_seed(40 + r), device=DEV)
        packed, norms = codec.qsgd_compress(d, q, seg_off=seg_off, nseg=nseg, seed=r, offset=3)[:2]
        msgs.append((packed, norms))
    x, hat, mem = _state(n, 11 + nmsg)
    xa, ha, ma = x.clone(), hat.clone(), mem.clone()
    xb, hb, mb = x.clone(), hat.clone(), mem.clone()
    # the sequence: uncompress, update_params_from_neighbor, the norm pass
    codec.qsgd_accumulate(msgs, weights, self_slot, n, q, ma, xhat_self=ha if self_slot >= 0 else None,
                          seg_off=seg_off, nseg=nseg)
    codec.gossip_step(xa, ma, ha, GAMMA)
    na = codec.qsgd_norms(xa, xhat=ha, seg_off=seg_off, nseg=nseg)
    # fused
    nb = codec.qsgd_recv_gossip_norms(msgs, weights, self_slot, xb, mb, hb, GAMMA, q, seg_off=seg_off, nseg=nseg)
    assert same_bits(host(xb), host(xa)) and same_bits(host(hb), host(ha)) and same_bits(host(mb), host(ma))
    # the oracle's receive + consensus step
    h0, m0, x0 = host(hat), host(mem), host(x)
    dec = []
    for p, nm in msgs:
        lv, neg = O.qsgd_unpack(host(p), n, q)
        off, parts = 0, []
        for si, L in enumerate(lens or [n]):
            parts.append(O.qsgd_decode(lv[off:off + L], neg[off:off + L], host(nm)[si], 15, L))
            off += L
        dec.append(np.concatenate(parts))
    hs = h0.copy()
    O.qsgd_accumulate(hs, m0, dec, weights, self_slot if self_slot >= 0 else -1)
    if self_slot < 0:
        hs = h0
    xo = O.gossip_step(x0, m0, hs, GAMMA)
    assert same_bits(host(xb), xo) and same_bits(host(mb), m0) and same_bits(host(hb), hs)
    # norms: the exact fp64 norms of x_new - x_hat, rounded once (both passes)
    exact = O.l2_norms((xo - hs).astype(np.float32), lens or [n])
    assert np.allclose(host(nb), exact, rtol=1e-6, atol=0) and np.allclose(host(na), exact, rtol=1e-6, atol=0)
    # this step's message from the fused pass's norms: the quantize pass as usual
    pa = codec.qsgd_compress(xb, q, xhat=hb, seg_off=seg_off, nseg=nseg, norm_in=nb, seed=9, offset=1)[0]
    pb = codec.qsgd_compress(xa, q, xhat=ha, seg_off=seg_off, nseg=nseg, norm_in=nb, seed=9, offset=1)[0]
    assert torch.equal(pa, pb)


def test_qsgd_recv_gossip_norms_repeated_steps():
    """A sequence of deferred steps (each step's fused pass applies the previous step's
    message) against the unfused sequence: the accumulators' replicas are left clean."""
    from chocosgd_amd import codec
    n, q = 2_000_003, 4
    x, hat, mem = _state(n, 5)
    xa, ha, ma = x.clone(), hat.clone(), mem.clone()
    xb, hb, mb = x.clone(), hat.clone(), mem.clone()
    pend_a = pend_b = None
    for step in range(4):
        if pend_a is not None:
            codec.qsgd_accumulate([pend_a], [1.0], 0, n, q, ma, xhat_self=ha)
            codec.gossip_step(xa, ma, ha, GAMMA)
            na = codec.qsgd_norms(xa, xhat=ha)
            nb = codec.qsgd_recv_gossip_norms([pend_b], [1.0], 0, xb, mb, hb, GAMMA, q)
            assert same_bits(host(xb), host(xa)) and same_bits(host(hb), host(ha))
            assert same_bits(host(mb), host(ma))
            assert np.allclose(host(nb), host(na), rtol=1e-6, atol=0)
        else:
            nb = codec.qsgd_norms(xb, xhat=hb, gossip=(mb, GAMMA))
            codec.gossip_step(xa, ma, ha, GAMMA)
        pend_a = codec.qsgd_compress(xa, q, xhat=ha, norm_in=nb, seed=step, offset=0)[:2]
        pend_b = codec.qsgd_compress(xb, q, xhat=hb, norm_in=nb, seed=step, offset=0)[:2]
        assert torch.equal(pend_a[0], pend_b[0])


def _sign_msgs(n, nmsg, seg_off, nseg):
    from chocosgd_amd import codec
    out = []
    for r in range(nmsg):
        d = torch.randn(n, generator=torch.Generator(device=DEV).manual_seed(60 + r), device=DEV)
        out.append(codec.sign_compress(d, seg_off=seg_off, nseg=nseg))
    return out


@pytest.mark.parametrize("case", ["flat", "odd_n", "one_message", "eight_messages", "ten_messages", "no_self",
                                  "segmented", "resnet20", "tiny_segments", "segmented_no_self"])
def test_sign_recv_gossip_compress_matches_sequence(case):
    """choco_sign_recv_gossip_compress (CHOCOSignCompressor.uncompress, parallel_choco_v.py:548-558,
    then the consensus step and the next compress, :476-506) against sign_accumulate +
    the gossip-fused pack, and against the oracle, bit for bit (norms: the exact fp64 L1
    norms rounded once, rtol 1e-6)."""
    from chocosgd_amd import codec
    # tiny_segments: 300 segments of 1-13 elements in the first runs (more than kRowSegLds in one
    # run: the global per-segment sums), then large ones
    lens = {"segmented": [3, 70_001, 5, 400_003], "segmented_no_self": [4097, 1, 250_000, 9],
            "resnet20": golden_json("layouts.json")["resnet20_cifar10"],
            "tiny_segments": [1 + (i * 7) % 13 for i in range(300)] + [65_536, 3, 200_001]}.get(case)
    n = sum(lens) if lens else {"flat": 4_000_000, "odd_n": 1_234_567}.get(case, 777_777)
    seg_off, nseg = _seg(lens)
    nmsg = {"one_message": 1, "eight_messages": 8, "ten_messages": 10}.get(case, 3)
    self_slot = -1 if case in ("no_self", "segmented_no_self") else min(1, nmsg - 1)
    weights = [0.25 + 0.5 / (q + 1) for q in range(nmsg)]
    msgs = _sign_msgs(n, nmsg, seg_off, nseg)
    x, hat, mem = _state(n, 21 + nmsg)
    xa, ha, ma = x.clone(), hat.clone(), mem.clone()
    xb, hb, mb = x.clone(), hat.clone(), mem.clone()
    codec.sign_accumulate(msgs, weights, self_slot, n, ma, xhat_self=ha if self_slot >= 0 else None,
                          seg_off=seg_off, nseg=nseg)
    pa, na = codec.sign_compress(xa, xhat=ha, seg_off=seg_off, nseg=nseg, gossip=(ma, GAMMA))
    pb, nb = codec.sign_recv_gossip_compress(msgs, weights, self_slot, xb, mb, hb, GAMMA, seg_off=seg_off, nseg=nseg)
    assert same_bits(host(xb), host(xa)) and same_bits(host(hb), host(ha)) and same_bits(host(mb), host(ma))
    assert torch.equal(pb, pa)
    # the oracle: receive, consensus step, pack
    seg_lens = lens or [n]
    h0, m0 = host(hat).copy(), host(mem).copy()
    O.sign_accumulate(h0 if self_slot >= 0 else None, m0, [(host(p), host(q)) for p, q in msgs], weights,
                      self_slot, seg_lens)
    xo = O.gossip_step(host(x), m0, h0, GAMMA)
    assert same_bits(host(xb), xo) and same_bits(host(mb), m0) and same_bits(host(hb), h0)
    d = (xo - h0).astype(np.float32)
    assert np.array_equal(host(pb), O.sign_pack(d))
    exact = O.l1_norms(d, seg_lens)
    assert np.allclose(host(nb), exact, rtol=1e-6, atol=0) and np.allclose(host(na), exact, rtol=1e-6, atol=0)


@pytest.mark.parametrize("n", [1, 7, 32, 33, 1_023, 32 * 4_096 + 1, 32 * 4_097 + 5, 32 * 8_192 - 3])
def test_sign_recv_gossip_compress_small_and_ragged(n):
    """Sizes at the edges of the receive's layout: fewer words than one 32-word plane block,
    word counts one past a 4096-column run, a last row shorter than the others -- against
    the unfused sequence and the oracle's pack, bit for bit."""
    from chocosgd_amd import codec
    nmsg, self_slot, weights = 2, 0, [0.5, 0.25]
    msgs = _sign_msgs(n, nmsg, None, 1)
    x, hat, mem = _state(n, 5)
    xa, ha, ma = x.clone(), hat.clone(), mem.clone()
    xb, hb, mb = x.clone(), hat.clone(), mem.clone()
    codec.sign_accumulate(msgs, weights, self_slot, n, ma, xhat_self=ha)
    pa, na = codec.sign_compress(xa, xhat=ha, gossip=(ma, GAMMA))
    pb, nb = codec.sign_recv_gossip_compress(msgs, weights, self_slot, xb, mb, hb, GAMMA)
    assert same_bits(host(xb), host(xa)) and same_bits(host(hb), host(ha)) and same_bits(host(mb), host(ma))
    assert torch.equal(pb, pa)
    d = (host(xb) - host(hb)).astype(np.float32)
    assert np.array_equal(host(pb), O.sign_pack(d))
    assert np.allclose(host(nb), O.l1_norms(d, [n]), rtol=1e-6, atol=0)


def test_sign_recv_workspace_reuse_across_layouts():
    """One cached receive workspace over calls whose accumulators and planes sit at different
    offsets (flat, 4 segments, 65 segments, flat again; largest n first so it is never
    reallocated): each call's norms are the exact per-segment L1 norms."""
    from chocosgd_amd import codec
    for lens in ([1_000_003], [3, 70_001, 5, 400_003], golden_json("layouts.json")["resnet20_cifar10"],
                 [1_000_003], [1 + (i * 7) % 13 for i in range(300)] + [65_536]):
        n = sum(lens)
        seg_off, nseg = _seg(lens if len(lens) > 1 else None)
        msgs = _sign_msgs(n, 2, seg_off, nseg)
        x, hat, mem = _state(n, 31)
        pb, nb = codec.sign_recv_gossip_compress(msgs, [0.5, 0.25], 0, x, mem, hat, GAMMA, seg_off=seg_off,
                                                 nseg=nseg)
        d = (host(x) - host(hat)).astype(np.float32)
        assert np.array_equal(host(pb), O.sign_pack(d))
        assert np.allclose(host(nb), O.l1_norms(d, lens), rtol=1e-6, atol=0)


def test_sign_recv_gossip_compress_repeated_steps():
    """Deferred sign steps (own message double-buffered, as bench.py --defer-receive) against
    the unfused sequence over several steps: the L1 accumulator is left clean each call."""
    from chocosgd_amd import codec
    n = 3_000_017
    x, hat, mem = _state(n, 9)
    xa, ha, ma = x.clone(), hat.clone(), mem.clone()
    xb, hb, mb = x.clone(), hat.clone(), mem.clone()
    bufs = [(torch.empty(codec.sign_words(n), dtype=torch.int32, device=DEV),
             torch.empty(1, dtype=torch.float32, device=DEV)) for _ in range(2)]
    other = _sign_msgs(n, 1, None, 1)[0]
    pend_a = pend_b = None
    for step in range(4):
        if pend_a is None:
            pa = codec.sign_compress(xa, xhat=ha, gossip=(ma, GAMMA))
            pb = codec.sign_compress(xb, xhat=hb, gossip=(mb, GAMMA), out=bufs[step % 2])
        else:
            codec.sign_accumulate([pend_a, other], [0.5, 0.5], 0, n, ma, xhat_self=ha)
            pa = codec.sign_compress(xa, xhat=ha, gossip=(ma, GAMMA))
            pb = codec.sign_recv_gossip_compress([pend_b, other], [0.5, 0.5], 0, xb, mb, hb, GAMMA,
                                                 out=bufs[step % 2])
        assert same_bits(host(xb), host(xa)) and same_bits(host(hb), host(ha)) and same_bits(host(mb), host(ma))
        assert torch.equal(pa[0], pb[0])
        assert np.allclose(host(pa[1]), host(pb[1]), rtol=1e-6, atol=0)
        pend_a, pend_b = pa, pb


def test_sign_recv_gossip_compress_rejects_aliased_output():
    from chocosgd_amd import codec
    n = 100_000
    msgs = _sign_msgs(n, 2, None, 1)
    x, hat, mem = _state(n, 3)
    with pytest.raises(RuntimeError, match="alias"):
        codec.sign_recv_gossip_compress(msgs, [0.5, 0.5], 0, x, mem, hat, GAMMA, out=msgs[0])
    # a PARTIAL overlap (the output words start inside message 1's words) is refused too
    words, norms = msgs[1]
    big = torch.zeros(words.numel() + 64, dtype=torch.int32, device=DEV)
    big[:words.numel()].copy_(words)
    shifted = (big[:words.numel()], norms)
    out = (big[32:32 + words.numel()], torch.empty_like(norms))
    with pytest.raises(RuntimeError, match="alias"):
        codec.sign_recv_gossip_compress([msgs[0], shifted], [0.5, 0.5], 0, x, mem, hat, GAMMA, out=out)


@pytest.mark.parametrize("lens", [[37, 40_000, 5, 123_457], [163_499], golden_json("layouts.json")["resnet20_cifar10"]],
                         ids=["ragged", "flat", "resnet20"])
@pytest.mark.parametrize("comm_op", ["quantize_qsgd", "sign"])
def test_fused_step_defer_receive_drop_in(comm_op, lens):
    """utils.fused_step(defer_receive=True) through the drop-in CHOCOCompressor against
    fused_step without it, over four steps of a two-worker neighbourhood (the neighbour's
    messages replayed): the model's params bit-identical after every step, x_hat / memory
    bit-identical after flush_receive(); a non-deferred step after deferred ones flushes
    first."""
    from chocosgd_amd import codec, utils
    from chocosgd_amd.parallel_choco import CHOCOCompressor
    from chocosgd_amd.tensor_buffer import TensorBuffer
    n = sum(lens)
    shapes = [(torch.Size([m]), m) for m in lens]
    nseg = len(lens)
    seg_off = torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int64, device=DEV) if nseg > 1 else None

    def neighbour_msg(step):
        d = torch.randn(n, generator=torch.Generator(device=DEV).manual_seed(500 + step), device=DEV)
        if comm_op == "sign":
            msg, out = codec.sign_wire(n, nseg, DEV)
            codec.sign_compress(d, seg_off=seg_off, nseg=nseg, out=out)
        else:
            msg, out = codec.qsgd_wire(n, 4, nseg, DEV)
            codec.qsgd_compress(d, 4, seg_off=seg_off, nseg=nseg, seed=step, out=out)
        return msg

    others = [neighbour_msg(s) for s in range(6)]

    class Agg:
        def __init__(self):
            self.calls = 0

        def _agg(self, data, op, force_wait=False):
            self.calls += 1
            return [], {0: data, 1: others[self.calls - 1]}

        def complete_wait(self, reqs):
            pass

    def run(defer_steps):
        torch.manual_seed(1)  # the QSGD seeds (one draw per compress)
        g = torch.Generator(device=DEV).manual_seed(2)
        params = [torch.randn(m, generator=g, device=DEV) for m in lens]
        groups = [{"params": [p], "name": f"p{i}"} for i, p in enumerate(params)]
        names = list(enumerate(gr["name"] for gr in groups))
        hat = torch.cat([p.detach() for p in params]) + 0.1 * torch.randn(n, generator=g, device=DEV)
        mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
        nhp = {0: TensorBuffer.from_flat(hat, [(m,) for m in lens]), "memory": TensorBuffer.from_flat(mem, [(m,) for m in lens])}
        comp = CHOCOCompressor(aggregator=Agg(), comm_op=comm_op, comm_device="gpu", compress_ratio=0.9,
                               quantize_level=4, is_biased=False, backend="nccl", use_ipc=False)
        xs = []
        for step, defer in enumerate(defer_steps):
            with torch.no_grad():
                for i, p in enumerate(params):  # apply_gradient stand-in: x only
                    p.sub_(0.01 * torch.randn(p.shape, generator=torch.Generator(device=DEV).manual_seed(step * 10 + i),
                                              device=DEV))
            utils.fused_step(comp, groups, names, shapes, nhp, {0: 0.5, 1: 0.5}, GAMMA, 0, defer_receive=defer)
            xs.append(torch.cat([p.detach() for p in params]).cpu().numpy())
        comp.flush_receive()
        return xs, host(hat), host(mem)

    xa, ha, ma = run([False] * 5)
    xb, hb, mb = run([True, True, True, False, True])
    for s, (a, b) in enumerate(zip(xa, xb)):
        assert same_bits(b, a), f"params after step {s}"
    assert same_bits(hb, ha) and same_bits(mb, ma)
