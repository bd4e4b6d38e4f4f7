"""GPU parity at BASELINE.json's full sizes, through size-independent sampled checks.

cfg 5 (sign + L1 norm on 345M fp32) and cfg 3 (QSGD q=4 on 100M fp32) are too
large for the CPU oracle to redo whole, but every output word / element depends
on a known set of inputs: word j of the (32, N') sign layout on elements
j + r*N' (sparsification.py:129-145), QSGD element e on d[e], u[e] and the norm
(sparsification.py:87-98).  So a column / element sample is checked EXACTLY
against the oracle, and the norms against fp64 sums of the whole buffer.
"""
import numpy as np
import pytest
import torch

from conftest import same_bits
from oracle import choco_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def host(t):
    return t.cpu().numpy()


def randn(n, seed, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(n, generator=g, device=DEV) * scale


def _sample(lo, hi, count, seed):
    rng = np.random.default_rng(seed)
    s = np.unique(np.concatenate([rng.integers(lo, hi, size=count), np.arange(lo, min(hi, lo + 64)),
                                  np.arange(max(lo, hi - 64), hi)]))
    return s.astype(np.int64)


def test_sign_345M_words_norm_accumulate():
    """cfg 5 per worker: n = 345,000,000, N' = 10,781,250 words.  Sampled words vs the
    oracle; the L1 norm vs fp64; the fused accumulate of two messages on the sampled
    columns (all 32 rows of each)."""
    from chocosgd_amd import codec
    n = 345_000_000
    Np = O.sign_words(n)
    x = randn(n, 2000)
    xh = randn(n, 2001, 0.25)
    packed, norms = codec.sign_compress(x, xhat=xh)
    cols = _sample(0, Np, 8192, 5)
    rows = np.arange(32, dtype=np.int64)
    elems = (cols[:, None] + rows[None, :] * Np).reshape(-1)
    elems_t = torch.from_numpy(elems).to(DEV)
    d_s = (host(x[elems_t]) - host(xh[elems_t])).reshape(len(cols), 32)
    exp_words = np.zeros(len(cols), dtype=np.uint64)
    for r in range(32):
        exp_words |= (d_s[:, r] < 0).astype(np.uint64) << np.uint64(r)
    got = host(packed[torch.from_numpy(cols).to(DEV)]).view(np.uint32)
    assert np.array_equal(got, exp_words.astype(np.uint32))
    d_full = x - xh
    exact = float(torch.sum(torch.abs(d_full), dtype=torch.float64))
    assert abs(float(host(norms)[0]) - exact) <= 1e-6 * exact
    # second message (another worker's delta), then accumulate [self, other]
    packed2, norms2 = codec.sign_compress(randn(n, 2002))
    del x, xh, d_full
    hat, mem = randn(n, 2003), randn(n, 2004)
    h0, m0 = host(hat[elems_t]), host(mem[elems_t])
    w = [1 / 3, 2 / 3]
    codec.sign_accumulate([(packed, norms), (packed2, norms2)], w, 0, n, mem, xhat_self=hat)
    words = [got, host(packed2[torch.from_numpy(cols).to(DEV)]).view(np.uint32)]
    nrm = [host(norms)[0], host(norms2)[0]]
    h, m = h0.reshape(len(cols), 32).copy(), m0.reshape(len(cols), 32).copy()
    for q in range(2):
        bits = (words[q][:, None] >> rows[None, :].astype(np.uint32)) & 1
        sg = np.where(bits == 1, np.float32(-1), np.float32(1))
        upd = ((np.float32(nrm[q]) / np.float32(n)).astype(np.float32) * sg).astype(np.float32)
        if q == 0:
            h = (h + upd).astype(np.float32)
        m = (np.float64(np.float32(w[q])) * upd.astype(np.float64) + m.astype(np.float64)).astype(np.float32)
    assert same_bits(host(hat[elems_t]), h.reshape(-1))
    assert same_bits(host(mem[elems_t]), m.reshape(-1))


def test_qsgd_100M_levels_wire_decode():
    """cfg 3: n = 100,000,000, q = 4 (s = 15).  Sampled levels and signs on the wire vs the
    oracle (the device SplitMix64 uniforms restated), the dense decode of those elements bit-exact,
    and the norm vs fp64."""
    from chocosgd_amd import codec
    n, q = 100_000_000, 4
    s = 2 ** q - 1
    x = randn(n, 1000)
    seed, offset = 0xC0FFEE, 3
    packed, norms, _ = codec.qsgd_compress(x, q, seed=seed, offset=offset)
    exact = float(torch.sqrt(torch.sum(x.double() ** 2)))
    nrm = float(host(norms)[0])
    assert abs(nrm - exact) <= 1e-6 * exact
    idx = _sample(0, n, 1 << 20, 9)
    d = host(x[torch.from_numpy(idx).to(DEV)])
    u = O.qsgd_uniforms_at(idx, seed, offset)
    lvl = O.qsgd_levels(d, s, u, nrm)
    exp_lvl = np.minimum(lvl, s).astype(np.int64)
    got_lvl, got_neg = O.qsgd_wire_at(host(packed), n, q, idx)
    assert np.array_equal(got_lvl, exp_lvl)
    assert np.array_equal(got_neg, d < 0)
    assert lvl.max() >= 1  # non-trivial levels are present in the sample
    dec = codec.qsgd_decode(packed, norms, n, q)
    assert same_bits(host(dec[torch.from_numpy(idx).to(DEV)]), O.qsgd_dense(d, s, u, nrm))


@pytest.mark.parametrize("n,nmsg", [(345_000_000, 1), (345_000_000, 3), ((1 << 30) - 1, 1), (1 << 30, 1)])
def test_sign_345M_deferred_receive_matches_sequence(n, nmsg):
    """cfg 5's deferred receive at full size: choco_sign_recv_gossip_compress (row runs over bit
    planes) against sign_accumulate + the gossip-fused pack on the same inputs, compared whole on
    the device -- x, x_hat, memory and the words bit for bit, the L1 norm to rtol 1e-6; also the
    largest one-pass size (2^30 - 1: 32-bit buffer offsets) and the first two-kernel one (2^30).
    (The sequence itself is pinned against the oracle at small sizes: test_gpu_deferred_receive.py.)"""
    from chocosgd_amd import codec
    gamma = 0.5
    msgs = [codec.sign_compress(randn(n, 2100 + q, 0.5)) for q in range(nmsg)]
    weights = [1.0 / 3.0 + 0.125 * q for q in range(nmsg)]
    self_slot = nmsg // 2
    x, xh, mem = randn(n, 2010), randn(n, 2011, 0.25), randn(n, 2012, 0.1)
    xa, ha, ma = x, xh, mem
    xb, hb, mb = x.clone(), xh.clone(), mem.clone()
    codec.sign_accumulate(msgs, weights, self_slot, n, ma, xhat_self=ha)
    pa, na = codec.sign_compress(xa, xhat=ha, gossip=(ma, gamma))
    pb, nb = codec.sign_recv_gossip_compress(msgs, weights, self_slot, xb, mb, hb, gamma)
    assert torch.equal(xb.view(torch.int32), xa.view(torch.int32))
    assert torch.equal(hb.view(torch.int32), ha.view(torch.int32))
    assert torch.equal(mb.view(torch.int32), ma.view(torch.int32))
    assert torch.equal(pb, pa)
    assert abs(float(nb[0]) - float(na[0])) <= 1e-6 * abs(float(na[0]))
    del msgs, x, xh, mem, xb, hb, mb
    codec.release_workspaces()
    torch.cuda.empty_cache()


def test_qsgd_100M_deferred_receive_matches_sequence():
    """cfg 3's deferred receive at full size (q = 4, three messages): choco_qsgd_recv_gossip_norms
    against qsgd_accumulate + the consensus step + the norm pass, compared whole on the device --
    x, x_hat, memory bit for bit, the norm to rtol 1e-6 -- and the next message from either."""
    from chocosgd_amd import codec
    n, q, nmsg, gamma = 100_000_000, 4, 3, 0.5
    msgs = [codec.qsgd_compress(randn(n, 2200 + r), q, seed=r, offset=3)[:2] for r in range(nmsg)]
    weights = [1.0 / nmsg] * nmsg
    x, xh, mem = randn(n, 2020), randn(n, 2021, 0.25), randn(n, 2022, 0.1)
    xa, ha, ma = x, xh, mem
    xb, hb, mb = x.clone(), xh.clone(), mem.clone()
    codec.qsgd_accumulate(msgs, weights, 1, n, q, ma, xhat_self=ha)
    codec.gossip_step(xa, ma, ha, gamma)
    na = codec.qsgd_norms(xa, xhat=ha)
    nb = codec.qsgd_recv_gossip_norms(msgs, weights, 1, xb, mb, hb, gamma, q)
    assert torch.equal(xb.view(torch.int32), xa.view(torch.int32))
    assert torch.equal(hb.view(torch.int32), ha.view(torch.int32))
    assert torch.equal(mb.view(torch.int32), ma.view(torch.int32))
    assert abs(float(nb[0]) - float(na[0])) <= 1e-6 * abs(float(na[0]))
    pa = codec.qsgd_compress(xa, q, xhat=ha, norm_in=nb, seed=9, offset=1)[0]
    pb = codec.qsgd_compress(xb, q, xhat=hb, norm_in=nb, seed=9, offset=1)[0]
    assert torch.equal(pa, pb)
    del msgs, x, xh, mem, xb, hb, mb
    codec.release_workspaces()
    torch.cuda.empty_cache()
