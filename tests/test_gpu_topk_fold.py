"""GPU parity: the self-message fold (choco_topk_compress_accumulate /
choco_gossip_topk_compress_accumulate) -- the top-k message plus x_hat += q and
memory += w q applied while the message is emitted -- against the unfused sequence
(topk, then choco_sparse_accumulate of the self message, parallel_choco_v.py:307-310)
and the oracle (the message, and x_hat / memory directly), bit for bit, on every emission path: K34 (cold and warm calls), the
exact fallback inside K34 (tie-heavy and all-equal inputs), the one-workgroup path
(n <= 65536) and k == n."""
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


def _inputs(kind, n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    if kind == "ties":       # the delta takes few distinct values: ties at T, the exact fallback
        hat = x - torch.round(torch.randn(n, generator=g, device=DEV) * 4) / 4
    elif kind == "all_equal":
        hat = x - 0.5
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    return x, hat, mem


@pytest.mark.parametrize("kind,n,ratio", [("randn", 3_000_011, 0.99), ("randn", 65536, 0.99), ("randn", 4097, 0.9),
                                          ("randn", 100_000, 0.0), ("ties", 2_000_003, 0.99),
                                          ("all_equal", 1_000_000, 0.99)])
@pytest.mark.parametrize("fold_memory", [True, False])
def test_topk_fold_matches_unfused(kind, n, ratio, fold_memory):
    from chocosgd_amd import codec
    w = 1.0 / 3.0
    k = codec.topk_k(n, ratio)
    x, hat, mem = _inputs(kind, n, 600 + n % 991)
    hat_a, mem_a = hat.clone(), mem.clone()
    hat_b, mem_b = hat.clone(), mem.clone()
    h_o, m_o = host(hat), host(mem)  # the oracle's x_hat / memory (direct, not only transitive)
    for call in range(3):  # cold, then warm calls (the window carried in the workspace)
        d = (host(x) - host(hat_a)).astype(np.float32)
        va, ia = codec.topk(x, k, xhat=hat_a, fold=(hat_a, mem_a if fold_memory else None, w))
        vb, ib = codec.topk(x, k, xhat=hat_b)
        codec.sparse_accumulate(vb, ib, mem_b, w, xhat_self=hat_b)
        ov, oi = O.topk(d, k)
        assert np.array_equal(host(ia).astype(np.int64), oi), call
        assert same_bits(host(va), ov), call
        assert same_bits(host(hat_a), host(hat_b)), call
        if fold_memory:
            assert same_bits(host(mem_a), host(mem_b)), call
        else:
            codec.sparse_accumulate(va, ia, mem_a, w)  # memory's self update in its turn
            assert same_bits(host(mem_a), host(mem_b)), call
        O.sparse_accumulate(h_o, m_o, ov, oi, w)
        assert same_bits(host(hat_a), h_o), call
        assert same_bits(host(mem_a), m_o), call
        x += 0.01 * randn(n, 7 + call)  # the next call compresses a moved delta


def test_topk_fold_separate_targets():
    """The bench's resident-delta form: compress d (no x_hat), fold into separate x_hat /
    memory buffers."""
    from chocosgd_amd import codec
    n = 5_000_000
    k = codec.topk_k(n, 0.99)
    d = randn(n, 31)
    hat_a, mem_a = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    hat_b, mem_b = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for call in range(3):
        va, ia = codec.topk(d, k, fold=(hat_a, mem_a, 0.5))
        vb, ib = codec.topk(d, k)
        codec.sparse_accumulate(vb, ib, mem_b, 0.5, xhat_self=hat_b)
        assert same_bits(host(va), host(vb)) and torch.equal(ia, ib)
        assert same_bits(host(hat_a), host(hat_b)) and same_bits(host(mem_a), host(mem_b))
        d.mul_(1.01)


@pytest.mark.parametrize("fold_memory", [True, False])
def test_gossip_topk_fold_sequence(fold_memory):
    """The fused consensus step + top-k + fold over a warm sequence (x, memory, x_hat
    evolving) against the unfused step, compress and accumulate, and the oracle."""
    from chocosgd_amd import codec
    n = 3_000_011
    k = codec.topk_k(n, 0.99)
    g = torch.Generator(device=DEV).manual_seed(452)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    xa, hat_a, mem_a = x.clone(), hat.clone(), mem.clone()
    xb, hat_b, mem_b = x.clone(), hat.clone(), mem.clone()
    h_o, m_o = host(hat), host(mem)
    for step in range(5):
        xo = O.gossip_step(host(xa), m_o, h_o, 0.9)
        d = (xo - host(hat_a)).astype(np.float32)
        va, ia = codec.topk(xa, k, xhat=hat_a, gossip=(mem_a, 0.9), fold=(hat_a, mem_a if fold_memory else None, 1.0))
        vb, ib = codec.topk(xb, k, xhat=hat_b, gossip=(mem_b, 0.9))
        codec.sparse_accumulate(vb, ib, mem_b, 1.0, xhat_self=hat_b)
        if not fold_memory:
            codec.sparse_accumulate(va, ia, mem_a, 1.0)
        assert same_bits(host(xa), xo)
        ov, oi = O.topk(d, k)
        assert np.array_equal(host(ia).astype(np.int64), oi)
        assert same_bits(host(va), ov)
        assert same_bits(host(hat_a), host(hat_b)) and same_bits(host(mem_a), host(mem_b))
        O.sparse_accumulate(h_o, m_o, ov, oi, 1.0)
        assert same_bits(host(hat_a), h_o) and same_bits(host(mem_a), m_o)
