"""GPU parity: the one-call receive of all messages (choco_sparse_accumulate_multi) against
the oracle's per-message sequence (parallel_choco_v.py:291-310: for each (rank, weight) in
neighbors_info, x_hat[idx] += v for the self rank, memory[idx] += weight * v), bit for
bit: messages whose indices share 64-B lines and elements, ranges with more than 256
updates, ragged n, more than 8 messages, the per-message path (sparse messages, an
unaligned memory view) and corrupt indices."""
import numpy as np
import pytest
import torch

from conftest import same_bits
from oracle import choco_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def host(t):
    return t.cpu().numpy()


def _messages(n, ks, seed, shared=0.3):
    """Ascending distinct index sets; message m > 0 re-uses a fraction `shared` of message
    0's indices (the same elements) and puts others next to them (the same lines)."""
    rng = np.random.default_rng(seed)
    base = np.sort(rng.choice(n, size=ks[0], replace=False))
    out = []
    for m, k in enumerate(ks):
        if m == 0:
            idx = base
        else:
            a = rng.choice(base, size=min(k, int(shared * k)), replace=False)
            b = np.clip(rng.choice(base, size=k // 4) + rng.integers(1, 15, size=k // 4), 0, n - 1)
            c = rng.choice(n, size=k, replace=False)
            idx = np.unique(np.concatenate([a, b, c]))[:k]
            if idx.size < k:  # top up with unused indices
                rest = np.setdiff1d(np.arange(n), idx)[: k - idx.size]
                idx = np.sort(np.concatenate([idx, rest]))
        vals = rng.standard_normal(idx.size).astype(np.float32)
        out.append((vals, idx.astype(np.int64)))
    return out


def _run(n, msgs, weights, self_slot, mem_view=None, guard=None):
    from chocosgd_amd import codec
    rng = np.random.default_rng(n)
    hat0 = rng.standard_normal(n).astype(np.float32)
    mem0 = rng.standard_normal(n).astype(np.float32)
    hat = torch.from_numpy(hat0).to(DEV)
    if mem_view is None:
        mem = torch.from_numpy(mem0).to(DEV)
        mem_t = mem
    else:
        mem_t = torch.zeros(n + mem_view, device=DEV)
        mem_t[mem_view:] = torch.from_numpy(mem0).to(DEV)
        mem = mem_t[mem_view:]
    dm = [(torch.from_numpy(v).to(DEV), torch.from_numpy(i.astype(np.int32)).to(DEV)) for v, i in msgs]
    codec.sparse_accumulate_multi(dm, weights, mem, self_slot=self_slot,
                                  xhat_self=hat if self_slot >= 0 else None, guard=guard)
    h, m = hat0.copy(), mem0.copy()
    for s, ((v, i), w) in enumerate(zip(msgs, weights)):
        ok = (i >= 0) & (i < n)
        O.sparse_accumulate(h if s == self_slot else None, m, v[ok], i[ok], w)
    return host(hat), host(mem), h, m


@pytest.mark.parametrize("n,ks,self_slot", [(2_000_003, [20_000, 20_000, 20_000], 1),
                                            (4096 * 300, [12_288, 12_288, 12_288], 0),
                                            (1_000_003, [600_000, 300_000, 5_000], 2),  # > 256 per range
                                            (100_000, [1_000, 900, 800, 700, 600, 500, 400, 300], 7),
                                            (3_000_017, [30_000] * 10, 4)])  # > 8: two chunks
def test_sparse_multi_matches_sequence(n, ks, self_slot):
    msgs = _messages(n, ks, seed=n % 1009)
    weights = [1.0 / len(ks)] * len(ks)
    weights[0] = 0.3
    h_gpu, m_gpu, h, m = _run(n, msgs, weights, self_slot)
    assert same_bits(h_gpu, h)
    assert same_bits(m_gpu, m)


def test_sparse_multi_last_element_and_partial_segment():
    """Updates in the buffer's last, partial 64-B segment and at index n - 1."""
    n = 4096 * 5 + 7
    rng = np.random.default_rng(5)
    msgs = []
    for m in range(3):
        idx = np.unique(np.concatenate([rng.choice(n - 16, 40, replace=False), [n - 7, n - 3, n - 1]]))
        msgs.append((rng.standard_normal(idx.size).astype(np.float32), idx))
    h_gpu, m_gpu, h, m = _run(n, msgs, [1 / 3] * 3, 1)
    assert same_bits(h_gpu, h) and same_bits(m_gpu, m)


@pytest.mark.parametrize("case", ["sparse_messages", "unaligned_memory", "no_self", "empty_message"])
def test_sparse_multi_per_message_paths(case):
    n = 2_000_000
    ks = {"sparse_messages": [100, 50, 10]}.get(case, [20_000, 15_000, 10_000])
    if case == "empty_message":
        ks = [20_000, 0, 10_000]
    msgs = _messages(n, [max(k, 1) for k in ks], seed=77)
    msgs = [(v[:k], i[:k]) for (v, i), k in zip(msgs, ks)]
    self_slot = -1 if case == "no_self" else 0
    h_gpu, m_gpu, h, m = _run(n, msgs, [0.25, 0.5, 0.25], self_slot,
                              mem_view=1 if case == "unaligned_memory" else None)
    assert same_bits(h_gpu, h) and same_bits(m_gpu, m)


def test_sparse_multi_bad_indices_counted():
    from chocosgd_amd import codec
    n = 1_000_000
    msgs = _messages(n, [10_000, 10_000, 10_000], seed=3)
    v, i = msgs[1]
    i = i.copy()
    i[-1] = n + 5  # out of range (still ascending)
    msgs[1] = (v, i)
    guard = codec.IndexGuard(torch.device(DEV))
    h_gpu, m_gpu, h, m = _run(n, msgs, [1 / 3] * 3, 0, guard=guard)
    assert same_bits(h_gpu, h) and same_bits(m_gpu, m)  # the bad update skipped, the rest applied
    guard.arm()
    with pytest.raises(RuntimeError, match="out of range"):
        guard.check(wait=True)


def test_sparse_multi_ring3_topk_messages():
    """A ring-3 receive of real top-k messages (k = 1 %) against the per-message kernel."""
    from chocosgd_amd import codec
    n = 5_000_011
    k = codec.topk_k(n, 0.99)
    g = torch.Generator(device=DEV).manual_seed(8)
    msgs = []
    for r in range(3):
        d = torch.randn(n, generator=g, device=DEV)
        msgs.append(codec.topk(d, k))
    hat = torch.randn(n, generator=g, device=DEV)
    mem = torch.randn(n, generator=g, device=DEV)
    h2, m2 = hat.clone(), mem.clone()
    w = [1 / 3] * 3
    codec.sparse_accumulate_multi(msgs, w, mem, self_slot=1, xhat_self=hat)
    for r, (v, i) in enumerate(msgs):
        codec.sparse_accumulate(v, i, m2, w[r], xhat_self=h2 if r == 1 else None)
    assert same_bits(host(hat), host(h2))
    assert same_bits(host(mem), host(m2))
