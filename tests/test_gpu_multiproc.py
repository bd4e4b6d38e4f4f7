"""The CHOCO gossip round across PROCESSES: CHOCOCompressor compress -> sync ->
uncompress on 2, 3, 4 and 8 ranks sharing the one GPU, exchanging through the
reference's DecentralizedAggregation over gloo with comm_device="cpu"
(communication.py:246-291, parallel_choco_v.py:262-310).  Every worker's
x_hat / memory is compared with the oracle's round over the same inputs.

The ranks are started by tests/_mp_choco_worker.py in a fresh interpreter, so
the processes that use the GPU are not forked from this (GPU-initialised) one.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, golden_json, same_bits
from oracle import choco_oracle as O

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _mp_choco_worker as W  # noqa: E402


def _neighborhood(rank, world):
    """The reference's own mixing-matrix row (RingGraph / CompleteGraph, generated from
    topology.py:122-299 into tests/golden/ring_neighborhoods.json)."""
    return {int(r): float(w) for r, w in golden_json("ring_neighborhoods.json")[str(world)][rank]}


def _hdr(nseg):
    return (nseg + 3) // 4 * 4


@pytest.mark.parametrize("comm_op,world", [("compress_top_k", 2), ("compress_top_k", 3), ("compress_random_k", 3),
                                           ("sign", 2), ("sign", 3), ("quantize_qsgd", 3),
                                           # rings larger than 3 (cfg 4 / 5 are 8-worker rings): every
                                           # rank exchanges with 2 of N - 1 peers and skips the rest
                                           ("compress_top_k", 4), ("sign", 4), ("quantize_qsgd", 4),
                                           ("compress_top_k", 8), ("sign_chunked", 4),
                                           ("quantize_qsgd_chunked", 2), ("quantize_qsgd_chunked", 3),
                                           ("sign_chunked", 2), ("sign_chunked", 3),
                                           ("sign_chunked_refagg", 3)])
def test_choco_round_across_processes(comm_op, world, tmp_path):
    """(`*_refagg`: the aggregator has the reference's `_agg(data, op, force_wait)` signature,
    without this package's `out=`: the chunked sign exchange posts each range as a message of
    its own and re-assembles the neighbours' messages after the wait.)"""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_mp_choco_worker.py"), comm_op, str(world),
                        str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    _verify_round(comm_op, world, tmp_path)


@pytest.mark.parametrize("comm_op,world", [("compress_top_k", 2), ("sign", 2), ("quantize_qsgd", 2)])
def test_parallel_choco_sync_process_ipc(comm_op, world, tmp_path):
    """ParallelCHOCO's process variant (parallel_choco.py:64-87,95-187): each trainer hands
    its CUDA x / x_hat / memory to a spawned sync process over torch.multiprocessing IPC;
    the sync processes run CHOCOCompressor.pipeline over gloo (comm_device="cpu") on the
    shared tensors; the trainers' own tensors then hold the oracle's x_hat / memory
    (tests/_mp_ipc_worker.py)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_mp_ipc_worker.py"), comm_op, str(world),
                        str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    _verify_round(comm_op, world, tmp_path)


@pytest.mark.parametrize("comm_op,world", [("efsign", 2), ("efsign", 3), ("dgc_top_k", 3)])
def test_centralized_aggregation_across_processes(comm_op, world, tmp_path):
    """EF-signSGD and DGC through CentralizedAggregation across PROCESSES (all-gather over
    gloo, comm_device="cpu"), the aggregator built exactly as the reference builds it
    (ef_sign_sgd.py:41-47, dgc.py:53-59 -> communication.py:138-224); every rank's state is
    checked against the oracle (EF-sign: ef_sign_sgd.py:167-219; DGC: dgc.py:153-252)."""
    import torch
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_mp_choco_worker.py"), comm_op, str(world),
                        str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lens = W.LENS
    nseg = len(lens)
    got = [dict(np.load(tmp_path / f"rank{q}.npz")) for q in range(world)]
    ins = [W.grads_of(q) for q in range(world)]
    if comm_op == "efsign":
        hw = _hdr(nseg)
        for q in range(world):
            g = ins[q][0]
            norms = O.l1_norms(g, lens)
            for rk in range(world):  # every rank received every rank's [norms | words], in rank order
                m = got[rk][f"msg{q}"]
                assert np.array_equal(m[hw:], O.sign_pack(g)), (rk, q)
                assert np.allclose(m[:hw].view(np.float32)[:nseg], norms, rtol=1e-6, atol=0)
        for me in range(world):
            nm_me = got[me][f"msg{me}"][:hw].view(np.float32)[:nseg]
            local = O.sign_local(ins[me][0], nm_me, lens)
            assert same_bits(got[me]["local"], local), me
            want = local.copy()
            for q in range(world):
                if q != me:
                    m = got[me][f"msg{q}"]
                    O.sign_axpy(want, m[hw:], m[:hw].view(np.float32)[:nseg], lens, 1.0, two_roundings=False)
            assert same_bits(got[me]["out"], (want / np.float32(world)).astype(np.float32)), me
        return
    # DGC top-k: every rank's message = top-k of grad + memory; memory <- x * nmask (255 / 254)
    msgs = []
    for q in range(world):
        g, mem, _ = ins[q]
        x = (g + mem).astype(np.float32)
        ov, oi, _ = O.topk_segmented(x, lens, W.RATIO)
        K = ov.size
        for rk in range(world):
            m = got[rk][f"msg{q}"]
            assert same_bits(m[:K].view(np.float32), ov) and np.array_equal(m[K:].astype(np.int64), oi), (rk, q)
        want_mem = (x * np.float32(255.0)).astype(np.float32)
        want_mem[oi] = (ov * np.float32(254.0)).astype(np.float32)
        assert same_bits(got[q]["mem"], want_mem), q
        msgs.append((ov, oi))
    dev = torch.device("cuda", 0)
    for me in range(world):
        acc = np.zeros(sum(lens), dtype=np.float32)
        for ov, oi in msgs:  # empty_grads[q_indices] += q_values, messages in rank order
            acc[oi] = (acc[oi] + ov).astype(np.float32)
        upd = torch.from_numpy(acc).to(dev) / torch.full((), float(world), dtype=torch.float32, device=dev)
        want = torch.from_numpy(ins[me][2]).to(dev).add(upd, alpha=-W.LR).cpu().numpy()
        assert same_bits(got[me]["params"], want), me


@pytest.mark.parametrize("comm_op,world", [("quantize_qsgd_defer", 3), ("sign_defer", 3), ("sign1_defer", 3),
                                           ("sign1_defer", 4)])
def test_deferred_receive_across_processes(comm_op, world, tmp_path):
    """utils.fused_step's deferred receive across PROCESSES (gloo, comm_device="cpu"): every
    rank runs DEFER_STEPS fused CHOCO steps twice from the same state -- receive applied at
    once, then deferred into the next step's first pass and flushed at the end -- and x after
    every step, x_hat and memory must be the same bits (`sign1`: one segment, the
    single-kernel receive; `sign`: six segments, receive + fused pack)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_mp_choco_worker.py"), comm_op, str(world),
                        str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    for q in range(world):
        g = dict(np.load(tmp_path / f"rank{q}.npz"))
        for s in range(W.DEFER_STEPS):
            assert same_bits(g[f"deferred_x{s}"], g[f"now_x{s}"]), (q, s)
        assert same_bits(g["deferred_hat"], g["now_hat"]), q
        assert same_bits(g["deferred_mem"], g["now_mem"]), q
        assert not np.array_equal(g["now_x0"], g[f"now_x{W.DEFER_STEPS - 1}"])  # the steps moved x


def _verify_round(comm_op, world, tmp_path):
    lens, nseg = W.LENS, len(W.LENS)
    n = sum(lens)
    ins = [W.inputs(q) for q in range(world)]
    deltas = [(x - xh).astype(np.float32) for x, xh, _, _ in ins]
    got = [dict(np.load(tmp_path / f"rank{q}.npz")) for q in range(world)]
    # every worker's message, checked once against the oracle (as its neighbours received it)
    msgs = {}
    for q in range(world):
        if comm_op == "quantize_qsgd_chunked":
            # the chunked wire, re-assembled into the one-message layout (each range is a
            # self-contained [level | sign] message of its own elements: checked against the
            # oracle's packing of exactly those elements)
            g = next(g for g in got if f"msg{q}_0" in g)
            d = deltas[q]
            hb = 4 * _hdr(nseg)
            norms = g[f"msg{q}_0"][:hb].view(np.float32)[:nseg]
            assert np.allclose(norms, O.l2_norms(d, lens), rtol=1e-6, atol=0)
            u = O.qsgd_uniforms(n, 1000 + q, 0)
            lvl, off = [], 0
            for s, m in enumerate(lens):
                lvl.append(O.qsgd_levels(d[off:off + m], 15, u[off:off + m], norms[s]))
                off += m
            lvl = np.concatenate(lvl)
            per = -(-(-(-n // W.CHUNKS)) // 8192) * 8192
            for i, e0 in enumerate(range(0, n, per)):
                e1 = min(e0 + per, n)
                assert np.array_equal(g[f"msg{q}_{i + 1}"], O.qsgd_pack(lvl[e0:e1], d[e0:e1], 4)), (q, i)
            levels, neg = O.qsgd_unpack(O.qsgd_pack(lvl, d, 4), n, 4)
            dec, off = [], 0
            for s, m in enumerate(lens):
                dec.append(O.qsgd_decode(levels[off:off + m], neg[off:off + m], norms[s], 15, m))
                off += m
            msgs[q] = np.concatenate(dec)
            continue
        rcv = next(g[f"msg{q}"] for g in got if f"msg{q}" in g)
        d = deltas[q]
        if "top_k" in comm_op or "random_k" in comm_op:
            if "top_k" in comm_op:
                ov, oi, _ = O.topk_segmented(d, lens, W.RATIO)
            else:
                ov, oi = O.randk_segmented(d, lens, W.RATIO, 1000 + q)
            K = ov.size
            assert np.array_equal(rcv[K:].astype(np.int64), oi)
            assert same_bits(rcv[:K].view(np.float32), ov)
            msgs[q] = (ov, oi)
        elif comm_op.startswith("sign"):  # sign_chunked: the same message, posted range by range
            hw = _hdr(nseg)
            norms = rcv[:hw].view(np.float32)[:nseg]
            assert np.array_equal(rcv[hw:], O.sign_pack(d))
            assert np.allclose(norms, O.l1_norms(d, lens), rtol=1e-6, atol=0)
            msgs[q] = (rcv[hw:], norms)
        else:
            hb = 4 * _hdr(nseg)
            norms = rcv[:hb].view(np.float32)[:nseg]
            assert np.allclose(norms, O.l2_norms(d, lens), rtol=1e-6, atol=0)
            u = O.qsgd_uniforms(n, 1000 + q, 0)
            lvl, dec, off = [], [], 0
            for s, m in enumerate(lens):
                lvl.append(O.qsgd_levels(d[off:off + m], 15, u[off:off + m], norms[s]))
                off += m
            assert np.array_equal(rcv[hb:], O.qsgd_pack(np.concatenate(lvl), d, 4))
            levels, neg = O.qsgd_unpack(rcv[hb:], n, 4)
            off = 0
            for s, m in enumerate(lens):
                dec.append(O.qsgd_decode(levels[off:off + m], neg[off:off + m], norms[s], 15, m))
                off += m
            msgs[q] = np.concatenate(dec)
    # every worker's accumulate, in its neighbors_info order
    for rank in range(world):
        _, _, hat, mem = (a.copy() for a in ins[rank])
        nb = _neighborhood(rank, world)
        ranks = list(nb)
        if "top_k" in comm_op or "random_k" in comm_op:
            for q in ranks:
                O.sparse_accumulate(hat if q == rank else None, mem, msgs[q][0], msgs[q][1], nb[q])
        elif comm_op.startswith("sign"):
            O.sign_accumulate(hat, mem, [msgs[q] for q in ranks], [nb[q] for q in ranks], ranks.index(rank), lens)
        else:
            O.qsgd_accumulate(hat, mem, [msgs[q] for q in ranks], [nb[q] for q in ranks], ranks.index(rank))
        assert same_bits(got[rank]["hat"], hat), f"rank {rank} x_hat"
        assert same_bits(got[rank]["mem"], mem), f"rank {rank} memory"
