"""C-ABI surface and host-side logic (no GPU needed: only host-only entry points are called)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, golden, golden_json
from oracle import choco_oracle as O

HEADER = os.path.join(ROOT, "include", "choco_codec.h")


def _header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|size_t)\s+(choco_[a-z0-9_]+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    from chocosgd_amd import _lib
    return _lib.load()


def test_library_exports_every_header_symbol(lib):
    from chocosgd_amd import _lib
    syms = _header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes table and header disagree"
    assert lib.choco_version() == 1


def test_exported_symbols_are_exactly_the_abi():
    import subprocess
    so = os.path.join(ROOT, "chocosgd_amd", "lib", "libchoco_codec.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True).stdout
    exported = sorted(l.split()[-1] for l in out.splitlines() if " T " in l and l.split()[-1].startswith("choco_"))
    assert exported == _header_symbols()


def test_topk_k_rule_matches_reference_table(lib):
    for n, ratio, k in golden_json("k_table.json"):
        assert lib.choco_topk_k(n, ratio) == k, (n, ratio)


def test_sizes_and_formats(lib):
    for n in [1, 31, 32, 33, 1_000_000, 345_000_000]:
        assert lib.choco_sign_words(n) == O.sign_words(n)
    for n in [1, 7, 8, 100003, 100_000_000]:
        for q in [1, 2, 3, 4, 5, 8, 9, 16]:
            cw = O.container_bits(q)
            assert lib.choco_qsgd_packed_bytes(n, q) == O.plane_bytes(n, cw) + O.plane_bytes(n, 1)
    assert lib.choco_qsgd_packed_bytes(10, 32) == 0
    # candidate entries (float4 + int32 per 4 elements) dominate: 5 bytes per element
    assert lib.choco_topk_workspace_size(100_000_000) > 5 * 100_000_000
    assert lib.choco_topk_workspace_size(1000) >= 256
    assert lib.choco_sign_workspace_size(161) >= 256 + 8 * 161 * 8  # 8 replicas of the per-segment sums


def test_sign_receive_workspace_sizes(lib):
    """choco_sign_recv_workspace_size: the accumulators plus bit planes of every message and of
    the output (n/8 bytes each, 32 x ceil(N'/32) words), growing with n, nseg and nmsg; past
    2^30 elements the two-kernel form's sign workspace."""
    for n in [1, 33, 4096 * 32 + 1, 345_000_000]:
        P = (O.sign_words(n) + 31) // 32
        for nseg in [1, 161]:
            for nmsg in [1, 3, 8]:
                sz = lib.choco_sign_recv_workspace_size(n, nseg, nmsg)
                assert sz >= 256 + 8 * nseg * 8 + (nmsg + 1) * 32 * P * 4
                assert sz % 256 == 0
                assert lib.choco_sign_recv_workspace_size(n, nseg, nmsg + 1) > sz
    assert lib.choco_sign_recv_workspace_size(1 << 30, 5, 3) == lib.choco_sign_workspace_size(5)


def test_segmented_plan(lib):
    from chocosgd_amd import _lib
    lens = golden_json("layouts.json")["resnet50_imagenet"]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    p_off, keep = _lib.i64_array(offs.tolist())
    plen = lib.choco_topk_segmented_plan_len(p_off, len(lens))
    tiles = [(m + 16383) // 16384 for m in lens]  # every ResNet-50 tensor is batched (< 16M)
    rk = [(m + (1 << 18) - 1) >> 18 for m in lens]  # random-k tiles of 2^18 (csrc/randk.hip)
    base = 8 * len(lens) + sum(tiles) + len(lens)
    assert plen == base + 1 + 4 * sum(rk) + 4 * sum(tiles) + 8 * sum(tiles)
    plan = (ctypes.c_int64 * plen)()
    total = lib.choco_topk_segmented_plan(p_off, len(lens), 0.99,
                                          ctypes.cast(plan, ctypes.POINTER(ctypes.c_int64)))
    flat = np.array(list(plan))
    rows = flat[:8 * len(lens)].reshape(-1, 8)
    ks = [O.topk_k(m, 0.99) for m in lens]
    assert total == sum(ks)
    assert rows[:, 0].tolist() == offs[:-1].tolist()
    assert rows[:, 1].tolist() == lens
    assert rows[:, 2].tolist() == ks
    assert rows[:, 3].tolist() == np.concatenate([[0], np.cumsum(ks)[:-1]]).tolist()
    assert rows[:, 4].tolist() == np.concatenate([[0], np.cumsum(tiles)[:-1]]).tolist()
    assert rows[:, 5].tolist() == tiles
    assert rows[0, 6] == sum(tiles) and rows[0, 7] == len(lens)
    tmap = flat[8 * len(lens):8 * len(lens) + sum(tiles)]
    assert tmap.tolist() == np.repeat(np.arange(len(lens)), tiles).tolist()
    assert flat[8 * len(lens) + sum(tiles):base].tolist() == list(range(len(lens)))
    # the random-k tile table: [R] then {segment, tile in segment, first tile, tiles}
    assert flat[base] == sum(rk)
    tab = flat[base + 1:base + 1 + 4 * sum(rk)].reshape(-1, 4)
    first = np.concatenate([[0], np.cumsum(rk)[:-1]])
    assert tab[:, 0].tolist() == np.repeat(np.arange(len(lens)), rk).tolist()
    assert tab[:, 1].tolist() == [t for m in rk for t in range(m)]
    assert tab[:, 2].tolist() == np.repeat(first, rk).tolist()
    assert tab[:, 3].tolist() == np.repeat(rk, rk).tolist()
    # the collect launch's dispatch order, {tile, segment, first element, length} per
    # workgroup: the tiles of single-tile segments, then the rest
    ob = base + 1 + 4 * sum(rk)
    order = flat[ob:ob + 4 * sum(tiles)].reshape(-1, 4)
    t0 = np.concatenate([[0], np.cumsum(tiles)[:-1]])
    segs = [s for s in range(len(lens)) if tiles[s] == 1] + [s for s in range(len(lens)) if tiles[s] > 1]
    exp = [(int(t0[s]) + t, s, int(offs[s]) + t * 16384, min(16384, lens[s] - t * 16384))
           for s in segs for t in range(tiles[s])]
    assert [tuple(r) for r in order.tolist()] == exp
    # per tile (tile-id order): its segment's row and the segment id
    trows = flat[ob + 4 * sum(tiles):].reshape(-1, 8)
    seg_of_tile = np.repeat(np.arange(len(lens)), tiles)
    assert np.array_equal(trows[:, :6], rows[seg_of_tile, :6])
    assert trows[:, 6].tolist() == seg_of_tile.tolist()
    # a segment over 16M elements is routed to the flat pipeline (no top-k tiles)
    big = np.array([0, 5, 5 + 20_000_000], dtype=np.int64)
    pb, keep2 = _lib.i64_array(big.tolist())
    assert lib.choco_topk_segmented_plan_len(pb, 2) == 16 + 1 + 1 + 1 + 4 * (1 + 77) + 4 + 8
    assert lib.choco_topk_segmented_plan(pb, 2, 1.5, None) < 0  # ratio outside [0, 1)


def test_error_reporting(lib):
    from chocosgd_amd import _lib
    rc = lib.choco_topk_compress(None, None, 10, 1, None, None, None, 0, None)
    assert rc == -1
    assert "null" in _lib.last_error()
    with pytest.raises(RuntimeError):
        _lib.check(rc, "choco_topk_compress")


def test_cpu_tensors_are_rejected_loudly():
    """The codec takes device tensors only; the reference-named primitives stage host
    tensors to the ROCm device -- with no device they raise (no host computation)."""
    from chocosgd_amd import codec, sparsification
    x = torch.randn(100)
    with pytest.raises(RuntimeError, match="ROCm device"):
        codec.topk(x, 5)
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError):
            sparsification.SparsificationCompressor().get_top_k(x, 0.9)
        with pytest.raises(RuntimeError):
            sparsification.SignCompressor().packing(x)


def test_uncompress_exact_integer_offsets():
    """SparsificationCompressor.uncompress: global index = local + segment start, in int64
    (the reference adds in fp32 and is wrong above 2^24, sparsification.py:76)."""
    from chocosgd_amd.sparsification import SparsificationCompressor
    c = SparsificationCompressor()
    big = 2 ** 24 + 5
    shapes = [(torch.Size([big]), big), (torch.Size([10]), 10)]
    values = torch.tensor([1.0, 2.0, 3.0])
    local = torch.tensor([big - 1, 3, 9], dtype=torch.int64)
    v, idx = c.uncompress(values, local, [1, 2], shapes)
    assert idx.tolist() == [big - 1, big + 3, big + 9]
    assert torch.equal(v, values)


def test_tensor_buffer_keeps_dtype():
    from chocosgd_amd.tensor_buffer import TensorBuffer
    ints = [torch.tensor([16777217, 3], dtype=torch.int64), torch.tensor([5], dtype=torch.int64)]
    tb = TensorBuffer(ints)
    assert tb.buffer.dtype == torch.int64 and tb.buffer.tolist() == [16777217, 3, 5]
    assert tb[1].tolist() == [5] and len(tb) == 2
    flat = torch.arange(6, dtype=torch.float32)
    tb2 = TensorBuffer.from_flat(flat, [(2, 2), (2,)])
    assert tb2[0].shape == (2, 2) and tb2[1].tolist() == [4.0, 5.0]


def test_neighborhood_matches_reference_topologies():
    from chocosgd_amd.communication import neighborhood
    assert neighborhood(0, 1) == {0: 1.0}
    assert neighborhood(1, 2) == {0: 0.5, 1: 0.5}
    assert neighborhood(0, 8) == {0: 1 / 3, 1: 1 / 3, 7: 1 / 3}
    assert list(neighborhood(1, 3).keys()) == [0, 1, 2]
    g = golden("choco_topk_mini_r09")
    assert list(neighborhood(1, 3).values()) == g["weights"].tolist()


def test_get_n_bits():
    from chocosgd_amd.sparsification import get_n_bits
    assert get_n_bits(torch.zeros(10, dtype=torch.float32)) == 320
    assert get_n_bits(torch.zeros(10, dtype=torch.int32)) == 320


@pytest.mark.parametrize("n", [1, 31, 32 * 1024, 32 * 1024 + 1, 1_000_007, 345_000_000])
@pytest.mark.parametrize("chunks", [1, 2, 3, 7, 64])
def test_chunked_wire_ranges(n, chunks):
    """The chunked exchanges' ranges (host side): they tile the buffer in order, starts on
    the kernels' alignment (QSGD: 8192 elements; sign: 1024 words), at most `chunks` of them."""
    from chocosgd_amd import codec
    for ranges, end, align in ((codec.qsgd_chunks(n, chunks), n, codec.QSGD_RANGE_ALIGN),
                               (codec.sign_chunks(n, chunks), codec.sign_words(n), codec.SIGN_RANGE_ALIGN)):
        assert 1 <= len(ranges) <= chunks
        assert ranges[0][0] == 0 and ranges[-1][1] == end
        for (a0, a1), (b0, _) in zip(ranges, ranges[1:]):
            assert a1 == b0
        for a0, a1 in ranges:
            assert a0 < a1 and a0 % align == 0 and (a1 % align == 0 or a1 == end)
