"""GPU parity: top-k / random-k / sparse accumulate through the C ABI vs the oracle
and the reference's golden vectors.  Run on an MI355X with `pytest -m gpu`."""
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


TOPK_CASES = ["topk_n1000_r09", "topk_n65536_r099", "topk_n262144_r099", "topk_n30011_r09", "topk_n50_k1",
              "topk_k1_tie", "topk_ties_n4096_r09"]


@pytest.mark.parametrize("name", TOPK_CASES)
def test_topk_golden(name):
    from chocosgd_amd import codec
    g = golden(name)
    k = int(g["k"])
    x = dev(g["x"])
    xh = dev(g["xhat"]) if "xhat" in g else None
    vals, idx = codec.topk(x, k, xhat=xh)
    torch.cuda.synchronize()
    d = (g["x"] - g["xhat"]).astype(np.float32) if "xhat" in g else g["x"]
    ov, oi = O.topk(d, k)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)
    if "ties" not in name:
        assert np.array_equal(np.sort(g["indices"]), oi)  # the reference's own set


@pytest.mark.parametrize("n", [1, 2, 7, 100, 4097, 65536, 65537, 100003, 1 << 20, 3_000_001, 25_000_000])
@pytest.mark.parametrize("ratio", [0.99, 0.9, 0.5])
def test_topk_random_sizes(n, ratio):
    from chocosgd_amd import codec
    x = randn(n, 1000 + n % 997)
    k = codec.topk_k(n, ratio)
    assert k == O.topk_k(n, ratio)
    vals, idx = codec.topk(x, k)
    ov, oi = O.topk(host(x), k)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)


def test_topk_fused_delta():
    """d = x - xhat formed inside the kernel vs the oracle's top-k of the host delta."""
    from chocosgd_amd import codec
    x, xh = randn(2_000_003, 5), randn(2_000_003, 6, 0.9)
    k = codec.topk_k(x.numel(), 0.99)
    v1, i1 = codec.topk(x, k, xhat=xh)
    ov, oi = O.topk(host(x) - host(xh), k)
    assert np.array_equal(host(i1).astype(np.int64), oi)
    assert same_bits(host(v1), ov)


@pytest.mark.parametrize("n", [2_000_003, 100_003])
def test_topk_k_equals_n_large(n):
    """ratio 0 (k = n): a multi-workgroup copy with iota indices."""
    from chocosgd_amd import codec
    x, xh = randn(n, 8), randn(n, 9)
    vals, idx = codec.topk(x, n, xhat=xh)
    assert np.array_equal(host(idx), np.arange(n, dtype=np.int32))
    assert same_bits(host(vals), host(x) - host(xh))


def test_topk_unaligned_base_pipeline():
    """A 3M-element view starting 1 and 3 floats past a 16-byte boundary runs the
    multi-workgroup pipeline (dword-aligned buffer loads)."""
    from chocosgd_amd import codec
    base, bh = randn(3_000_010, 13), randn(3_000_010, 14, 0.5)
    for off in (1, 3):
        x, xh = base[off:off + 3_000_000], bh[off:off + 3_000_000]
        k = codec.topk_k(x.numel(), 0.99)
        vals, idx = codec.topk(x, k, xhat=xh)
        ov, oi = O.topk(host(x) - host(xh), k)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)


@pytest.mark.slow
def test_topk_100M_bench_shape():
    from chocosgd_amd import codec
    n = 100_000_000
    x = randn(n, 1000)
    k = codec.topk_k(n, 0.99)
    vals, idx = codec.topk(x, k)
    ov, oi = O.topk(host(x), k)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)


@pytest.mark.parametrize("kind", ["ties", "clustered", "zeros", "tiny_k", "k_equals_n", "nan"])
def test_topk_fallback_and_edge_inputs(kind):
    """Inputs that defeat the sampled threshold (heavy ties, values hidden between sample
    chunks, all-zero tails) must still give the exact canonical answer."""
    from chocosgd_amd import codec
    n = 4_000_000
    g = torch.Generator(device=DEV).manual_seed(77)
    if kind == "ties":
        x = torch.round(torch.randn(n, generator=g, device=DEV) * 4) / 4
    elif kind == "clustered":
        x = torch.zeros(n, device=DEV)
        x[1_000_003:1_006_003] = torch.randn(6000, generator=g, device=DEV) + 10
    elif kind == "zeros":
        x = torch.zeros(n, device=DEV)
        x[::1000] = 1.0
    elif kind == "tiny_k":
        x = torch.randn(n, generator=g, device=DEV)
    elif kind == "k_equals_n":
        x = torch.randn(100_000, generator=g, device=DEV)
    else:
        x = torch.randn(n, generator=g, device=DEV)
        x[12345] = float("nan")
    ratio = {"tiny_k": 0.999999, "k_equals_n": 0.0}.get(kind, 0.99)
    k = codec.topk_k(x.numel(), ratio)
    vals, idx = codec.topk(x.contiguous(), k)
    ov, oi = O.topk(host(x), k)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)


@pytest.mark.parametrize("kind", ["ties", "all_equal", "zeros_xhat"])
def test_topk_wide_fallback_100M(kind):
    """The exact fallback at BASELINE size (every K34 workgroup on the ticketed radix
    select, csrc/topk.hip wide_fallback): tie clusters, an all-equal buffer (side
    lists overflow), and x == x_hat on most elements (exact zeros), bit-exact against
    the oracle; run twice so the queue's self-reset is exercised."""
    from chocosgd_amd import codec
    n = 100_000_000
    g = torch.Generator(device=DEV).manual_seed(91)
    xh = None
    if kind == "ties":
        x = torch.round(torch.randn(n, generator=g, device=DEV) * 8) / 8
    elif kind == "all_equal":
        x = torch.full((n,), 0.5, device=DEV)
    else:
        x = torch.randn(n, generator=g, device=DEV)
        xh = x.clone()
        xh[::97] += 1.0  # d = 0 except every 97th element (-1)
    k = codec.topk_k(n, 0.99)
    d = host(x) if xh is None else (host(x) - host(xh)).astype(np.float32)
    ov, oi = O.topk(d, k)
    for _ in range(2):
        vals, idx = codec.topk(x, k, xhat=xh)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)


def test_topk_wide_fallback_under_concurrent_load():
    """The exact fallback's bounded waits (csrc/topk.hip wave0_poll_ge, CHOCO_POLL_BUDGET)
    while a second stream keeps every CU busy with long streaming kernels (as RCCL or the
    training step would share the chip): the tie-heavy 100M input still gives the exact
    answer, no status bit is raised, and the load was still running when the call ended."""
    from chocosgd_amd import codec
    n = 100_000_000
    g = torch.Generator(device=DEV).manual_seed(93)
    x = torch.round(torch.randn(n, generator=g, device=DEV) * 8) / 8
    k = codec.topk_k(n, 0.99)
    ov, oi = O.topk(host(x), k)
    before = codec.topk_fallback_count()
    big = torch.ones(1 << 29, device=DEV)  # 2 GiB: ~1 ms per pass
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        for _ in range(60):
            big.mul_(1.0000001)
        done = torch.cuda.Event()
        done.record(side)
    vals, idx = codec.topk(x, k)
    torch.cuda.current_stream().synchronize()
    overlapped = not done.query()
    torch.cuda.synchronize()
    codec.check_topk_status(wait=True)  # raises on a poll that gave up
    assert codec.topk_fallback_count() > before  # the exact fallback ran
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)
    assert overlapped, "the load finished before the top-k call: nothing was shared"


@pytest.mark.parametrize("layout", ["resnet20_cifar10", "resnet50_imagenet"])
@pytest.mark.parametrize("ratio", [0.9, 0.99])
def test_topk_segmented_model_layouts(layout, ratio):
    from chocosgd_amd import codec
    lens = golden_json("layouts.json")[layout]
    n = sum(lens)
    x, xh = randn(n, 11), randn(n, 12, 0.5)
    plan = codec.SegmentPlan(lens, ratio, x.device)
    vals, idx = codec.topk_segmented(x, plan, xhat=xh)
    ov, oi, ks = O.topk_segmented(host(x) - host(xh), lens, ratio)
    assert plan.k_per_seg == ks
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)


UNALIGNED_LAYOUT = [3, 70_001, 5, 1_200_003, 17, 300, 1_048_577, 2]


@pytest.mark.parametrize("ratio", [0.9, 0.99])
def test_topk_segmented_unaligned_large(ratio):
    """Segments over 64K and over 1M elements that start off a 16-byte boundary."""
    from chocosgd_amd import codec
    lens = UNALIGNED_LAYOUT
    n = sum(lens)
    x, xh = randn(n, 41), randn(n, 42, 0.5)
    plan = codec.SegmentPlan(lens, ratio, x.device)
    vals, idx = codec.topk_segmented(x, plan, xhat=xh)
    ov, oi, ks = O.topk_segmented(host(x) - host(xh), lens, ratio)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)


@pytest.mark.parametrize("case", ["ties", "ties_many_tiles", "ratio0", "ratio05", "nan", "tile_edges", "huge_mixed"])
def test_topk_segmented_edge_layouts(case):
    """The batched segmented select (topk_seg.hip) on tie-heavy tensors, k = len, k = len/2,
    NaN, tensors at tile edges (16384 +- 1, exactly 1024 tiles) and a tensor over 16M
    elements that takes the flat pipeline next to batched ones.  ties_many_tiles: the tie
    quota of a 306-tile tensor is split over tiles past the first 256 (S4 sums the
    earlier tiles' counts four per thread)."""
    from chocosgd_amd import codec
    ratio = {"ratio0": 0.0, "ratio05": 0.5}.get(case, 0.99)
    if case == "tile_edges":
        lens = [16383, 16384, 16385, 1, 16_777_216, 32768]
    elif case == "huge_mixed":
        lens = [7, 20_000_001, 3000, 1_100_001]
    elif case == "ties_many_tiles":
        lens = [5_000_003, 16384, 9]
    else:
        lens = [100, 50_000, 16384, 16385, 3, 700_001]
    n = sum(lens)
    x, xh = randn(n, 61), randn(n, 62, 0.5)
    if case in ("ties", "ties_many_tiles"):
        x = torch.round(x * 2) / 2
        xh = torch.zeros_like(x)
    if case == "nan":
        x[[5, 60_000, 90_000]] = float("nan")
    plan = codec.SegmentPlan(lens, ratio, x.device)
    vals, idx = codec.topk_segmented(x, plan, xhat=xh)
    ov, oi, ks = O.topk_segmented(host(x) - host(xh), lens, ratio)
    assert plan.k_per_seg == ks
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)


def test_topk_segmented_repeat_calls_self_clean():
    """Workspace histograms are reset by every call: repeated calls on new data stay exact."""
    from chocosgd_amd import codec
    layouts = [golden_json("layouts.json")["resnet20_cifar10"], UNALIGNED_LAYOUT]
    plans = [codec.SegmentPlan(lens, r, torch.device(DEV)) for lens, r in zip(layouts, (0.9, 0.99))]
    for seed in range(4):  # two plans interleaved, each on new data
        lens, plan = layouts[seed % 2], plans[seed % 2]
        x = randn(sum(lens), 70 + seed)
        vals, idx = codec.topk_segmented(x, plan)
        ov, oi, _ = O.topk_segmented(host(x), lens, (0.9, 0.99)[seed % 2])
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)
        codec.topk(x, codec.topk_k(x.numel(), 0.99))  # the flat path's workspace is separate


@pytest.mark.parametrize("layout", ["unaligned", "resnet20_cifar10"])
@pytest.mark.parametrize("is_biased", [True, False])
def test_randk_segmented_vs_oracle(layout, is_biased):
    from chocosgd_amd import codec
    lens = UNALIGNED_LAYOUT if layout == "unaligned" else golden_json("layouts.json")[layout]
    n = sum(lens)
    x, xh = randn(n, 51), randn(n, 52, 0.5)
    seed = 0xDEADBEEF12345
    plan = codec.SegmentPlan(lens, 0.95, x.device)
    vals, idx = codec.randk_segmented(x, plan, seed, is_biased=is_biased, xhat=xh)
    ov, oi = O.randk_segmented(host(x) - host(xh), lens, 0.95, seed, is_biased=is_biased)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)


@pytest.mark.parametrize("n", [1, 2, 1000, 65536, 100003, 262144, 262145, 2_000_003])
@pytest.mark.parametrize("seed", [1, 2 ** 40 + 3])
def test_randk_matches_sampler_oracle(n, seed):
    """The direct sampler (csrc/randk.hip) against its restatement: single- and multi-tile
    (2^18) draws, exact tile edges."""
    from chocosgd_amd import codec
    x = randn(n, 3)
    k = codec.topk_k(n, 0.95)
    vals, idx = codec.randk(x, k, seed)
    oi = O.randk_indices(n, k, seed)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), host(x)[oi])
    vu, iu = codec.randk(x, k, seed, is_biased=False)
    assert torch.equal(iu, idx)
    assert same_bits(host(vu), O.gather(host(x), oi, n, k, is_biased=False))


def test_gather_golden():
    from chocosgd_amd import codec
    g = golden("randk_n20000_r095")
    x = dev(g["x"])
    n, k = g["x"].size, O.topk_k(g["x"].size, float(g["ratio"]))
    out = codec.gather(x, dev(g["idx_biased"].astype(np.int64)))
    assert same_bits(host(out), g["vals_biased"])
    out = codec.gather(x, dev(g["idx_unbiased"].astype(np.int64)), scale=float(np.float32(n / k)))
    assert same_bits(host(out), g["vals_unbiased"])


@pytest.mark.parametrize("name,ratio", [("choco_topk_mini_r09", 0.9), ("choco_topk_mini_r099", 0.99)])
def test_choco_topk_round_trip_golden(name, ratio):
    """Per-tensor top-k of 3 workers -> accumulate into x_hat_1 / memory: bit-exact vs the reference."""
    from chocosgd_amd import codec
    g = golden(name)
    lens = g["layout"].tolist()
    self_rank = int(g["self_rank"])
    hat, mem = dev(g["hat0"]), dev(g["mem0"])
    plan = codec.SegmentPlan(lens, ratio, torch.device(DEV))
    for r in range(3):
        vals, idx = codec.topk_segmented(dev(g["x"][r]), plan, xhat=dev(g["xhat"][r]))
        codec.sparse_accumulate(vals, idx, mem, float(g["weights"][r]), xhat_self=hat if r == self_rank else None)
    assert same_bits(host(hat), g["hat1"])
    assert same_bits(host(mem), g["mem1"])


def test_release_workspaces_then_recompute():
    """codec.release_workspaces frees the cached scratch; the next call allocates a fresh
    zeroed one and gives the same exact answer."""
    from chocosgd_amd import codec
    d = randn(3_000_000, 77)
    k = codec.topk_k(d.numel(), 0.99)
    v1, i1 = codec.topk(d, k)
    torch.cuda.synchronize()
    assert codec.workspace_bytes() > 0
    codec.release_workspaces()
    assert codec.workspace_bytes() == 0
    v2, i2 = codec.topk(d, k)
    torch.cuda.synchronize()
    assert torch.equal(i1, i2) and torch.equal(v1.view(torch.int32), v2.view(torch.int32))
    ov, oi = O.topk(host(d), k)
    assert np.array_equal(host(i2).astype(np.int64), oi)


def test_dropped_plan_frees_its_workspace():
    """A SegmentPlan that is garbage-collected takes its device workspaces with it (the
    status registry holds addresses, not tensors) and the codec's host-side state keyed
    by them; a new plan afterwards (possibly at the same address) starts cold and exact
    (plans built per layout leaked their workspaces)."""
    import gc
    from chocosgd_amd import codec
    lens = [300_000, 7, 1_200_000, 4096, 50_000]
    x = randn(sum(lens), 91)
    torch.cuda.synchronize()
    gc.collect()
    base = torch.cuda.memory_allocated()
    for rep in range(3):
        plan = codec.SegmentPlan(lens, 0.99, x.device)
        for _ in range(2):  # cold, then warm (the miss flag is allocated)
            vals, idx = codec.topk_segmented(x, plan)
        torch.cuda.synchronize()
        assert torch.cuda.memory_allocated() > base
        ov, oi, ks = O.topk_segmented(host(x), lens, 0.99)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)
        del plan, vals, idx
        gc.collect()
        torch.cuda.synchronize()
        assert torch.cuda.memory_allocated() <= base, (rep, torch.cuda.memory_allocated(), base)


def _check_topk(x, k, xh=None):
    from chocosgd_amd import codec
    vals, idx = codec.topk(x, k, xhat=xh)
    d = host(x) if xh is None else (host(x) - host(xh)).astype(np.float32)
    ov, oi = O.topk(d, k)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)
    return vals, idx


@pytest.mark.parametrize("n", [3_000_000, 25_000_000])
def test_topk_warm_start_badly_wrong_windows(n):
    """Warm start (include/choco_codec.h): consecutive calls with the same (n, k) on one
    workspace select inside the window the previous call left.  Every call stays exact,
    including those whose window is badly wrong: the buffer scaled x100, then all zeros,
    then random again, x1e-3, a tie-heavy buffer, a constant buffer, and random."""
    from chocosgd_amd import codec
    k = codec.topk_k(n, 0.99)
    g = torch.Generator(device=DEV).manual_seed(400)
    seq = [randn(n, 401), randn(n, 402), randn(n, 403) * 100, torch.zeros(n, device=DEV), randn(n, 404),
           randn(n, 405) * 1e-3, torch.round(torch.randn(n, generator=g, device=DEV) * 4) / 4,
           torch.full((n,), -2.5, device=DEV), randn(n, 406), randn(n, 407)]
    for x in seq:
        _check_topk(x, k)


def test_topk_warm_start_drift_and_cold_equal():
    """A slowly drifting delta (the CHOCO case: scale shrinks 3 % per call) stays exact on
    the warm path, and the warm and cold (workspace reset / warm start off) answers agree."""
    from chocosgd_amd import codec, _lib
    n = 4_000_037
    k = codec.topk_k(n, 0.99)
    base = randn(n, 410)
    for step in range(12):
        x = base * (0.97 ** step) + randn(n, 411 + step, 0.05)
        _check_topk(x, k)
    lib = _lib.load()
    x = randn(n, 430)
    v_w, i_w = codec.topk(x, k)
    lib.choco_topk_set_warm_start(0)
    try:
        v_c, i_c = codec.topk(x, k)
    finally:
        lib.choco_topk_set_warm_start(1)
    assert torch.equal(i_w, i_c) and torch.equal(v_w.view(torch.int32), v_c.view(torch.int32))


def test_topk_warm_start_alternating_shapes():
    """Calls of different (n, k) on the shared workspace alternate: each is cold (the window
    is keyed by (n, k)), then warm again; all exact."""
    from chocosgd_amd import codec
    for i in range(6):
        n = (2_000_003, 3_000_017)[i % 2]
        ratio = (0.99, 0.9)[(i // 2) % 2]
        _check_topk(randn(n, 440 + i), codec.topk_k(n, ratio))


def test_topk_warm_start_gossip_sequence():
    """The fused consensus step on the warm path: x, memory, x_hat evolve over calls."""
    from chocosgd_amd import codec
    n = 3_000_011
    k = codec.topk_k(n, 0.99)
    g = torch.Generator(device=DEV).manual_seed(450)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    for step in range(5):
        xa = O.gossip_step(host(x), host(mem), host(hat), 0.9)
        d = (xa - host(hat)).astype(np.float32)
        vals, idx = codec.topk(x, k, xhat=hat, gossip=(mem, 0.9))
        assert same_bits(host(x), xa)
        ov, oi = O.topk(d, k)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)
        codec.sparse_accumulate(vals, idx, mem, 1.0, xhat_self=hat)


def _ws_word(off):
    from chocosgd_amd import codec
    return codec.topk_workspace_word(off)


def test_topk_fused_gossip_cold_run_takes_host_k1():
    """Deterministic check of the round-5 race fix: a fused-gossip
    call on a workspace that a warm miss put on a cold run must take its window from the
    host-launched sample kernel (K1), never from K2's own prologue sample (K2 rewrites x
    while it streams).  At 25M: (1) a cold fused call; (2) a warm fused call whose delta is
    1000x larger, so the carried window misses (exact fallback, cold run started and
    mirrored to the host); (3) a fused call on the cold run: K1 runs (profile count), K2's
    sample counter does not move, the output is exact.  Then (4) the same cold run WITHOUT
    the fused step samples inside K2 (the counter moves), so the counter is live."""
    from chocosgd_amd import _lib, codec
    n = 25_000_000
    k = codec.topk_k(n, 0.99)
    torch.cuda.synchronize()
    codec.release_workspaces()
    g = torch.Generator(device=DEV).manual_seed(4711)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)

    def fused_call(xx, mm, hh, expect_k1):
        xa = O.gossip_step(host(xx), host(mm), host(hh), 0.9)
        d = (xa - host(hh)).astype(np.float32)
        codec.profile_reset()
        codec.profile_enable(True)
        vals, idx = codec.topk(xx, k, xhat=hh, gossip=(mm, 0.9))
        torch.cuda.synchronize()
        codec.profile_enable(False)
        assert codec.profile_read("topk_bounds")[1] == (1 if expect_k1 else 0)
        assert same_bits(host(xx), xa)
        ov, oi = O.topk(d, k)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)

    fused_call(x, mem, hat, expect_k1=True)                       # (1) cold: K1
    s0 = _ws_word(_lib.TOPK_K2_SAMPLES_OFFSET)
    f0 = _ws_word(_lib.TOPK_FALLBACKS_OFFSET)
    mem.mul_(1000.0)
    fused_call(x, mem, hat, expect_k1=False)                      # (2) warm window, misses
    assert _ws_word(_lib.TOPK_FALLBACKS_OFFSET) == f0 + 1
    assert _ws_word(_lib.TOPK_COLD_LEFT_OFFSET) >= 64             # the cold run (K34's backoff)
    fused_call(x, mem, hat, expect_k1=True)                       # (3) cold run, fused: host K1
    assert _ws_word(_lib.TOPK_K2_SAMPLES_OFFSET) == s0            # K2 never sampled
    # (4) the same cold run without the fused step: K2 samples its own window
    vals, idx = codec.topk(x, k, xhat=hat)
    torch.cuda.synchronize()
    assert _ws_word(_lib.TOPK_K2_SAMPLES_OFFSET) == s0 + 1
    ov, oi = O.topk((host(x) - host(hat)).astype(np.float32), k)
    assert np.array_equal(host(idx).astype(np.int64), oi)


def test_topk_warm_start_drained_delta():
    """The CHOCO drain: x fixed, x_hat catching up with every call's top-k (the selected
    entries of the delta become 0), so every call's k-th key is the previous call's ~2k-th.
    Every call exact; the first warm miss puts the workspace on a cold run (K34's backoff:
    the window is sampled in K2's prologue), so no later call takes the exact fallback."""
    from chocosgd_amd import codec
    n = 4_000_037
    k = codec.topk_k(n, 0.99)
    torch.cuda.synchronize()
    codec.release_workspaces()  # a fresh workspace: cold first call, counter at 0
    d = randn(n, 470)
    counts = []
    for step in range(12):
        vals, idx = _check_topk(d, k)
        d[idx.long()] = 0.0
        counts.append(codec.topk_fallback_count())
    assert counts[-1] <= 1, counts


def test_topk_status_word_clean_after_calls():
    """No call of this module left the workspace status word set (bounded waits never gave up)."""
    from chocosgd_amd import codec
    _check_topk(randn(2_000_003, 460), codec.topk_k(2_000_003, 0.99))
    codec.check_topk_status(wait=True)


@pytest.mark.parametrize("case", ["offsets", "k1", "all", "xhat_unaligned"])
def test_randk_sampler_cases(case):
    """(seed, offset) streams, k = 1, k = n (every index), and x - xhat on an unaligned view."""
    from chocosgd_amd import codec
    n = 1_000_003
    if case == "offsets":
        x = randn(n, 31)
        k = codec.topk_k(n, 0.99)
        seen = []
        for off in (0, 1, 2):
            vals, idx = codec.randk(x, k, 77, offset=off)
            oi = O.randk_indices(n, k, 77, off)
            assert np.array_equal(host(idx).astype(np.int64), oi)
            assert same_bits(host(vals), host(x)[oi])
            seen.append(oi)
        assert not np.array_equal(seen[0], seen[1])
    elif case in ("k1", "all"):
        x = randn(n, 32)
        k = 1 if case == "k1" else n
        vals, idx = codec.randk(x, k, 5, is_biased=False)
        oi = O.randk_indices(n, k, 5)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), O.gather(host(x), oi, n, k, is_biased=False))
    else:
        base, bh = randn(n + 3, 33), randn(n + 3, 34)
        x, xh = base[3:], bh[1:n + 1]
        k = codec.topk_k(n, 0.9)
        vals, idx = codec.randk(x, k, 6, xhat=xh)
        oi = O.randk_indices(n, k, 6)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), (host(x) - host(xh))[oi])


@pytest.mark.slow
def test_randk_100M_bench_shape():
    """BASELINE cfg-4 shape (100M, k = 1M): 382 tiles, the count pass and the per-tile draws."""
    from chocosgd_amd import codec
    n = 100_000_000
    x = randn(n, 1000)
    k = codec.topk_k(n, 0.99)
    vals, idx = codec.randk(x, k, 12345, offset=3)
    oi = O.randk_indices(n, k, 12345, 3)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), host(x)[oi])


def _check_seg(x, plan, lens, ratio, xh=None):
    from chocosgd_amd import codec
    vals, idx = codec.topk_segmented(x, plan, xhat=xh)
    d = host(x) if xh is None else (host(x) - host(xh)).astype(np.float32)
    ov, oi, _ = O.topk_segmented(d, lens, ratio)
    assert np.array_equal(host(idx).astype(np.int64), oi)
    assert same_bits(host(vals), ov)
    return vals, idx


@pytest.mark.parametrize("layout", ["resnet20_cifar10", "resnet50_imagenet", "edges"])
def test_topk_segmented_warm_sequence(layout):
    """Warm segmented calls (one read: each segment's window from the previous call):
    drifting data, then windows that are badly wrong -- x100, all zeros (k_s-th key 0),
    tie-heavy, x1e-3, back to random -- every call exact (a missed segment is selected
    exactly by its tile workgroups together in S4w, which re-centres its window)."""
    from chocosgd_amd import codec
    lens = ([16383, 16384, 16385, 1, 3, 700_001, 32768, 2_500_007] if layout == "edges"
            else golden_json("layouts.json")[layout])
    n = sum(lens)
    ratio = 0.99
    plan = codec.SegmentPlan(lens, ratio, torch.device(DEV))
    base = randn(n, 500)
    g = torch.Generator(device=DEV).manual_seed(501)
    seq = [base, base * 0.98 + randn(n, 502, 0.05), base * 0.95 + randn(n, 503, 0.05), randn(n, 504) * 100,
           torch.zeros(n, device=DEV), torch.round(torch.randn(n, generator=g, device=DEV) * 4) / 4,
           randn(n, 505) * 1e-3, randn(n, 506), randn(n, 507)]
    for x in seq:
        _check_seg(x, plan, lens, ratio)


def test_topk_segmented_warm_drained_delta():
    """The drain on the segmented path (ResNet-50's layout): the selected entries of every
    call are zeroed before the next.  Every call exact; the first call whose windows miss
    (S4w's shared exact select) raises the miss flag, an isolated miss stays warm, and the
    second one within kSegMissGap calls sends the host to the cold sequence (S1 + S2) for a
    run of calls: no later window misses (each call here is synchronised, so each flag is
    seen at the very next call)."""
    from chocosgd_amd import codec
    lens = golden_json("layouts.json")["resnet50_imagenet"]
    n = sum(lens)
    ratio = 0.99
    plan = codec.SegmentPlan(lens, ratio, torch.device(DEV))
    d = randn(n, 540)
    counts = []
    for step in range(10):
        vals, idx = _check_seg(d, plan, lens, ratio)
        d[idx.long()] = 0.0
        counts.append(codec.topk_fallback_count(plan=plan))
    assert counts[-1] == counts[2], counts


def test_topk_segmented_warm_miss_shared_select_max_segment():
    """A missed window in the largest batched segment (1024 tiles, kSegBatchMax elements):
    its 1024 tile workgroups select it together in S4w (wide.h, the segment's own queue;
    phase 4's offsets sum up to 1023 earlier tiles over 256 threads) -- T far above the
    window (x100), far below it (x1e-3), tie clusters (the kept-key lists overflow), all
    exact, each queue reset for the next miss."""
    from chocosgd_amd import codec
    lens = [16384 * 1024, 16385, 5]
    n = sum(lens)
    ratio = 0.99
    plan = codec.SegmentPlan(lens, ratio, torch.device(DEV))
    base = randn(n, 570)
    g = torch.Generator(device=DEV).manual_seed(571)
    ties = torch.round(torch.randn(n, generator=g, device=DEV) * 8) / 8
    misses = []
    # (each call is synchronised here: an isolated miss stays warm, a second one within 32
    # calls starts a cold run that ends after one call whose prepared window would have held)
    for x in (base, base, base * 100, base * 100, base * 100, base * 1e-3, base * 1e-3, base * 1e-3, ties, ties,
              base):
        _check_seg(x, plan, lens, ratio)
        misses.append(codec.topk_fallback_count(plan=plan))
    assert misses[-1] > misses[1], misses  # the shared select ran
    codec.check_topk_status(wait=True)


def test_topk_segmented_gossip_warm_miss():
    """The consensus step fused into W2 and then a missed window (the delta x100 in one
    warm step): S4w's shared select reads x_new as W2 left it; x and the selection exact."""
    from chocosgd_amd import codec
    lens = golden_json("layouts.json")["resnet50_imagenet"]
    n = sum(lens)
    plan = codec.SegmentPlan(lens, 0.99, torch.device(DEV))
    g = torch.Generator(device=DEV).manual_seed(580)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    prev_clean, before, checked = False, None, False
    for step in range(12):
        s1 = codec.launch_count("topk_seg_hist")  # the cold sequence's first launch
        m0 = codec.topk_fallback_count(plan=plan)
        jump = prev_clean and before is None  # after a warm call without a miss the host stays warm
        if jump:
            x = hat + 100.0 * (x - hat)
            before = m0
        xa = O.gossip_step(host(x), host(mem), host(hat), 0.9)
        vals, idx = codec.topk_segmented(x, plan, xhat=hat, gossip=(mem, 0.9))
        assert same_bits(host(x), xa)
        ov, oi, _ = O.topk_segmented((xa - host(hat)).astype(np.float32), lens, 0.99)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)
        warm = codec.launch_count("topk_seg_hist") == s1
        if jump:
            assert warm and codec.topk_fallback_count(plan=plan) > before  # warm, and its windows missed
            checked = True
        prev_clean = warm and codec.topk_fallback_count(plan=plan) == m0
        codec.sparse_accumulate(vals, idx, mem, 1.0, xhat_self=hat)
    assert checked
    codec.check_topk_status(wait=True)


def test_topk_segmented_warm_ratio0_and_half():
    """k_s = len_s (every element) and k_s = len_s / 2 on the warm path."""
    from chocosgd_amd import codec
    lens = [100, 50_000, 16384, 16385, 3, 700_001]
    n = sum(lens)
    for ratio in (0.0, 0.5):
        plan = codec.SegmentPlan(lens, ratio, torch.device(DEV))
        for i in range(3):
            _check_seg(randn(n, 510 + i), plan, lens, ratio, xh=randn(n, 520 + i, 0.5))


def test_topk_segmented_gossip_warm_sequence():
    """The consensus step fused into the warm path's single read (S2) over several steps."""
    from chocosgd_amd import codec
    lens = golden_json("layouts.json")["resnet20_cifar10"] + [1_100_003]
    n = sum(lens)
    plan = codec.SegmentPlan(lens, 0.99, torch.device(DEV))
    g = torch.Generator(device=DEV).manual_seed(530)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    for step in range(4):
        xa = O.gossip_step(host(x), host(mem), host(hat), 0.9)
        vals, idx = codec.topk_segmented(x, plan, xhat=hat, gossip=(mem, 0.9))
        assert same_bits(host(x), xa)
        ov, oi, _ = O.topk_segmented((xa - host(hat)).astype(np.float32), lens, 0.99)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)
        codec.sparse_accumulate(vals, idx, mem, 1.0, xhat_self=hat)


def test_topk_segmented_warm_bin_list_overflow():
    """Warm calls on tie-heavy tensors (values on a 1/8 grid): the k-th key's window bin holds
    thousands of equal keys, more than the bin list takes (topk_seg.hip kListCap), so the
    segment is selected exactly in S4w -- every call exact, and not counted as a window
    miss (the window itself holds T)."""
    from chocosgd_amd import codec
    lens = [1_000_000, 500_000, 40_000, 33]
    n = sum(lens)
    plan = codec.SegmentPlan(lens, 0.99, torch.device(DEV))
    counts = []
    for step in range(5):
        g = torch.Generator(device=DEV).manual_seed(560 + step)
        x = torch.round(torch.randn(n, generator=g, device=DEV) * 8) / 8
        _check_seg(x, plan, lens, 0.99)
        counts.append(codec.topk_fallback_count(plan=plan))
    assert counts[-1] == counts[1], counts


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_topk_segmented_warm_random_layouts(seed):
    """Random layouts (single-tile and multi-tile tensors, tile-edge lengths) through a run of
    warm calls whose data changes in kind -- drift, a sign flip, a few huge entries, a block
    of zeros, quantised values (ties at the k-th key), a tensor made all equal -- every call
    exact against the oracle (the warm tail's kept keys, their tie counts, the overflow and
    missed-window paths)."""
    from chocosgd_amd import codec
    rng = np.random.default_rng(seed)
    lens = [int(v) for v in rng.choice([1, 7, 300, 16383, 16384, 16385, 40_000, 131_072, 250_001], size=9)]
    lens += [int(rng.integers(20_000, 600_000))]
    n = sum(lens)
    ratio = float(rng.choice([0.9, 0.99, 0.999]))
    plan = codec.SegmentPlan(lens, ratio, torch.device(DEV))
    base = randn(n, seed)
    seq = [base, base * 0.97 + randn(n, seed + 1, 0.05), -base]
    spikes = base.clone()
    spikes[torch.from_numpy(rng.choice(n, 50, replace=False)).to(DEV)] = 1e6
    seq.append(spikes)
    zeros = base.clone()
    zeros[: n // 3] = 0.0
    seq.append(zeros)
    seq.append(torch.round(base * 8) / 8)
    flat = base.clone()
    off = int(np.sum(lens[:-1]))
    flat[off:] = 0.25  # the last tensor all equal: every key ties at T
    seq.append(flat)
    seq.append(randn(n, seed + 2))
    for x in seq:
        _check_seg(x, plan, lens, ratio)
        _check_seg(x, plan, lens, ratio, xh=randn(n, seed + 3, 0.01))


def _ties_data(n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.round(torch.randn(n, generator=g, device=DEV) * 4096) / 4096  # ~100 ties per value near T


@pytest.mark.parametrize("n", [16_777_216, 16_789_561, 33_554_431, 100_000_000])
@pytest.mark.parametrize("ratio", [0.99, 0.985])
@pytest.mark.parametrize("kind", ["randn", "ties", "xhat"])
def test_topk_large_exact_cold_and_warm(n, ratio, kind):
    """The flat pipeline from 2^24 (a partial last chunk and tile at 2^24 + 12345, 2^25 - 1)
    to the north-star 100M, at k = 1 % and 1.5 %, on Gaussian data, on tie-heavy data (the
    k-th value shared by ~100 elements: ties split inside one tile), and on a delta
    x - x_hat; a cold call then a warm call, bit-exact against the oracle."""
    from chocosgd_amd import codec
    k = codec.topk_k(n, ratio)
    x = _ties_data(n, 61) if kind == "ties" else randn(n, 62)
    xh = randn(n, 63, 0.5) if kind == "xhat" else None
    d = host(x) if xh is None else (host(x) - host(xh)).astype(np.float32)
    ov, oi = O.topk(d, k)
    for _ in range(2):  # cold, then warm
        vals, idx = codec.topk(x, k, xhat=xh)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)


def test_topk_gossip_and_drain_20m():
    """The fused consensus step over a warm sequence at 20M (x, memory, x_hat evolve; every
    call exact, x_new bit-identical), then the CHOCO drain on a fixed delta (every call's
    k-th key moves: windows miss, the exact fallback and the cold run)."""
    from chocosgd_amd import codec
    n = 20_000_003
    k = codec.topk_k(n, 0.99)
    torch.cuda.synchronize()
    codec.release_workspaces()
    g = torch.Generator(device=DEV).manual_seed(64)
    x = torch.randn(n, generator=g, device=DEV)
    hat = x + 0.1 * torch.randn(n, generator=g, device=DEV)
    mem = hat + 0.05 * torch.randn(n, generator=g, device=DEV)
    for step in range(4):
        xa = O.gossip_step(host(x), host(mem), host(hat), 0.9)
        d = (xa - host(hat)).astype(np.float32)
        vals, idx = codec.topk(x, k, xhat=hat, gossip=(mem, 0.9))
        assert same_bits(host(x), xa)
        ov, oi = O.topk(d, k)
        assert np.array_equal(host(idx).astype(np.int64), oi)
        assert same_bits(host(vals), ov)
        codec.sparse_accumulate(vals, idx, mem, 1.0, xhat_self=hat)
    dd = randn(n, 65)
    for step in range(5):
        vals, idx = _check_topk(dd, k)
        dd[idx.long()] = 0.0
