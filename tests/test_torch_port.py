"""Pin oracle/torch_port.py -- the torch-CPU op sequence bench.py times as the CPU
baseline -- against the golden vectors the reference itself produced
(tests/golden/gen_golden.py).  CPU only: the baseline is a faithful restatement, not an
unpinned one."""
import numpy as np
import pytest
import torch

from conftest import golden, same_bits
from oracle import choco_oracle as O
from oracle import torch_port as P

TOPK_CASES = ["topk_n1000_r09", "topk_n65536_r099", "topk_n262144_r099", "topk_n30011_r09", "topk_n50_k1"]


@pytest.mark.parametrize("name", TOPK_CASES)
def test_port_topk_set(name):
    """get_top_k (sparsification.py:18-31): same index set, values gathered from d."""
    g = golden(name)
    d = torch.from_numpy(g["x"] - g["xhat"] if "xhat" in g else g["x"]).float()
    vals, idx = P.topk_compress(d, float(g["ratio"]))
    order = np.argsort(idx.numpy())
    ref = np.argsort(g["indices"])
    assert np.array_equal(idx.numpy()[order], g["indices"][ref])
    assert same_bits(vals.numpy()[order], g["values"][ref])


@pytest.mark.parametrize("name", ["qsgd_n32771_q4", "qsgd_n32771_q4_biased", "qsgd_n4099_q2", "qsgd_n4099_q8",
                                  "qsgd_n257_q4_small"])
def test_port_qsgd_with_reference_draws(name, monkeypatch):
    """get_qsgd (sparsification.py:87-98) with the reference's own torch.rand_like draws
    replayed: bit-exact."""
    g = golden(name)
    u = torch.from_numpy(g["u"])
    monkeypatch.setattr(torch, "rand_like", lambda x, *a, **k: u.clone())
    out = P.qsgd_compress(torch.from_numpy(g["x"]), 2 ** int(g["q"]) - 1, is_biased=bool(g["biased"]))
    assert same_bits(out.numpy(), g["out"])


@pytest.mark.parametrize("name", ["sign_n31", "sign_n4096", "sign_n40003_pad"])
def test_port_sign_words_and_decode(name):
    """SignCompressor.packing / unpacking (sparsification.py:129-163) with the repo's bit
    convention: words equal the fixture's, the decode equals the reference's +-1."""
    g = golden(name)
    x = torch.from_numpy(g["x"])
    words, norm = P.sign_compress(x)
    assert np.array_equal(words.numpy().astype(np.uint32), g["packed"].view(np.uint32))
    n = x.numel()
    mem = torch.zeros(n)
    P.sign_decompress(None, mem, words, torch.tensor(float(n)), n, 1.0)  # norm / n = 1: the bare signs
    assert same_bits(mem.numpy(), g["decoded"])
    assert norm.item() == x.norm(p=1).item()


def test_port_sign_accumulate_matches_oracle():
    """One segment: hat.add_(upd), mem.add_(upd, alpha=w) (parallel_choco_v.py:549-558) --
    the oracle's pinned sign_accumulate on the same message."""
    g = golden("sign_n40003_pad")
    x = torch.from_numpy(g["x"])
    n = x.numel()
    words, norm = P.sign_compress(x)
    rng = np.random.default_rng(3)
    hat0, mem0 = rng.standard_normal(n).astype(np.float32), rng.standard_normal(n).astype(np.float32)
    hat, mem = torch.from_numpy(hat0.copy()), torch.from_numpy(mem0.copy())
    P.sign_decompress(hat, mem, words, norm, n, 1.0 / 3)
    oh, om = hat0.copy(), mem0.copy()
    O.sign_accumulate(oh, om, [(g["packed"], np.array([norm.item()], dtype=np.float32))], [1.0 / 3], 0, [n])
    assert same_bits(hat.numpy(), oh)
    assert same_bits(mem.numpy(), om)


@pytest.mark.parametrize("name", ["choco_topk_mini_r09", "choco_topk_mini_r099"])
def test_port_sparse_decompress(name):
    """x_hat[idx] += v; memory[idx] += w * v (parallel_choco_v.py:307-310) over the
    reference's three messages -> its x_hat / memory, bit-exact."""
    g = golden(name)
    lens = g["layout"].tolist()
    ks = g["selected_shapes"].tolist()
    hat, mem = torch.from_numpy(g["hat0"].copy()), torch.from_numpy(g["mem0"].copy())
    s = int(g["self_rank"])
    for r in range(3):
        msg = g[f"msg{r}"]
        K = msg.size // 2
        glob = msg[K:].astype(np.int64) + np.repeat(np.cumsum([0] + lens[:-1]), ks)
        P.sparse_decompress(hat if r == s else None, mem, torch.from_numpy(msg[:K].copy()),
                            torch.from_numpy(glob), float(g["weights"][r]))
    assert same_bits(hat.numpy(), g["hat1"])
    assert same_bits(mem.numpy(), g["mem1"])


def test_port_dense_decompress():
    """hat += q; memory += w * q (parallel_choco_v.py:430-433) over the reference's three
    dense QSGD messages -> its x_hat / memory, bit-exact."""
    g = golden("choco_qsgd_mini_q4")
    hat, mem = torch.from_numpy(g["hat0"].copy()), torch.from_numpy(g["mem0"].copy())
    s = int(g["self_rank"])
    for r in range(3):
        P.dense_decompress(hat if r == s else None, mem, torch.from_numpy(g[f"msg{r}"]), float(g["weights"][r]))
    assert same_bits(hat.numpy(), g["hat1"])
    assert same_bits(mem.numpy(), g["mem1"])


def test_port_gossip_step():
    g = golden("gossip_n10007")
    x = torch.from_numpy(g["x"].copy())
    P.gossip_step(x, torch.from_numpy(g["mem"]), torch.from_numpy(g["hat"]), float(g["gamma"]))
    assert same_bits(x.numpy(), g["out"])
