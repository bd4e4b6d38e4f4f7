"""CPU BASELINE (port) of the reference compressor path -- TEST/BENCH INFRASTRUCTURE ONLY.

The reference never travels to the GPU box, so the CPU baseline that bench.py
times next to the GPU numbers is this restatement of the reference's own torch
op sequences, run with torch on the host cores:
  top-k     : SparsificationCompressor.get_top_k        (sparsification.py:18-31)
  random-k  : SparsificationCompressor.get_random_k     (sparsification.py:40-54)
              + receiver x_hat[idx] += v; memory[idx] += w * v
                                                         (parallel_choco_v.py:307-310)
  QSGD      : QuantizationCompressor.get_qsgd           (sparsification.py:87-98)
              + receiver hat += q; memory += w * q       (parallel_choco_v.py:430-433)
  sign+norm : per-tensor L1 norm + SignCompressor.packing with the bit2byte
              step replaced by torch bit ops            (sparsification.py:129-163,
                                                         parallel_choco_v.py:476-558)
Its outputs are checked against the reference's golden vectors in tests/test_torch_port.py
(top-k sets, QSGD with the reference's draws, sign words, the three decompresses).
Only tests/ and bench.py's cpu_baseline leg may import it.
"""
import torch


def topk_compress(d, ratio):
    x_data = d.view(-1)
    top_k = max(1, int(x_data.nelement() * (1 - ratio)))
    if top_k == 1:
        _, idx = torch.max(x_data.abs(), dim=0, keepdim=True)
    else:
        _, idx = torch.topk(x_data.abs(), top_k, largest=True, sorted=False)
    return x_data[idx], idx


def randk_compress(d, ratio):
    """SparsificationCompressor.get_random_k (sparsification.py:40-54), biased branch."""
    import numpy as np
    x_data = d.view(-1)
    x_len = x_data.nelement()
    top_k = max(1, int(x_len * (1 - ratio)))
    selected_indices = np.random.choice(x_len, top_k, replace=False)
    selected_indices = torch.LongTensor(selected_indices)
    return x_data[selected_indices], selected_indices


def sparse_decompress(hat, mem, values, idx, weight):
    if hat is not None:
        hat[idx] += values
    mem[idx] += weight * values


def qsgd_compress(x, s, is_biased=False):
    norm = x.norm(p=2)
    level_float = s * x.abs() / norm
    previous_level = torch.floor(level_float)
    is_next_level = (torch.rand_like(x) < (level_float - previous_level)).float()
    new_level = previous_level + is_next_level
    scale = 1
    if is_biased:
        d = x.nelement()
        scale = 1.0 / (min(d / (s ** 2), d ** 0.5 / s) + 1.0)
    return scale * torch.sign(x) * norm * new_level / s


def dense_decompress(hat, mem, q, weight):
    if hat is not None:
        hat += q
    mem += weight * q


_SHIFTS = None


def sign_compress(d):
    """sign + L1 norm + (32, N') packing with torch ops in place of bit2byte."""
    global _SHIFTS
    norm = d.norm(p=1)
    s = torch.sign(d).view(-1)
    n = s.numel()
    pad = (32 - n % 32) % 32
    s = torch.cat([s, torch.zeros(pad, dtype=s.dtype)]).view(32, -1).to(torch.int32)
    if _SHIFTS is None:
        _SHIFTS = torch.arange(32, dtype=torch.int64).view(32, 1)
    words = ((s == -1).to(torch.int64) << _SHIFTS).sum(dim=0)  # uint32 value held in int64
    return words, norm


def sign_decompress(hat, mem, words, norm, n, weight):
    w = words.view(1, -1)
    bits = (w >> torch.arange(32, dtype=torch.int64).view(32, 1)) & 1
    sign = (1 - 2 * bits).view(-1)[:n].float()
    upd = norm / n * sign
    if hat is not None:
        hat.add_(upd)
    mem.add_(upd, alpha=weight)


def gossip_step(x, mem, hat, gamma):
    """optim/utils.py:70-72 (update_params_from_neighbor), as torch ops."""
    x.add_(gamma * (mem - hat))
    return x
