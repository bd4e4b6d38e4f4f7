"""Drop-in for dl_code/pcode/utils/sparsification.py (the reference's compressor primitives).

Same class names, method names, argument meaning and return types as the
reference; every compute call goes to the HIP codec (codec.py -> libchoco_codec.so).

Deliberate differences (all documented in DESIGN.md):
  * top-k output order: ascending index (the reference's torch.topk(sorted=False)
    order is implementation-defined, sparsification.py:28-30); the selected SET is
    identical for tie-free inputs; ties at the k-th magnitude go to the lowest
    index (what the reference's k == 1 path, torch.max, does).
  * random-k indices are a uniform k-subset drawn on the device (a seeded bijection
    gives the per-tile counts and the in-tile positions, include/choco_codec.h)
    instead of the host's numpy RandomState (sparsification.py:48); the seed is taken
    from torch's default generator, so torch.manual_seed makes runs reproducible.
  * QSGD uniforms come from in-kernel xoroshiro128+ streams (seeded by SplitMix64,
    include/choco_codec.h) instead of
    torch.rand_like (sparsification.py:91); norms are fp64-accumulated (the
    reference's fp32 CPU norm drifts by up to 1e-2 relative at 1e8 elements).
  * host (CPU) tensors are accepted as the reference accepts them (BASELINE cfg 1 runs
    the sign compressor on CPU tensors): they are staged to the current ROCm device,
    computed there by the same kernels and the results returned on the input's device.
    Nothing is computed on the host.
"""
import math

import numpy as np
import torch

from . import codec


def get_n_bits(tensor):
    """8 * numel * element_size  (sparsification.py:10-11)."""
    return 8 * tensor.nelement() * tensor.element_size()


def _draw_seed():
    return int(torch.randint(0, 2**62, (1,)).item())


def _on_device(t):
    """(device tensor, the device results go back to): host tensors are staged to the
    current ROCm device (the compute never runs on the host)."""
    if t.is_cuda:
        return t, None
    return t.to(torch.device("cuda", torch.cuda.current_device())), t.device


def _home(t, home):
    return t if home is None else t.to(home)


class SparsificationCompressor(object):
    """top-k / random-k  (sparsification.py:17-83)."""

    def get_top_k(self, x, ratio):
        x, home = _on_device(x)
        x_data = x.view(-1)
        top_k = codec.topk_k(x_data.nelement(), ratio)
        values, indices = codec.topk(x_data, top_k)
        return _home(values, home), _home(indices.long(), home)

    def get_mask(self, flatten_arr, indices):
        # identical torch ops to sparsification.py:33-38 (including ~ on uint8)
        mask = torch.zeros_like(flatten_arr)
        mask[indices] = 1
        mask = mask.byte()
        return mask.float(), (~mask).float()

    def get_random_k(self, x, ratio, is_biased=True):
        x, home = _on_device(x)
        x_data = x.view(-1)
        top_k = codec.topk_k(x_data.nelement(), ratio)
        values, indices = codec.randk(x_data, top_k, _draw_seed(), is_biased=is_biased)
        return _home(values, home), _home(indices.long(), home)

    def compress(self, arr, op, compress_ratio, is_biased):
        if "top_k" in op:
            values, indices = self.get_top_k(arr, compress_ratio)
        elif "random_k" in op:
            # the reference never forwards is_biased here (sparsification.py:60)
            values, indices = self.get_random_k(arr, compress_ratio)
        else:
            raise NotImplementedError
        return values, indices

    def uncompress(self, values, indices, selected_shapes, original_shapes):
        """Local -> global indices with EXACT integer offsets (the reference adds in fp32)."""
        counts = [int(c) for c in selected_shapes]
        offsets, pointer = [], 0
        for i in range(len(counts)):
            offsets.append(pointer)
            pointer += int(original_shapes[i][1])
        total = sum(counts)
        dev = indices.device
        off = torch.repeat_interleave(torch.tensor(offsets, dtype=torch.int64, device=dev),
                                      torch.tensor(counts, dtype=torch.int64, device=dev))
        idx = indices[:total].long() + off
        return values[:total], idx


class QuantizationCompressor(object):
    """QSGD random quantization  (sparsification.py:86-123)."""

    def get_qsgd(self, x, s, is_biased=False):
        if not codec.is_pow2_minus1(int(s)):
            raise RuntimeError(f"QSGD level count s={s} must be 2^q - 1 with 1 <= q <= 16")
        q = int(round(math.log2(int(s) + 1)))
        xd, home = _on_device(x)
        x_flat = xd.reshape(-1).contiguous()
        _, _, dense = codec.qsgd_compress(x_flat, q, is_biased=is_biased, seed=_draw_seed(), want_dense=True)
        return _home(dense.view_as(xd), home)

    def qsgd_quantize_numpy(self, x, s, is_biased=False):
        """numpy in / numpy out; computed on the current ROCm device."""
        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
        return self.get_qsgd(t, s, is_biased).numpy()

    def compress(self, arr, op, quantize_level, is_biased):
        if quantize_level != 32:
            s = 2 ** quantize_level - 1
            values = self.get_qsgd(arr, s, is_biased)
        else:
            values = arr
        return values

    def uncompress(self, arr):
        return arr


class SignCompressor(object):
    """1-bit sign packing in the reference's (32, N') layout  (sparsification.py:126-194)."""

    def packing(self, src_tensor):
        size = src_tensor.size()
        src, home = _on_device(src_tensor)
        packed, _ = codec.sign_compress(src.reshape(-1).contiguous(), want_norms=False)
        return _home(packed, home), size

    def unpacking(self, src_tensor, src_tensor_size):
        n = self.element_num(src_tensor_size)
        src, home = _on_device(src_tensor)
        out = codec.sign_unpack(src.int().contiguous(), n)
        return _home(out.view(src_tensor_size), home)

    def majority_vote(self, src_tensor_list):
        """Per (row, word) majority of the voters' decoded signs; a tie encodes as "+"."""
        n = 32 * src_tensor_list[0].numel()
        home = None if src_tensor_list[0].is_cuda else src_tensor_list[0].device
        total = None
        for t in src_tensor_list:
            t, _ = _on_device(t)
            dec = codec.sign_unpack(t.int().contiguous(), n)
            total = dec if total is None else total + dec
        packed, _ = codec.sign_compress(total, want_norms=False)
        return _home(packed, home)

    def element_num(self, size):
        num = 1
        for i in range(len(size)):
            num *= size[i]
        return num

    def compress(self, src_tensor):
        return self.packing(src_tensor)

    def uncompress(self, src_tensor, src_tensor_size):
        return self.unpacking(src_tensor, src_tensor_size)
