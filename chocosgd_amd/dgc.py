"""The communication half of DGC (dl_code/pcode/optim/dgc.py:153-252, with
compress_or_quantize at :327-343): error-feedback top-k / random-k of every
gradient tensor, an all-gather of the [values | indices] messages and the
averaged sparse update -- or, for a quantize op, the QSGD dense floats all-reduced.

`DGCCodec(world_aggregator, comm_op, comm_device, n_nodes, quantize_level=, is_biased=,
strict_reference=True)` keeps the reference's three steps as methods:
  * `compress(grads, memory_tb, compress_ratio)` -> (values, indices, n_bits):
    _grad = grad + memory per tensor, top-k of _grad, memory <- `_grad * nmask`
    (dgc.py:174-176).  The reference's nmask is `(~mask.byte()).float()`
    (sparsification.py:33-38): a bitwise NOT of uint8 under the PyTorch this
    runs on, i.e. 255 for unselected and 254 for selected entries, and
    `strict_reference=True` (the default) reproduces exactly that, bit for bit.
    `strict_reference=False` applies the evident intent instead (1 - mask, what `~`
    gave for a ByteTensor in PyTorch <= 1.1: the selected entries zeroed, the rest
    kept).  The error-feedback memory is ONE flat TensorBuffer (the reference keeps a
    dict of per-parameter vectors) so the whole layout is one batched launch;
    `indices` are GLOBAL int32.  For a quantize op the reference leaves memory alone
    (dgc.py:183-185): _grad = grad + memory is a temporary;
  * `sync(values, indices)` -> (synced_message, message_size);
  * `recover_info(flatten_params, synced_message, message_size, lr)` -> params - lr *
    (sum of messages) / n_nodes.
The momentum-factor masking of dgc.py:175-179 (`mask_momentum`) is optimizer state and
is NOT applied here, in either mode: `last_indices` holds the selected global indices the
optimizer needs for it.

strict_reference=True multiplies the unselected memory by 255 every step, so the memory
overflows to inf after ~16 steps and DGC top-k / random-k diverges -- as the reference
does on the PyTorch it runs on; a one-time warning says so.
"""
import warnings

import torch

from . import codec
from .communication import recover_device
from .parallel_choco import _Layout
from .sparsification import _draw_seed, get_n_bits
from .tensor_buffer import flatten


_warned = []


def _warn_strict_once():
    if not _warned:
        _warned.append(True)
        warnings.warn("DGCCodec(strict_reference=True) reproduces the reference's nmask = "
                      "(~mask.byte()).float() = 255 / 254 (sparsification.py:33-38): the error-feedback "
                      "memory grows 255x per step and overflows after ~16 steps; pass "
                      "strict_reference=False for the intended 1 - mask", RuntimeWarning, stacklevel=3)


class DGCCodec(object):
    def __init__(self, world_aggregator, comm_op, comm_device, n_nodes, quantize_level=None, is_biased=False,
                 strict_reference=True):
        self.strict_reference = strict_reference
        self.world_aggregator = world_aggregator
        self.comm_op = comm_op
        self.comm_device = comm_device
        self.n_nodes = n_nodes
        self.quantize_level = quantize_level
        self.is_biased = is_biased
        self.is_compress_op = "compress" in comm_op
        self.selected_shapes = None
        self.last_indices = None
        if strict_reference and "compress" in comm_op:
            _warn_strict_once()

    def compress(self, grads, memory_tb, compress_ratio):
        memory = memory_tb.buffer
        lens = tuple(int(g.nelement()) for g in grads)
        lay = _Layout.get(lens, memory.device)
        if self.is_compress_op:
            x = memory
            x.add_(flatten(grads))  # _grad = grad + memory (dgc.py:157; fp32 add commutes), in place
            plan = lay.topk_plan(float(compress_ratio))
            if "top_k" in self.comm_op:
                values, indices = codec.topk_segmented(x, plan)
            elif "random_k" in self.comm_op:
                values, indices = codec.randk_segmented(x, plan, _draw_seed(), is_biased=True)
            else:
                raise NotImplementedError
            if self.strict_reference:
                # _grad * nmask with nmask = (~mask.byte()).float(): 255 unselected, 254 selected
                x.mul_(255.0)
                x.index_put_((indices.long(),), values * 254.0)
            else:
                # _grad * (1 - mask): the selected entries (values == x[idx]) become 0
                codec.sparse_accumulate(torch.neg(values), indices, x, 1.0)
            self.selected_shapes = list(plan.k_per_seg)
            self.last_indices = indices
            # nominal bits as compress_or_quantize counts them (dgc.py:335-337): fp32 values and
            # the int64 indices torch.topk returns (the wire here carries int32)
            return values, indices, 32 * values.numel() + 64 * indices.numel()
        if "quantize" in self.comm_op:
            x = memory + flatten(grads)  # _grad: a temporary, memory keeps its value (dgc.py:183-185)
            q = int(self.quantize_level)
            if q == 32:
                dense = x.clone()
            else:
                _, _, dense = codec.qsgd_compress(x, q, is_biased=self.is_biased, seg_off=lay.seg_off, nseg=lay.nseg,
                                                  seed=_draw_seed(), want_dense=True)
            self.selected_shapes = list(lens)
            return dense, None, get_n_bits(dense) * q / 32
        raise NotImplementedError

    def sync(self, selected_values, selected_indices):
        if self.is_compress_op:
            message = torch.cat([selected_values.view(torch.int32), selected_indices])
            if self.comm_device == "cpu":
                message = message.cpu().pin_memory()
            synced = self.world_aggregator._agg(message, communication_scheme="all_gather")
        else:
            message = selected_values
            if self.comm_device == "cpu":
                message = message.cpu().pin_memory()
            synced = self.world_aggregator._agg(message, op="sum", communication_scheme="all_reduce")
        return synced, len(message)

    def recover_info(self, flatten_params, synced_message, message_size, lr):
        if self.is_compress_op:
            K = int(message_size / 2)
            grads = torch.zeros_like(flatten_params)
            for message in synced_message:
                m = recover_device(message, device=flatten_params.device)
                # empty_grads[q_indices] += q_values  (dgc.py:234-242), messages in rank order
                codec.sparse_accumulate(m[:K].view(torch.float32), m[K:], grads, 1.0)
            update = grads
        else:
            update = recover_device(synced_message, device=flatten_params.device)
        # true division by n_nodes (a device 0-dim divisor: torch turns a CPU-scalar division
        # into a reciprocal multiply on the GPU), then params.add(-lr, update) (dgc.py:244-249)
        update = update / torch.full((), float(self.n_nodes), dtype=torch.float32, device=flatten_params.device)
        return flatten_params.add(update, alpha=-lr)
