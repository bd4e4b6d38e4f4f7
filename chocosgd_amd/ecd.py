"""Drop-in for the ECD-PSGD compressor (dl_code/pcode/optim/ecd_psgd.py:186-455).

`ECDCompressor(aggregator=, comm_op=, comm_device=, compress_ratio=,
quantize_level=, is_biased=, backend=, use_ipc=)` with `.compress(sync_buffer)`
(input key `flatten_updated_params`: the extrapolated model, compressed as is),
`.sync(sync_buffer)` and `.uncompress(sync_buffer, neighbor_hat_params,
local_index)`, which extrapolates every neighbour replica with that neighbour's
message: hat <- (1 - 2/t) hat + (2/t) q  (t = local_index), in the reference's
rounding (mul, then torch's fused add with alpha; the sign receiver folds 2/t
into the per-tensor scale first, ecd_psgd.py:448-454).  Receivers are the
*_extrapolate kernels of include/choco_codec.h.
"""
import torch

from . import codec
from .communication import recover_device
from .dcd import _ConsumerBase
from .tensor_buffer import TensorBuffer


class ECDCompressor(object):
    def __init__(self, **kargs):
        if "top_k" in kargs["comm_op"] or "random_k" in kargs["comm_op"]:
            self.compressor_fn = ECDSparsificationCompressor(**kargs)
        elif "quantize" in kargs["comm_op"]:
            self.compressor_fn = ECDQuantizationCompressor(**kargs)
        elif "sign" in kargs["comm_op"]:
            self.compressor_fn = ECDSignCompressor(**kargs)
        else:
            raise NotImplementedError

    def compress(self, *args, **kargs):
        return self.compressor_fn.compress(*args, **kargs)

    def sync(self, *args, **kargs):
        return self.compressor_fn.sync(*args, **kargs)

    def uncompress(self, *args, **kargs):
        return self.compressor_fn.uncompress(*args, **kargs)


def _coeffs(local_index):
    # Python doubles, rounded to fp32 where torch applies them to fp32 tensors
    return 1 - 2 / local_index, 2 / local_index


class _ECDBase(_ConsumerBase):
    def _x(self, sync_buffer):
        x = sync_buffer["flatten_updated_params"].buffer
        return x, self._layout(sync_buffer, x.device)


class ECDSparsificationCompressor(_ECDBase):
    """top-k / random-k  (ecd_psgd.py:211-303)."""

    def __init__(self, *args, **kargs):
        super().__init__(*args, **kargs)
        self._guards = {}

    def compress(self, sync_buffer):
        x, lay = self._x(sync_buffer)
        self._sparse_message(sync_buffer, x, None, lay)

    def sync(self, sync_buffer):
        message = sync_buffer["wire_message"]
        sync_buffer["synced_message"] = self._send(message)
        sync_buffer["sycned_message_size"] = len(message)

    def uncompress(self, sync_buffer, neighbor_hat_params, local_index):
        K = int(sync_buffer["sycned_message_size"] / 2)
        a, b = _coeffs(local_index)
        for rank, hat_params in neighbor_hat_params.items():
            dev = hat_params.buffer.device
            guard = self._guards.get(dev)
            if guard is None:
                guard = self._guards[dev] = codec.IndexGuard(dev)
            msg = recover_device(sync_buffer["synced_message"][rank], device=dev)
            codec.sparse_extrapolate(msg[:K].view(torch.float32), msg[K:], hat_params.buffer, a, b, guard=guard)
        for guard in self._guards.values():  # bad indices of an earlier step, after this step's work
            guard.check_then_arm()


class ECDQuantizationCompressor(_ECDBase):
    """QSGD  (ecd_psgd.py:306-423)."""

    def compress(self, sync_buffer):
        x, lay = self._x(sync_buffer)
        self._qsgd_message(sync_buffer, x, None, lay)

    def sync(self, sync_buffer):
        sync_buffer["synced_message"] = self._send(sync_buffer["flatten_updates"].buffer)

    def uncompress(self, sync_buffer, neighbor_hat_params, local_index):
        q = int(self.quantize_level)
        a, b = _coeffs(local_index)
        for rank, hat_params in neighbor_hat_params.items():
            dev = hat_params.buffer.device
            lay = self._layout(sync_buffer, dev)
            msg = recover_device(sync_buffer["synced_message"][rank], device=dev)
            if q == 32:
                hat_params.buffer.mul_(a).add_(msg.view(torch.float32), alpha=b)
                continue
            packed, norms = self._qsgd_part(msg, lay)
            codec.qsgd_extrapolate(packed, norms, lay.n, q, hat_params.buffer, a, b, is_biased=self.is_biased,
                                   seg_off=lay.seg_off, nseg=lay.nseg)


class ECDSignCompressor(_ECDBase):
    """sign + per-tensor L1 norm  (ecd_psgd.py:426-455); one [norms | words] message,
    `synced_flatten_norms` / `synced_signs` are views of it."""

    def compress(self, sync_buffer):
        x, lay = self._x(sync_buffer)
        signs, norms = self._sign_message(sync_buffer, x, None, lay)
        sync_buffer["flatten_norms"] = TensorBuffer.from_flat(norms, [() for _ in range(lay.nseg)])
        sync_buffer["flatten_updates"] = None

    def sync(self, sync_buffer):
        norms = sync_buffer["flatten_norms"].buffer
        synced = self._send(self._sign_wire(sync_buffer))
        sync_buffer["synced_message"] = synced
        sync_buffer["synced_flatten_norms"], sync_buffer["synced_signs"] = self._sign_parts(synced, norms.numel())

    def uncompress(self, sync_buffer, neighbor_hat_params, local_index):
        a, b = _coeffs(local_index)
        for rank, hat_params in neighbor_hat_params.items():
            dev = hat_params.buffer.device
            lay = self._layout(sync_buffer, dev)
            nm = recover_device(sync_buffer["synced_flatten_norms"][rank], device=dev).contiguous()
            sg = recover_device(sync_buffer["synced_signs"][rank], device=dev)
            codec.sign_extrapolate(sg, nm, lay.n, hat_params.buffer, a, b, seg_off=lay.seg_off, nseg=lay.nseg)
