"""Drop-in for the DeepSqueeze compressor (dl_code/pcode/optim/deep_squeeze.py:133-489).

`DeepSqueezeCompressor(aggregator=, rank=, comm_op=, comm_device=, compress_ratio=,
quantize_level=, is_biased=, backend=, use_ipc=, consensus_stepsize=)`:
  * `.compress(sync_buffer)` compresses the error-compensated memory
    `sync_buffer["params_tb"]` and RETURNS the local compressed copy (the
    decoded message as this rank sees it) as a TensorBuffer -- the caller's
    error feedback is `memory - local` (deep_squeeze.py:110-115);
  * `.sync(sync_buffer)` exchanges with the reference's blocking `_agg`;
  * `.uncompress(sync_buffer, neighbors_info)` RETURNS
    sum_r consensus_stepsize * (w_r - [r == rank]) * decode(msg_r).

Device side: the same batched codec as CHOCO / DCD; the local copy comes from
kernels (top-k: a scatter of the message into zeros with the accumulate kernel,
QSGD: the quantize pass's dense decode, sign: choco_sign_local_decode with
torch.sign's sign(0) = 0); the aggregate uses the receivers with the
reference's two-rounding add_(c * u) (include/choco_codec.h).
"""
import torch

from . import codec
from .communication import recover_device
from .dcd import _ConsumerBase
from .tensor_buffer import TensorBuffer


class DeepSqueezeCompressor(object):
    def __init__(self, **kargs):
        if "top_k" in kargs["comm_op"] or "random_k" in kargs["comm_op"]:
            self.compressor_fn = DeepSqueezeSparsificationCompressor(**kargs)
        elif "quantize" in kargs["comm_op"]:
            self.compressor_fn = DeepSqueezeQuantizationCompressor(**kargs)
        elif "sign" in kargs["comm_op"]:
            self.compressor_fn = DeepSqueezeSignCompressor(**kargs)
        else:
            raise NotImplementedError

    def compress(self, *args, **kargs):
        return self.compressor_fn.compress(*args, **kargs)

    def sync(self, *args, **kargs):
        return self.compressor_fn.sync(*args, **kargs)

    def uncompress(self, *args, **kargs):
        return self.compressor_fn.uncompress(*args, **kargs)


class _DeepSqueezeBase(_ConsumerBase):
    def __init__(self, aggregator, rank, comm_op, comm_device, compress_ratio, quantize_level, is_biased, backend,
                 use_ipc, consensus_stepsize, **kargs):
        super().__init__(aggregator, comm_op, comm_device, compress_ratio, quantize_level, is_biased, backend,
                         use_ipc, **kargs)
        self.rank = rank
        self.consensus_stepsize = consensus_stepsize

    def _inputs(self, sync_buffer):
        tb = sync_buffer["params_tb"]
        x = tb.buffer
        lay = self._layout(sync_buffer, x.device)
        if lay.n != x.numel():
            raise RuntimeError("original_shapes do not match params_tb")
        return tb, x, lay

    def _weight(self, neighbors_info, rank):
        # deep_squeeze.py:275-277 -- a Python double, rounded to fp32 where torch multiplies
        return self.consensus_stepsize * (neighbors_info[rank] - (1 if rank == self.rank else 0))

    @staticmethod
    def _like(tb, buffer):
        return TensorBuffer.from_flat(buffer, tb._tensors_sizes)


class DeepSqueezeSparsificationCompressor(_DeepSqueezeBase):
    """top-k / random-k  (deep_squeeze.py:158-279)."""

    def __init__(self, *args, **kargs):
        super().__init__(*args, **kargs)
        self._guards = {}

    def _guard(self, dev):
        g = self._guards.get(dev)
        if g is None:
            g = self._guards[dev] = codec.IndexGuard(dev)
        return g

    def compress(self, sync_buffer):
        tb, x, lay = self._inputs(sync_buffer)
        values, indices = self._sparse_message(sync_buffer, x, None, lay)
        local = torch.zeros_like(x)
        codec.sparse_accumulate(values, indices, local, 1.0)  # local[idx] = v  (deep_squeeze.py:206-208)
        return self._like(tb, local)

    def sync(self, sync_buffer):
        message = sync_buffer["wire_message"]
        sync_buffer["synced_message"] = self._send(message)
        sync_buffer["sycned_message_size"] = len(message)

    def uncompress(self, sync_buffer, neighbors_info):
        tb = sync_buffer["params_tb"]
        dev = tb.buffer.device
        agg = torch.zeros_like(tb.buffer)
        K = int(sync_buffer["sycned_message_size"] / 2)
        guard = self._guard(dev)
        for rank in neighbors_info.keys():
            msg = recover_device(sync_buffer["synced_message"][rank], device=dev)
            # agg[idx] += c * v  (two roundings, deep_squeeze.py:274-278)
            codec.sparse_accumulate(msg[:K].view(torch.float32), msg[K:], agg, self._weight(neighbors_info, rank),
                                    guard=guard)
        guard.check_then_arm()  # bad indices of an earlier step, after this step's work
        return self._like(tb, agg)


class DeepSqueezeQuantizationCompressor(_DeepSqueezeBase):
    """QSGD  (deep_squeeze.py:282-376)."""

    def compress(self, sync_buffer):
        tb, x, lay = self._inputs(sync_buffer)
        dense = self._qsgd_message(sync_buffer, x, None, lay, want_dense=True)
        return self._like(tb, dense.clone() if int(self.quantize_level) == 32 else dense)

    def sync(self, sync_buffer):
        sync_buffer["synced_message"] = self._send(sync_buffer["flatten_updates"].buffer)

    def uncompress(self, sync_buffer, neighbors_info):
        tb = sync_buffer["params_tb"]
        dev = tb.buffer.device
        lay = self._layout(sync_buffer, dev)
        agg = torch.zeros_like(tb.buffer)
        q = int(self.quantize_level)
        for rank in neighbors_info.keys():
            msg = recover_device(sync_buffer["synced_message"][rank], device=dev)
            c = self._weight(neighbors_info, rank)
            if q == 32:
                agg.add_(c * msg.view(torch.float32))
                continue
            # agg += c * decode(msg)  (two roundings, deep_squeeze.py:371-375)
            codec.qsgd_accumulate([self._qsgd_part(msg, lay)], [c], -1, lay.n, q, agg, is_biased=self.is_biased,
                                  seg_off=lay.seg_off, nseg=lay.nseg)
        return self._like(tb, agg)


class DeepSqueezeSignCompressor(_DeepSqueezeBase):
    """sign + per-tensor L1 norm  (deep_squeeze.py:379-489); norms and signs travel in ONE
    message, `synced_param_norms` / `synced_signs` are views of it."""

    def compress(self, sync_buffer):
        tb, x, lay = self._inputs(sync_buffer)
        signs, norms = self._sign_message(sync_buffer, x, None, lay)
        sync_buffer["param_norms_tb"] = TensorBuffer.from_flat(norms, [() for _ in range(lay.nseg)])
        # (norm_s * torch.sign(x)) / numel_s  (deep_squeeze.py:416-422)
        local = codec.sign_local_decode(x, norms, seg_off=lay.seg_off, nseg=lay.nseg)
        return self._like(tb, local)

    def sync(self, sync_buffer):
        norms = sync_buffer["param_norms_tb"].buffer
        synced = self._send(self._sign_wire(sync_buffer))
        sync_buffer["synced_message"] = synced
        sync_buffer["synced_param_norms"], sync_buffer["synced_signs"] = self._sign_parts(synced, norms.numel())

    def uncompress(self, sync_buffer, neighbors_info):
        tb = sync_buffer["params_tb"]
        dev = tb.buffer.device
        lay = self._layout(sync_buffer, dev)
        agg = torch.zeros_like(tb.buffer)
        for rank in neighbors_info.keys():
            nm = recover_device(sync_buffer["synced_param_norms"][rank], device=dev).contiguous()
            sg = recover_device(sync_buffer["synced_signs"][rank], device=dev)
            # agg_s.add_(c * (norm_s / numel_s * sign_s))  (two roundings, deep_squeeze.py:481-488)
            codec.sign_axpy([(sg, nm)], [self._weight(neighbors_info, rank)], lay.n, agg, seg_off=lay.seg_off,
                            nseg=lay.nseg, two_roundings=True)
        return self._like(tb, agg)
