"""Drop-in for the DCD-PSGD compressor (dl_code/pcode/optim/dcd_psgd.py:150-446).

`DCDCompressor(aggregator=, comm_op=, comm_device=, compress_ratio=,
quantize_level=, is_biased=, backend=, use_ipc=)` with `.compress(sync_buffer)`,
`.sync(sync_buffer)`, `.uncompress(sync_buffer, neighbor_hat_params)`; input keys
`original_shapes`, `flatten_half_params`, `flatten_params`.  DCD compresses
d = half_params - params per tensor and every rank adds each neighbour's decoded
message into its replica of that neighbour's model (no memory, no weights).

Same primitives as the CHOCO drop-in (parallel_choco.py): one batched device
compress over the flat buffers and this codec's packed wire; the receiver is
the fused accumulate with weight 1 (x[idx] + 1.0f * v = x[idx] + v bit for bit;
the sign receiver uses torch's add_(u, alpha) rounding, dcd_psgd.py:446).  The
exchange keeps the reference's blocking `_agg(..., force_wait=True)` call.
"""
import torch

from . import codec
from .communication import recover_device
from .parallel_choco import _Layout, _hdr_words, _seg_lens
from .sparsification import _draw_seed, get_n_bits
from .tensor_buffer import TensorBuffer


class DCDCompressor(object):
    def __init__(self, **kargs):
        if "top_k" in kargs["comm_op"] or "random_k" in kargs["comm_op"]:
            self.compressor_fn = DCDSparsificationCompressor(**kargs)
        elif "quantize" in kargs["comm_op"]:
            self.compressor_fn = DCDQuantizationCompressor(**kargs)
        elif "sign" in kargs["comm_op"]:
            self.compressor_fn = DCDSignCompressor(**kargs)
        else:
            raise NotImplementedError

    def compress(self, *args, **kargs):
        return self.compressor_fn.compress(*args, **kargs)

    def sync(self, *args, **kargs):
        return self.compressor_fn.sync(*args, **kargs)

    def uncompress(self, *args, **kargs):
        return self.compressor_fn.uncompress(*args, **kargs)


class _ConsumerBase(object):
    """Shared state of the non-CHOCO consumers (DCD here, DeepSqueeze in deep_squeeze.py)."""

    def __init__(self, aggregator, comm_op, comm_device, compress_ratio, quantize_level, is_biased, backend,
                 use_ipc, **kargs):
        self.aggregator_fn = aggregator
        self.comm_op = comm_op
        self.comm_device = comm_device
        self.compress_ratio = compress_ratio
        self.quantize_level = quantize_level
        self.is_biased = is_biased
        self.backend = backend
        self.use_ipc = use_ipc
        self.kargs = kargs

    def _send(self, message):
        if self.comm_device == "cpu":
            message = message.cpu().pin_memory()
        return self.aggregator_fn._agg(message, op="get_raw_sync_data", force_wait=True)

    @staticmethod
    def _layout(sync_buffer, device):
        return _Layout.get(_seg_lens(sync_buffer["original_shapes"]), device)

    # the three codecs on a flat buffer x (d = x - xhat when xhat is given) --------
    def _sparse_message(self, sync_buffer, x, xh, lay):
        plan = lay.topk_plan(float(self.compress_ratio))
        K = plan.k_total
        message = torch.empty(2 * K, dtype=torch.int32, device=x.device)
        values, indices = message[:K].view(torch.float32), message[K:]
        if "top_k" in self.comm_op:
            codec.topk_segmented(x, plan, xhat=xh, out=(values, indices))
        elif "random_k" in self.comm_op:
            # the reference never forwards is_biased to get_random_k (sparsification.py:60)
            codec.randk_segmented(x, plan, _draw_seed(), is_biased=True, xhat=xh, out=(values, indices))
        else:
            raise NotImplementedError
        local = torch.sub(indices, plan.selected_base())
        shapes = list(plan.k_per_seg)
        sync_buffer["selected_shapes"] = shapes
        sync_buffer["flatten_selected_values"] = TensorBuffer.from_flat(values, [(k,) for k in shapes])
        sync_buffer["flatten_selected_indices"] = TensorBuffer.from_flat(local, [(k,) for k in shapes])
        sync_buffer["n_bits"] = get_n_bits(values) + get_n_bits(local)
        sync_buffer["wire_message"] = message
        return values, indices

    def _qsgd_message(self, sync_buffer, x, xh, lay, want_dense=False):
        q = int(self.quantize_level)
        dense = None
        if q == 32:  # QuantizationCompressor passes the tensor through (sparsification.py:118-119)
            d = torch.sub(x, xh) if xh is not None else x
            message = d.contiguous().view(torch.uint8)
            dense = d
        else:
            message, out = codec.qsgd_wire(lay.n, q, lay.nseg, x.device)  # written in place by the kernels
            _, _, dense = codec.qsgd_compress(x, q, is_biased=self.is_biased, xhat=xh, seg_off=lay.seg_off,
                                              nseg=lay.nseg, seed=_draw_seed(), want_dense=want_dense, out=out)
        sync_buffer["flatten_updates"] = TensorBuffer.from_flat(message, [(message.numel(),)])
        sync_buffer["n_bits"] = get_n_bits(x) * self.quantize_level / 32  # nominal, as the reference
        sync_buffer["n_bits_wire"] = 8 * message.numel()
        return dense

    def _sign_message(self, sync_buffer, x, xh, lay):
        message, (signs, norms) = codec.sign_wire(lay.n, lay.nseg, x.device)  # written in place by the kernels
        codec.sign_compress(x, xhat=xh, seg_off=lay.seg_off, nseg=lay.nseg, want_norms=True, out=(signs, norms))
        sync_buffer["sign_message"] = message
        sync_buffer["signs"] = signs
        sync_buffer["sign_size"] = torch.Size([lay.n])
        sync_buffer["n_bits"] = get_n_bits(norms) + get_n_bits(signs)
        return signs, norms

    @staticmethod
    def _sign_wire(sync_buffer):
        """[norms | signs]: the norms and signs of _sign_message are views of this one message."""
        return sync_buffer["sign_message"]

    @staticmethod
    def _sign_parts(synced, nseg):
        hw = _hdr_words(nseg)
        return ({r: m[:hw].view(torch.float32)[:nseg] for r, m in synced.items()},
                {r: m[hw:] for r, m in synced.items()})

    def _qsgd_part(self, message, lay):
        hb = 4 * _hdr_words(lay.nseg)
        return message[hb:], message[:hb].view(torch.float32)[:lay.nseg].contiguous()


class DCDSparsificationCompressor(_ConsumerBase):
    """top-k / random-k  (dcd_psgd.py:175-275)."""

    def __init__(self, *args, **kargs):
        super().__init__(*args, **kargs)
        self._guards = {}

    def compress(self, sync_buffer):
        x = sync_buffer["flatten_half_params"].buffer
        xh = sync_buffer["flatten_params"].buffer
        self._sparse_message(sync_buffer, x, xh, self._layout(sync_buffer, x.device))

    def sync(self, sync_buffer):
        message = sync_buffer["wire_message"]
        sync_buffer["synced_message"] = self._send(message)
        sync_buffer["sycned_message_size"] = len(message)

    def uncompress(self, sync_buffer, neighbor_hat_params):
        K = int(sync_buffer["sycned_message_size"] / 2)
        for rank, hat_params in neighbor_hat_params.items():
            dev = hat_params.buffer.device
            guard = self._guards.get(dev)
            if guard is None:
                guard = self._guards[dev] = codec.IndexGuard(dev)
            msg = recover_device(sync_buffer["synced_message"][rank], device=dev)
            # hat[idx] += v  (dcd_psgd.py:275) == hat[idx] + 1.0f * v
            codec.sparse_accumulate(msg[:K].view(torch.float32), msg[K:], hat_params.buffer, 1.0, guard=guard)
        for guard in self._guards.values():  # bad indices of an earlier step, after this step's work
            guard.check_then_arm()


class DCDQuantizationCompressor(_ConsumerBase):
    """QSGD  (dcd_psgd.py:278-352)."""

    def compress(self, sync_buffer):
        x = sync_buffer["flatten_half_params"].buffer
        xh = sync_buffer["flatten_params"].buffer
        self._qsgd_message(sync_buffer, x, xh, self._layout(sync_buffer, x.device))

    def sync(self, sync_buffer):
        sync_buffer["synced_message"] = self._send(sync_buffer["flatten_updates"].buffer)

    def uncompress(self, sync_buffer, neighbor_hat_params):
        q = int(self.quantize_level)
        for rank, hat_params in neighbor_hat_params.items():
            dev = hat_params.buffer.device
            lay = self._layout(sync_buffer, dev)
            msg = recover_device(sync_buffer["synced_message"][rank], device=dev)
            if q == 32:
                hat_params.buffer.add_(msg.view(torch.float32))
                continue
            # hat += decode(msg)  (dcd_psgd.py:352) == hat + 1.0f * v
            codec.qsgd_accumulate([self._qsgd_part(msg, lay)], [1.0], -1, lay.n, q, hat_params.buffer,
                                  is_biased=self.is_biased, seg_off=lay.seg_off, nseg=lay.nseg)


class DCDSignCompressor(_ConsumerBase):
    """sign + per-tensor L1 norm  (dcd_psgd.py:355-446); norms and signs travel in ONE
    message, `synced_flatten_norms` / `synced_signs` are views of it."""

    def compress(self, sync_buffer):
        x = sync_buffer["flatten_half_params"].buffer
        xh = sync_buffer["flatten_params"].buffer
        lay = self._layout(sync_buffer, x.device)
        signs, norms = self._sign_message(sync_buffer, x, xh, lay)
        sync_buffer["flatten_norms"] = TensorBuffer.from_flat(norms, [() for _ in range(lay.nseg)])
        sync_buffer["flatten_updates"] = None  # the delta is never materialised (fused)

    def sync(self, sync_buffer):
        norms = sync_buffer["flatten_norms"].buffer
        synced = self._send(self._sign_wire(sync_buffer))
        sync_buffer["synced_message"] = synced
        sync_buffer["synced_flatten_norms"], sync_buffer["synced_signs"] = self._sign_parts(synced, norms.numel())

    def uncompress(self, sync_buffer, neighbor_hat_params):
        for rank, hat_params in neighbor_hat_params.items():
            dev = hat_params.buffer.device
            lay = self._layout(sync_buffer, dev)
            nm = recover_device(sync_buffer["synced_flatten_norms"][rank], device=dev).contiguous()
            sg = recover_device(sync_buffer["synced_signs"][rank], device=dev)
            # hat_s.add_(norm_s / numel_s, sign_s)  (dcd_psgd.py:442-446)
            codec.sign_axpy([(sg, nm)], [1.0], lay.n, hat_params.buffer, seg_off=lay.seg_off, nseg=lay.nseg)
