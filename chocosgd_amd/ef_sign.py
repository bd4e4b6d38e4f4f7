"""Drop-in for the EF-signSGD compressor (dl_code/pcode/optim/ef_sign_sgd.py:126-219).

`EFSignCompressor(rank, world_size, aggregator, comm_op, comm_device, use_ipc)`:
  * `.compress(grads_tb)` -> sync_buffer with the per-tensor L1 norms, the packed
    signs and `synced_grads_tb` = this rank's decoded copy (norm * sign(g) / numel,
    sign(0) = 0) that the optimizer's error feedback subtracts;
  * `.sync(sync_buffer)` all-gathers ONE [norms | words] message per rank through a
    centralized aggregator (`_agg(..., communication_scheme="all_gather")`);
  * `.decompress(sync_buffer)` adds every other rank's decoded signs (in rank
    order) and divides by the world size.
Kernels: the batched sign pack (norms fused), choco_sign_local_decode and the
fused multi-message sign receiver (weight 1).
"""
import torch

from . import codec
from .communication import recover_device
from .parallel_choco import _Layout, _hdr_words
from .sparsification import get_n_bits
from .tensor_buffer import TensorBuffer


class EFSignCompressor(object):
    def __init__(self, rank, world_size, aggregator, comm_op, comm_device, use_ipc, **kargs):
        self.rank = rank
        self.world_size = world_size
        self.aggregator_fn = aggregator
        self.comm_op = comm_op
        self.comm_device = comm_device
        self.use_ipc = use_ipc
        self.kargs = kargs

    @staticmethod
    def _layout(tb):
        lens = tuple(int(torch.Size(s).numel()) for s in tb._tensors_sizes)
        return _Layout.get(lens, tb.buffer.device)

    def compress(self, grads_tb):
        g = grads_tb.buffer
        lay = self._layout(grads_tb)
        message, (signs, norms) = codec.sign_wire(lay.n, lay.nseg, g.device)  # written in place by the kernels
        codec.sign_compress(g, seg_off=lay.seg_off, nseg=lay.nseg, want_norms=True, out=(signs, norms))
        local = codec.sign_local_decode(g, norms, seg_off=lay.seg_off, nseg=lay.nseg)
        return {"grad_norms_tb": TensorBuffer.from_flat(norms, [() for _ in range(lay.nseg)]),
                "grads_tb": grads_tb,
                "synced_grads_tb": TensorBuffer.from_flat(local, grads_tb._tensors_sizes),
                "signs": signs, "sign_message": message, "sign_size": torch.Size([lay.n]),
                "n_bits": get_n_bits(norms) + get_n_bits(signs)}

    def sync(self, sync_buffer):
        norms = sync_buffer["grad_norms_tb"].buffer
        hw = _hdr_words(norms.numel())
        message = sync_buffer["sign_message"]  # [norms | signs]: written in place by compress
        if self.comm_device == "cpu":
            message = message.cpu().pin_memory()
        synced = self.aggregator_fn._agg(message, communication_scheme="all_gather", async_op=False)
        nseg = norms.numel()
        sync_buffer["synced_message"] = synced
        sync_buffer["synced_grad_norms"] = [m[:hw].view(torch.float32)[:nseg] for m in synced]
        sync_buffer["synced_signs"] = [m[hw:] for m in synced]

    def decompress(self, sync_buffer):
        tb = sync_buffer["synced_grads_tb"]
        dev = tb.buffer.device
        lay = self._layout(tb)
        parts = []
        for rank in range(self.world_size):
            if rank == self.rank:
                continue
            nm = recover_device(sync_buffer["synced_grad_norms"][rank], device=dev).contiguous()
            sg = recover_device(sync_buffer["synced_signs"][rank], device=dev)
            parts.append((sg, nm))
        if parts:
            # synced_grad_s.add_(norm_s * sign_s / numel_s)  (ef_sign_sgd.py:212-215), ranks in order
            codec.sign_axpy(parts, [1.0] * len(parts), lay.n, tb.buffer, seg_off=lay.seg_off, nseg=lay.nseg)
        # true division (a device 0-dim divisor: torch multiplies by the reciprocal of a CPU scalar)
        tb.buffer.div_(torch.full((), self.world_size * 1.0, dtype=torch.float32, device=dev))
        return tb
