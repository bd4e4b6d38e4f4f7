"""Drop-in for the CHOCO compressor operator API of
dl_code/pcode/optim/parallel_choco_v.py:158-558 (byte-identical copy in
parallel_choco.py:209-609).

`CHOCOCompressor(aggregator=, comm_op=, comm_device=, compress_ratio=,
quantize_level=, is_biased=, backend=, use_ipc=)` with `.pipeline / .compress /
.sync / .uncompress(sync_buffer, neighbor_hat_params, neighbors_info)` and the
same `sync_buffer` contract: input keys `original_shapes`, `flatten_params`,
`flatten_hat_params`; `n_bits` is the reference's nominal bit count.

What changes underneath:
  * compress is ONE fused device pass over the whole flat buffer (delta
    x - x_hat, per-tensor selection / quantization / sign + L1 norms) instead of
    a Python loop over parameter tensors plus TensorBuffer copies;
  * the wire is this codec's packed format: top-k = [fp32 values | int32 GLOBAL
    indices] (exact beyond 2^24, unlike the reference's fp32 indices);
    QSGD = [fp32 norms | level plane | sign plane]; sign = [fp32 norms | packed
    words] in ONE message (the reference sends norms and signs separately);
  * uncompress applies all neighbour messages with fused kernels in
    `neighbors_info` order, reproducing the reference's fp32 rounding sequence;
  * optional input key `gossip` = (memory buffer, consensus_stepsize): compress
    first applies ParallelCHOCO_V.step's update_params_from_neighbor
    (optim/utils.py:67-72) to `flatten_params` inside its own first pass
    (utils.fused_step drives it; include/choco_codec.h "fused gossip step");
  * optional input key `defer_receive` (QSGD, sign): uncompress keeps the received
    messages and the NEXT compress applies them in the same pass as its consensus step
    (include/choco_codec.h "deferred receive"); x_hat / memory lag by one step until that
    compress or `flush_receive()` (utils.fused_step(defer_receive=True) drives it).
"""
import inspect

import torch

from . import codec
from .communication import recover_device
from .sparsification import get_n_bits, _draw_seed
from .tensor_buffer import TensorBuffer


def _seg_lens(original_shapes):
    return tuple(int(s[1]) for s in original_shapes)


class _Layout:
    """Device-side segment table + top-k plans for one parameter layout."""

    _cache = {}

    def __init__(self, lens, device):
        self.lens = lens
        self.nseg = len(lens)
        offs = [0]
        for s in lens:
            offs.append(offs[-1] + s)
        self.n = offs[-1]
        self.seg_off_list = offs
        self.seg_off = torch.tensor(offs, dtype=torch.int64, device=device) if self.nseg > 1 else None
        self.device = device
        self._plans = {}

    @classmethod
    def get(cls, lens, device):
        key = (lens, str(device))
        lay = cls._cache.get(key)
        if lay is None:
            lay = cls(lens, device)
            cls._cache[key] = lay
        return lay

    def topk_plan(self, ratio):
        p = self._plans.get(ratio)
        if p is None:
            p = codec.SegmentPlan(self.lens, ratio, self.device)
            self._plans[ratio] = p
        return p


_hdr_words = codec.wire_header_words  # int32 words of the fp32 norms header (16-byte aligned)


class CHOCOCompressor(object):
    def __init__(self, **kargs):
        if "top_k" in kargs["comm_op"] or "random_k" in kargs["comm_op"]:
            self.compressor_fn = CHOCOSparsificationCompressor(**kargs)
        elif "quantize" in kargs["comm_op"]:
            self.compressor_fn = CHOCOQuantizationCompressor(**kargs)
        elif "sign" in kargs["comm_op"]:
            self.compressor_fn = CHOCOSignCompressor(**kargs)
        else:
            raise NotImplementedError

    def pipeline(self, *args, **kargs):
        return self.compressor_fn.pipeline(*args, **kargs)

    def compress(self, *args, **kargs):
        return self.compressor_fn.compress(*args, **kargs)

    def sync(self, *args, **kargs):
        return self.compressor_fn.sync(*args, **kargs)

    def uncompress(self, *args, **kargs):
        return self.compressor_fn.uncompress(*args, **kargs)

    def flush_receive(self):
        return self.compressor_fn.flush_receive()


class _CHOCOBase(object):
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
        # the reference binds the current stream here (parallel_choco_v.py:214-218)
        self.gossip_stream = torch.cuda.current_stream()
        # deferred receive: (messages, weights, self slot, memory, x_hat_i, layout) that the
        # next compress applies in its first pass (or flush_receive() applies alone)
        self._pending = None

    def pipeline(self, sync_buffer, neighbor_hat_params, neighbors_info):
        with torch.cuda.stream(self.gossip_stream):
            try:
                self.compress(sync_buffer)
                self.sync(sync_buffer)
                self.uncompress(sync_buffer, neighbor_hat_params, neighbors_info)
            except RuntimeError as e:
                print("Error: {}".format(e))

    # helpers --------------------------------------------------------------
    def _flat_inputs(self, sync_buffer):
        x = sync_buffer["flatten_params"].buffer
        xh = sync_buffer["flatten_hat_params"].buffer
        lay = _Layout.get(_seg_lens(sync_buffer["original_shapes"]), x.device)
        if lay.n != x.numel():
            raise RuntimeError("original_shapes do not match flatten_params")
        return x, xh, lay

    @staticmethod
    def _gossip(sync_buffer):
        g = sync_buffer.get("gossip")
        return None if g is None else (g[0], float(g[1]))

    def _send(self, sync_buffer, message, out=None):
        if self.comm_device == "cpu":
            message = message.cpu().pin_memory()
        if out is None:
            return self.aggregator_fn._agg(message, op="get_raw_sync_data", force_wait=False)
        return self.aggregator_fn._agg(message, op="get_raw_sync_data", force_wait=False, out=out)

    # deferred receive ---------------------------------------------------------
    def _defer(self, parts, weights, self_slot, memory, xhat_self, lay):
        if self._pending is not None:
            raise RuntimeError("deferred receive: the previous step's messages were never applied")
        self._pending = (parts, weights, self_slot, memory, xhat_self, lay)

    def _require_fused_consensus(self, g):
        """A pending receive may only be applied by a compress whose first pass runs the
        consensus step itself (then that pass reads x_hat / memory after the receive).  With
        the consensus step run outside (g is None: the reference's ParallelCHOCO_V.step),
        recover_params and update_params_from_neighbor have already read the stale x_hat and
        memory, so x and this step's message would silently diverge from the reference."""
        if self._pending is not None and g is None:
            raise RuntimeError("deferred receive pending: call compressor.flush_receive() before recover_params / "
                               "update_params_from_neighbor (the previous step ran with defer_receive=True)")

    def _flush_before_pass(self, g):
        """Compress paths that never take a receive into their own pass: apply a pending one
        first (valid only with the consensus step fused into this compress)."""
        self._require_fused_consensus(g)
        self.flush_receive()

    def _take_pending(self, x, xh, g, lay):
        """The pending receive if this compress can apply it in its first pass (the
        consensus step fused, x_hat_i itself -- not a copy -- as flatten_hat_params);
        otherwise it is applied on its own first (flush_receive; the fused consensus step
        then reads the updated x_hat / memory), and None.  Raises when the consensus step
        is not fused into this compress (_require_fused_consensus)."""
        pend = self._pending
        if pend is None:
            return None
        self._require_fused_consensus(g)
        parts, weights, slot, memory, xhat_self, play = pend
        if play is not lay:
            self.flush_receive()
            return None
        if g[0].data_ptr() != memory.data_ptr() or (slot >= 0 and xh.data_ptr() != xhat_self.data_ptr()):
            raise RuntimeError("deferred receive: the next compress must take the same memory buffer and x_hat_i "
                               "itself as flatten_hat_params (utils.fused_step(defer_receive=True))")
        self._pending = None
        return parts, weights, slot

    def flush_receive(self):
        """Apply a deferred receive now (before reading x_hat / memory between steps).  It runs
        on the gossip stream, where the pending messages, memory and x_hat were written."""
        pend, self._pending = self._pending, None
        if pend is not None:
            with torch.cuda.stream(self.gossip_stream):
                self._apply(*pend)

    @staticmethod
    def _self_slot(ranks, neighbor_hat_params):
        slots = [i for i, r in enumerate(ranks) if r in neighbor_hat_params]
        if len(slots) > 1:
            raise RuntimeError("more than one local x_hat in neighbor_hat_params")
        return slots[0] if slots else -1


class CHOCOSparsificationCompressor(_CHOCOBase):
    """top-k / random-k  (parallel_choco_v.py:189-332).

    compress writes values and GLOBAL int32 indices straight into the wire
    message [fp32 values | int32 indices]; `flatten_selected_indices` holds the
    reference's LOCAL per-tensor indices (parallel_choco_v.py:248-249), derived
    from the wire with the plan's cached segment starts."""

    def __init__(self, *args, **kargs):
        super().__init__(*args, **kargs)
        self._guards = {}

    def compress(self, sync_buffer):
        x, xh, lay = self._flat_inputs(sync_buffer)
        plan = lay.topk_plan(float(self.compress_ratio))
        K = plan.k_total
        message = torch.empty(2 * K, dtype=torch.int32, device=x.device)
        values, indices = message[:K].view(torch.float32), message[K:]
        g = self._gossip(sync_buffer)
        if "top_k" in self.comm_op:
            codec.topk_segmented(x, plan, xhat=xh, out=(values, indices), gossip=g)
        elif "random_k" in self.comm_op:
            # the reference never forwards is_biased to get_random_k (sparsification.py:60)
            codec.randk_segmented(x, plan, _draw_seed(), is_biased=True, xhat=xh, out=(values, indices), gossip=g)
        else:
            raise NotImplementedError
        selected_shapes = list(plan.k_per_seg)
        local = torch.sub(indices, plan.selected_base())
        sync_buffer["selected_shapes"] = selected_shapes
        sync_buffer["flatten_selected_values"] = TensorBuffer.from_flat(values, [(k,) for k in selected_shapes])
        sync_buffer["flatten_selected_indices"] = TensorBuffer.from_flat(local, [(k,) for k in selected_shapes])
        sync_buffer["wire_message"] = message
        # nominal bits as in parallel_choco_v.py:252-254 (32-bit values + 32-bit indices)
        sync_buffer["n_bits"] = get_n_bits(values) + get_n_bits(local)

    def sync(self, sync_buffer):
        message = sync_buffer["wire_message"]
        reqs, synced = self._send(sync_buffer, message)
        sync_buffer["sync_reqs"] = reqs
        sync_buffer["synced_message"] = synced
        sync_buffer["sycned_message_size"] = len(message)

    def _guard(self, device):
        g = self._guards.get(device)
        if g is None:
            g = self._guards[device] = codec.IndexGuard(device)
        return g

    def uncompress(self, sync_buffer, neighbor_hat_params, neighbors_info):
        K = int(sync_buffer["sycned_message_size"] / 2)
        memory = neighbor_hat_params["memory"]
        guard = self._guard(memory.buffer.device)
        # x_hat takes only the local message (hat_params.buffer += q_values,
        # parallel_choco_v.py:307-308): with remote messages pending, its scatter is
        # queued BEFORE waiting for them, so it runs while the exchange is in flight.
        # Bit-identical: memory's updates keep the neighbour order below.
        local = [r for r in neighbors_info if r in neighbor_hat_params]
        hat_early = len(local) == 1 and len(neighbors_info) > 1
        if hat_early:
            hat = neighbor_hat_params[local[0]].buffer
            msg = sync_buffer["wire_message"]
            codec.sparse_accumulate(msg[:K].view(torch.float32), msg[K:], hat, 1.0, guard=guard)
        self.aggregator_fn.complete_wait(sync_buffer["sync_reqs"])
        # every message applied by ONE call that runs the per-message kernels in neighbors_info
        # order (bit-identical to the reference's per-neighbour loop); a merged one-sweep form
        # was measured slower and removed ("Sparse accumulate")
        msgs, weights, slot, hat = [], [], -1, None
        for rank, weight in neighbors_info.items():
            hat_params = neighbor_hat_params[rank if rank in neighbor_hat_params else "memory"]
            msg = recover_device(sync_buffer["synced_message"][rank], device=hat_params.buffer.device)
            if rank in neighbor_hat_params and not hat_early:
                slot, hat = len(msgs), hat_params.buffer
            msgs.append((msg[:K].view(torch.float32), msg[K:]))
            weights.append(weight)
        codec.sparse_accumulate_multi(msgs, weights, memory.buffer, self_slot=slot, xhat_self=hat, guard=guard)
        # out-of-range indices of an EARLIER step (lazy, no sync), reported once this step's
        # messages are applied; pipeline() prints it as the reference prints its RuntimeErrors
        guard.check_then_arm()

    def check(self, wait=True):
        """Report bad received indices now (teardown / checkpoint): raises RuntimeError."""
        for g in self._guards.values():
            g.check(wait=wait)


class CHOCOQuantizationCompressor(_CHOCOBase):
    """QSGD  (parallel_choco_v.py:335-433).

    `exchange_chunks=C` (> 1, a constructor keyword every rank must pass alike) pipelines
    the exchange (communication.py:259-262): the norm pass, then C element
    ranges each quantized and SENT as soon as it is packed (the transfer of range c overlaps
    the quantize of range c + 1), and uncompress decodes range c as soon as it has arrived
    (overlapping the transfer of c + 1).  The wire is the chunked form of
    codec.qsgd_chunked_wire; x_hat / memory are bit-identical to C = 1 (every element sees
    the same messages in the same neighbour order).  `synced_message[rank]` is then the list
    [norms header, range 0, range 1, ...]."""

    def __init__(self, *args, **kargs):
        super().__init__(*args, **kargs)
        self.exchange_chunks = int(self.kargs.get("exchange_chunks", 1))

    def compress(self, sync_buffer):
        x, xh, lay = self._flat_inputs(sync_buffer)
        q = int(self.quantize_level)
        g = self._gossip(sync_buffer)
        if q == 32 or self.exchange_chunks > 1:
            self._flush_before_pass(g)  # (never deferred on these paths)
        if q != 32 and self.exchange_chunks > 1:
            return self._compress_chunked(sync_buffer, x, xh, lay, q, g)
        sync_buffer.pop("chunked", None)
        if q == 32:  # the reference sends the raw delta (sparsification.py:118-119)
            if g is not None:
                codec.gossip_step(x, g[0], xh, g[1])
            message = torch.sub(x, xh).view(torch.uint8)
        else:
            message, out = codec.qsgd_wire(lay.n, q, lay.nseg, x.device)  # written in place by the kernels
            pend = self._take_pending(x, xh, g, lay)
            if pend is not None:
                # the previous step's receive + the consensus step + the norm pass, one kernel;
                # then the quantize pass with those norms
                codec.qsgd_recv_gossip_norms(pend[0], pend[1], pend[2], x, g[0], xh, g[1], q,
                                             is_biased=self.is_biased, seg_off=lay.seg_off, nseg=lay.nseg,
                                             out=out[1])
                codec.qsgd_compress(x, q, is_biased=self.is_biased, xhat=xh, seg_off=lay.seg_off, nseg=lay.nseg,
                                    norm_in=out[1], seed=_draw_seed(), out=out)
            else:
                codec.qsgd_compress(x, q, is_biased=self.is_biased, xhat=xh, seg_off=lay.seg_off, nseg=lay.nseg,
                                    seed=_draw_seed(), gossip=g, out=out)
        sync_buffer["flatten_updates"] = TensorBuffer.from_flat(message, [(message.numel(),)])
        # nominal bits as in parallel_choco_v.py:393
        sync_buffer["n_bits"] = get_n_bits(x) * self.quantize_level / 32
        sync_buffer["n_bits_wire"] = 8 * message.numel()

    def _compress_chunked(self, sync_buffer, x, xh, lay, q, g):
        message, norms, parts = codec.qsgd_chunked_wire(lay.n, q, lay.nseg, self.exchange_chunks, x.device)
        codec.qsgd_norms(x, xhat=xh, seg_off=lay.seg_off, nseg=lay.nseg, gossip=g, out=norms)
        hb = 4 * _hdr_words(lay.nseg)
        # the norms header leaves first; every range is posted right after its quantize launch,
        # so its transfer (ordered after it on the stream) overlaps the next range's quantize
        head = self._send(sync_buffer, message[:hb])
        seed = _draw_seed()
        posted = []
        for e0, e1, part in parts:
            codec.qsgd_quantize_range(x, q, norms, e0, e1, part, is_biased=self.is_biased, xhat=xh,
                                      seg_off=lay.seg_off, nseg=lay.nseg, seed=seed)
            posted.append(self._send(sync_buffer, part))
        sync_buffer["chunked"] = (head, [(e0, e1) for e0, e1, _ in parts], posted)
        sync_buffer["flatten_updates"] = TensorBuffer.from_flat(message, [(message.numel(),)])
        sync_buffer["n_bits"] = get_n_bits(x) * self.quantize_level / 32  # nominal (parallel_choco_v.py:393)
        sync_buffer["n_bits_wire"] = 8 * message.numel()

    def sync(self, sync_buffer):
        if "chunked" in sync_buffer:  # posted by compress, range by range
            (h_reqs, h_synced), _, posted = sync_buffer["chunked"]
            sync_buffer["sync_reqs"] = h_reqs + [r for p in posted for r in p[0]]
            sync_buffer["synced_message"] = {r: [h_synced[r]] + [p[1][r] for p in posted] for r in h_synced}
            return
        reqs, synced = self._send(sync_buffer, sync_buffer["flatten_updates"].buffer)
        sync_buffer["sync_reqs"] = reqs
        sync_buffer["synced_message"] = synced

    def _uncompress_chunked(self, sync_buffer, neighbor_hat_params, neighbors_info):
        (h_reqs, h_synced), ranges, posted = sync_buffer["chunked"]
        memory = neighbor_hat_params["memory"]
        dev = memory.buffer.device
        lay = _Layout.get(_seg_lens(sync_buffer["original_shapes"]), dev)
        ranks = list(neighbors_info.keys())
        weights = [neighbors_info[r] for r in ranks]
        self_slot = self._self_slot(ranks, neighbor_hat_params)
        xhat_self = neighbor_hat_params[ranks[self_slot]].buffer if self_slot >= 0 else None
        self.aggregator_fn.complete_wait(h_reqs)
        norms = [recover_device(h_synced[r], device=dev).view(torch.float32)[:lay.nseg].contiguous() for r in ranks]
        for (e0, e1), (reqs, synced) in zip(ranges, posted):
            self.aggregator_fn.complete_wait(reqs)  # this range only: later ones are still in flight
            msgs = [(recover_device(synced[r], device=dev), nm) for r, nm in zip(ranks, norms)]
            codec.qsgd_accumulate_range(msgs, weights, self_slot, lay.n, int(self.quantize_level), memory.buffer,
                                        e0, e1, xhat_self=xhat_self, is_biased=self.is_biased,
                                        seg_off=lay.seg_off, nseg=lay.nseg)

    def uncompress(self, sync_buffer, neighbor_hat_params, neighbors_info):
        if "chunked" in sync_buffer:
            return self._uncompress_chunked(sync_buffer, neighbor_hat_params, neighbors_info)
        self.aggregator_fn.complete_wait(sync_buffer["sync_reqs"])
        memory = neighbor_hat_params["memory"]
        dev = memory.buffer.device
        lay = _Layout.get(_seg_lens(sync_buffer["original_shapes"]), dev)
        ranks = list(neighbors_info.keys())
        weights = [neighbors_info[r] for r in ranks]
        self_slot = self._self_slot(ranks, neighbor_hat_params)
        xhat_self = neighbor_hat_params[ranks[self_slot]].buffer if self_slot >= 0 else None
        q = int(self.quantize_level)
        msgs = [recover_device(sync_buffer["synced_message"][r], device=dev) for r in ranks]
        if q == 32:
            for i, (m, w) in enumerate(zip(msgs, weights)):
                v = m.view(torch.float32)
                if i == self_slot:
                    xhat_self += v
                memory.buffer += w * v
            return
        hb = 4 * _hdr_words(lay.nseg)
        parts = [(m[hb:], m[:hb].view(torch.float32)[:lay.nseg].contiguous()) for m in msgs]
        if sync_buffer.get("defer_receive"):  # applied by the next compress's first pass
            return self._defer(parts, weights, self_slot, memory.buffer, xhat_self, lay)
        self._apply(parts, weights, self_slot, memory.buffer, xhat_self, lay)

    def _apply(self, parts, weights, self_slot, memory, xhat_self, lay):
        codec.qsgd_accumulate(parts, weights, self_slot, lay.n, int(self.quantize_level), memory,
                              xhat_self=xhat_self, is_biased=self.is_biased, seg_off=lay.seg_off, nseg=lay.nseg)


class _Reassembled(dict):
    """{rank: [norms | words] message} of a chunked sign exchange over an aggregator without
    `out=`: each neighbour's message is concatenated from its received ranges on first
    access, i.e. after uncompress has waited for every request."""

    def __init__(self, rank, message, head, parts):
        super().__init__()
        self._src = {r: (head[r], [p[r] for p in parts]) for r in head if r != rank}
        self[rank] = message
        for r in self._src:
            dict.__setitem__(self, r, None)

    def __getitem__(self, r):
        v = dict.__getitem__(self, r)
        if v is None:
            h, ps = self._src[r]
            v = torch.cat([h] + ps)
            dict.__setitem__(self, r, v)
        return v

    def items(self):
        return [(r, self[r]) for r in self.keys()]

    def values(self):
        return [self[r] for r in self.keys()]


class _LazyMap(dict):
    """{rank: fn(src[rank])}, evaluated on access."""

    def __init__(self, src, fn):
        super().__init__((r, None) for r in src.keys())
        self._src, self._fn = src, fn

    def __getitem__(self, r):
        return self._fn(self._src[r])

    def items(self):
        return [(r, self[r]) for r in self.keys()]

    def values(self):
        return [self[r] for r in self.keys()]


class CHOCOSignCompressor(_CHOCOBase):
    """sign + per-tensor L1 norm  (parallel_choco_v.py:436-558).

    `exchange_chunks=C` (> 1, every rank alike) pipelines the send with the pack: the
    words are packed in C column ranges and each range's words are posted as soon as its
    pack is queued (its transfer overlaps the next range's pack); the norms header, complete
    only after the last range, leaves last.  Every range of the (32, N') layout touches
    every row's segments, so the receiver decodes after the whole message, as with C = 1
    (include/choco_codec.h "Chunked sign pack").  Neighbours receive straight into one
    message per rank, so the wire, `synced_message` and the decode are those of C = 1."""

    def __init__(self, *args, **kargs):
        super().__init__(*args, **kargs)
        self.exchange_chunks = int(self.kargs.get("exchange_chunks", 1))

    def compress(self, sync_buffer):
        x, xh, lay = self._flat_inputs(sync_buffer)
        message, (signs, norms) = codec.sign_wire(lay.n, lay.nseg, x.device)  # written in place by the kernels
        g = self._gossip(sync_buffer)
        sync_buffer.pop("chunked", None)
        if self.exchange_chunks > 1:
            self._flush_before_pass(g)  # (never deferred on this path)
            sync_buffer["chunked"] = self._pack_and_post(sync_buffer, x, xh, lay, g, message, signs, norms)
        else:
            pend = self._take_pending(x, xh, g, lay)
            if pend is not None:  # the previous step's receive + the consensus step + the pack, one pass
                codec.sign_recv_gossip_compress(pend[0], pend[1], pend[2], x, g[0], xh, g[1], seg_off=lay.seg_off,
                                                nseg=lay.nseg, out=(signs, norms))
            else:
                codec.sign_compress(x, xhat=xh, seg_off=lay.seg_off, nseg=lay.nseg, want_norms=True, gossip=g,
                                    out=(signs, norms))
        sync_buffer["sign_message"] = message
        sync_buffer["flatten_norms"] = TensorBuffer.from_flat(norms, [() for _ in range(lay.nseg)])
        sync_buffer["flatten_directions"] = None  # the delta is never materialised (fused)
        sync_buffer["signs"] = signs
        sync_buffer["sign_size"] = torch.Size([lay.n])
        # nominal bits as in parallel_choco_v.py:492
        sync_buffer["n_bits"] = get_n_bits(norms) + get_n_bits(signs)

    def _agg_takes_out(self):
        """Whether the aggregator's _agg accepts `out=` (this package's DecentralizedAggregation
        does; the reference's, communication.py:246, does not)."""
        try:
            ps = inspect.signature(self.aggregator_fn._agg).parameters
        except (TypeError, ValueError):
            return False
        return "out" in ps or any(p.kind == p.VAR_KEYWORD for p in ps.values())

    def _pack_and_post(self, sync_buffer, x, xh, lay, g, message, signs, norms):
        try:
            return self._pack_and_post_ranges(sync_buffer, x, xh, lay, g, message, signs, norms)
        except BaseException:
            # the per-segment L1 sums of the ranges packed so far stay in the stream's
            # accumulator workspace until the `finish` range clears them: drop it, so the next
            # sign / QSGD call does not add stale sums into its norms
            codec.drop_workspace(x.device, "acc")
            raise

    def _pack_and_post_ranges(self, sync_buffer, x, xh, lay, g, message, signs, norms):
        hw = _hdr_words(lay.nseg)
        ranges = codec.sign_chunks(lay.n, self.exchange_chunks)
        if not self._agg_takes_out():
            # the reference's aggregator: every range travels as a message of its own (same
            # posting order); uncompress re-assembles each neighbour's [norms | words]
            parts, reqs = [], []
            for i, (w0, w1) in enumerate(ranges):
                codec.sign_compress_range(x, w0, w1, i == len(ranges) - 1, xhat=xh, seg_off=lay.seg_off,
                                          nseg=lay.nseg, gossip=g, out=(signs, norms))
                r, synced = self._send(sync_buffer, message[hw + w0:hw + w1])
                reqs += r
                parts.append(synced)
            r, head = self._send(sync_buffer, message[:hw])
            return reqs + r, _Reassembled(self.aggregator_fn.rank, message, head, parts)
        peers = [r for r in self.aggregator_fn.neighbor_ranks]
        host = self.comm_device == "cpu"
        recv = {r: torch.empty(message.shape, dtype=message.dtype, device="cpu" if host else message.device,
                               pin_memory=host) for r in peers}
        reqs = []
        for i, (w0, w1) in enumerate(ranges):
            codec.sign_compress_range(x, w0, w1, i == len(ranges) - 1, xhat=xh, seg_off=lay.seg_off,
                                      nseg=lay.nseg, gossip=g, out=(signs, norms))
            r, _ = self._send(sync_buffer, message[hw + w0:hw + w1],
                              out={p: recv[p][hw + w0:hw + w1] for p in peers})
            reqs += r
        r, _ = self._send(sync_buffer, message[:hw], out={p: recv[p][:hw] for p in peers})
        recv[self.aggregator_fn.rank] = message
        return reqs + r, recv

    def sync(self, sync_buffer):
        norms = sync_buffer["flatten_norms"].buffer
        hw = _hdr_words(norms.numel())
        if "chunked" in sync_buffer:  # posted by compress, range by range
            reqs, synced = sync_buffer["chunked"]
        else:
            reqs, synced = self._send(sync_buffer, sync_buffer["sign_message"])  # [norms | signs]
        sync_buffer["sync_reqs_1"] = reqs
        sync_buffer["sync_reqs_2"] = []
        sync_buffer["synced_message"] = synced
        # the reference's two received dicts (parallel_choco_v.py:521-522), as views of
        # the one message per rank: [fp32 norms (16-B padded) | int32 words]
        nseg = norms.numel()
        if isinstance(synced, _Reassembled):  # assembled after uncompress's wait, not now
            sync_buffer["synced_flatten_norms"] = _LazyMap(synced, lambda m: m[:hw].view(torch.float32)[:nseg])
            sync_buffer["synced_signs"] = _LazyMap(synced, lambda m: m[hw:])
        else:
            sync_buffer["synced_flatten_norms"] = {r: m[:hw].view(torch.float32)[:nseg] for r, m in synced.items()}
            sync_buffer["synced_signs"] = {r: m[hw:] for r, m in synced.items()}

    def uncompress(self, sync_buffer, neighbor_hat_params, neighbors_info):
        self.aggregator_fn.complete_wait(sync_buffer["sync_reqs_1"])
        self.aggregator_fn.complete_wait(sync_buffer["sync_reqs_2"])
        memory = neighbor_hat_params["memory"]
        dev = memory.buffer.device
        lay = _Layout.get(_seg_lens(sync_buffer["original_shapes"]), dev)
        ranks = list(neighbors_info.keys())
        weights = [neighbors_info[r] for r in ranks]
        self_slot = self._self_slot(ranks, neighbor_hat_params)
        xhat_self = neighbor_hat_params[ranks[self_slot]].buffer if self_slot >= 0 else None
        parts = []
        for r in ranks:
            nm = recover_device(sync_buffer["synced_flatten_norms"][r], device=dev).contiguous()
            sg = recover_device(sync_buffer["synced_signs"][r], device=dev)
            parts.append((sg, nm))
        if sync_buffer.get("defer_receive") and "chunked" not in sync_buffer:  # the next compress applies them
            return self._defer(parts, weights, self_slot, memory.buffer, xhat_self, lay)
        self._apply(parts, weights, self_slot, memory.buffer, xhat_self, lay)

    def _apply(self, parts, weights, self_slot, memory, xhat_self, lay):
        codec.sign_accumulate(parts, weights, self_slot, lay.n, memory, xhat_self=xhat_self, seg_off=lay.seg_off,
                              nseg=lay.nseg)
