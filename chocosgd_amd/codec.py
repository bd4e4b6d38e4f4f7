"""Tensor-level entry points of the MI355X CHOCO codec.

Thin, allocation-light wrappers over the C ABI (include/choco_codec.h): they
validate that every tensor is a contiguous ROCm device tensor, allocate the
outputs with torch, pass raw pointers + the current HIP stream, and raise
RuntimeError on any library error.  CPU tensors are rejected -- there is no CPU
fallback anywhere in the product path.
"""
import ctypes
import math
import threading

import torch

from . import _lib

_ws_lock = threading.Lock()
_ws_cache = {}


def _require(t, dtype=None, name="tensor"):
    if not isinstance(t, torch.Tensor):
        raise RuntimeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise RuntimeError(
            f"chocosgd_amd runs on ROCm device tensors only; {name} is on {t.device}")
    if dtype is not None and t.dtype != dtype:
        raise RuntimeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    return t


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _new_workspace(dev, nbytes):
    """A zero-filled workspace; the library forgets any warm-start record it kept for
    that address range (a freed workspace's address can come back)."""
    buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    lib().choco_topk_workspace_reset(_ptr(buf), buf.numel())
    return buf


def workspace(dev, kind, nbytes):
    """Per (device, stream, kind) scratch buffer; zero-filled on allocation.

    The sign/qsgd accumulators rely on starting zeroed; every kernel that uses
    them leaves them zeroed again (self-cleaning), so the buffer is reused as is.
    A top-k workspace also carries the warm-start window from one call to the next
    (include/choco_codec.h).
    """
    nbytes = max(int(nbytes), 256)
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream, kind)
    with _ws_lock:
        buf = _ws_cache.get(key)
        if buf is None or buf.numel() < nbytes:
            if buf is not None:
                torch.cuda.current_stream(dev).synchronize()
                _status.pop(buf.data_ptr(), None)
            buf = _new_workspace(dev, nbytes)
            _ws_cache[key] = buf
        return buf


class TopkStatus:
    """Check of a top-k workspace's sticky status word (include/choco_codec.h,
    CHOCO_TOPK_STATUS_OFFSET) through its pinned host mirror: the device raises the bits
    there with a system-scope store, so `check()` -- called before every top-k call --
    reads host memory only (no copy on the stream, no synchronisation) and raises
    RuntimeError as soon as a call whose bounded fallback wait gave up has run on the GPU;
    that call's output (and whatever was computed from it: the model state of a CHOCO step
    that applied it) is invalid.  `check(wait=True)` first waits for the stream (teardown,
    checkpoints).  Holds the workspace's address only, never the tensor: a dropped
    workspace or SegmentPlan frees its device memory."""

    def __init__(self, ws):
        self.ptr = ws.data_ptr()
        self.device = ws.device
        # the stream the workspace belongs to (workspaces are per (device, stream): it is the
        # current stream when the workspace is taken, codec.workspace / SegmentPlan.workspace)
        self.stream = torch.cuda.current_stream(ws.device)

    def check(self, wait=False):
        if wait:
            self.stream.synchronize()
        bad = int(lib().choco_topk_host_status(ctypes.c_void_p(self.ptr), 1, _stream(self.device)))
        if bad < 0:
            raise RuntimeError(f"choco_topk_host_status failed: {_lib.last_error()}")
        if bad:
            raise RuntimeError(f"top-k: status word {bad:#x}: a bounded wait of the exact fallback gave up, so the "
                               "output of an earlier call on this workspace is invalid (and every state it was "
                               "applied to)")


_status = {}


def topk_status(ws):
    """The TopkStatus of a workspace tensor (one per workspace address)."""
    st = _status.get(ws.data_ptr())
    if st is None:
        st = _status[ws.data_ptr()] = TopkStatus(ws)
    return st


def check_topk_status(wait=True):
    """Check every top-k workspace's status word now (raises RuntimeError)."""
    for st in list(_status.values()):
        st.check(wait=wait)


def topk_fallback_count(dev=None, plan=None):
    """Diagnostic: calls on this stream's flat top-k workspace that took the exact fallback,
    or (plan=...) segments of that plan whose warm window missed (include/choco_codec.h
    CHOCO_TOPK_FALLBACKS_OFFSET).  Synchronises the stream."""
    dev = torch.device(dev) if dev is not None else torch.device("cuda", torch.cuda.current_device())
    if plan is not None:
        ws = plan.workspace(dev)
    else:
        with _ws_lock:
            ws = _ws_cache.get((dev.index, torch.cuda.current_stream(dev).cuda_stream, "topk"))
        if ws is None:
            return 0
    off = _lib.TOPK_FALLBACKS_OFFSET
    torch.cuda.current_stream(dev).synchronize()
    return int(ws[off:off + 4].view(torch.int32).item())


def workspace_bytes():
    """Device bytes held by the cached scratch buffers (top-k: ~9 bytes per element of
    the largest flat input, sized for 288 GB HBM rather than packed)."""
    with _ws_lock:
        return sum(b.numel() for b in _ws_cache.values())


def drop_workspace(dev, kind):
    """Forget this stream's cached `kind` workspace (after a call sequence failed part-way:
    e.g. the sign / QSGD accumulators of an interrupted chunked pack are no longer zero);
    the next call allocates a fresh zero-filled one."""
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream, kind)
    with _ws_lock:
        buf = _ws_cache.pop(key, None)
    if buf is not None:
        torch.cuda.current_stream(dev).synchronize()
        _status.pop(buf.data_ptr(), None)
        lib().choco_topk_workspace_reset(_ptr(buf), buf.numel())


def release_workspaces(dev=None):
    """Drop the cached scratch buffers (all devices, or `dev`) after synchronising the
    streams that used them; the next call on that stream allocates a fresh, zeroed one.
    SegmentPlan workspaces belong to their plan and go with it."""
    with _ws_lock:
        for key in list(_ws_cache):
            if dev is not None and key[0] != torch.device(dev).index:
                continue
            torch.cuda.synchronize(key[0])
            buf = _ws_cache.pop(key)
            _status.pop(buf.data_ptr(), None)
            lib().choco_topk_workspace_reset(_ptr(buf), buf.numel())


def lib():
    return _lib.load()


def _gossip(gossip, x, xhat):
    """`gossip=(memory, gamma)`: the fused consensus step x += gamma * (memory - xhat)
    (optim/utils.py:67-72) in the compressor's first pass; x is written in place and
    the codec compresses d = x_new - xhat (include/choco_codec.h)."""
    if gossip is None:
        return None
    memory, gamma = gossip
    _require(memory, torch.float32, "memory")
    if xhat is None:
        raise RuntimeError("the fused gossip step needs xhat")
    if memory.numel() != x.numel():
        raise RuntimeError("memory and x must have the same number of elements")
    return memory, float(gamma)


# ----------------------------------------------------------------------------- top-k
def topk_k(n, ratio):
    """k = max(1, int(n * (1 - ratio))) (sparsification.py:22,45)."""
    return int(lib().choco_topk_k(int(n), float(ratio)))


def topk(x, k, xhat=None, out=None, gossip=None, fold=None):
    """Exact top-k by |x - xhat| (signed values, int32 indices, ascending index).

    `out=(values f32[k], indices i32[k])` writes into caller buffers (e.g. two views
    of one wire message) instead of allocating; `gossip=(memory, gamma)` fuses the
    consensus step (x is updated in place first).  `fold=(hat_self, memory, weight)`
    (either may be None) applies the self message's uncompress while the message is
    emitted: hat_self[idx] += v, memory[idx] += weight * v.  Folding memory is only
    bit-identical to the reference when the self rank is the first message applied to
    memory (include/choco_codec.h, choco_topk_compress_accumulate).  With `gossip`,
    hat_self must be xhat and memory the gossip memory (or None)."""
    _require(x, torch.float32, "x")
    if xhat is not None:
        _require(xhat, torch.float32, "xhat")
        if xhat.numel() != x.numel():
            raise RuntimeError("x and xhat must have the same number of elements")
    n = x.numel()
    dev = x.device
    if out is not None:
        vals, idx = out
        _require(vals, torch.float32, "out values")
        _require(idx, torch.int32, "out indices")
        if vals.numel() != k or idx.numel() != k:
            raise RuntimeError("out buffers must hold exactly k elements")
    else:
        vals = torch.empty(k, dtype=torch.float32, device=dev)
        idx = torch.empty(k, dtype=torch.int32, device=dev)
    L = lib()
    ws = workspace(dev, "topk", L.choco_topk_workspace_size(n))
    st = topk_status(ws)
    st.check()
    g = _gossip(gossip, x, xhat)
    if fold is not None:
        fhat, fmem, fw = fold
        for t, nm in ((fhat, "hat_self"), (fmem, "memory")):
            if t is not None:
                _require(t, torch.float32, nm)
                if t.numel() != n:
                    raise RuntimeError(f"{nm} and x must have the same number of elements")
        if fhat is None and fmem is None:
            raise RuntimeError("fold: hat_self and memory are both None")
        if g is not None:
            if fhat is None or fhat.data_ptr() != xhat.data_ptr():
                raise RuntimeError("with gossip, the fold's hat_self must be xhat")
            if fmem is not None and fmem.data_ptr() != g[0].data_ptr():
                raise RuntimeError("with gossip, the folded memory must be the gossip memory")
            _lib.check(L.choco_gossip_topk_compress_accumulate(
                _ptr(x), _ptr(g[0]), _ptr(xhat), g[1], n, int(k), _ptr(vals), _ptr(idx), int(fmem is not None),
                float(fw), _ptr(ws), ws.numel(), _stream(dev)), "choco_gossip_topk_compress_accumulate")
        else:
            _lib.check(L.choco_topk_compress_accumulate(
                _ptr(x), _ptr(xhat), n, int(k), _ptr(vals), _ptr(idx), _ptr(fhat), _ptr(fmem), float(fw),
                _ptr(ws), ws.numel(), _stream(dev)), "choco_topk_compress_accumulate")
    elif g is not None:
        _lib.check(L.choco_gossip_topk_compress(_ptr(x), _ptr(g[0]), _ptr(xhat), g[1], n, int(k), _ptr(vals),
                                                _ptr(idx), _ptr(ws), ws.numel(), _stream(dev)),
                   "choco_gossip_topk_compress")
    else:
        _lib.check(L.choco_topk_compress(_ptr(x), _ptr(xhat), n, int(k), _ptr(vals), _ptr(idx), _ptr(ws),
                                         ws.numel(), _stream(dev)), "choco_topk_compress")
    return vals, idx


class SegmentPlan:
    """Host + device copies of the per-segment top-k plan (include/choco_codec.h):
    rows {off, len, k, out_off, first tile, tiles, ..} + the tile -> segment map."""

    def __init__(self, seg_lens, ratio, device):
        L = lib()
        self.seg_lens = [int(s) for s in seg_lens]
        self.nseg = len(self.seg_lens)
        offs = [0]
        for s in self.seg_lens:
            offs.append(offs[-1] + s)
        self.seg_off = offs
        self.n = offs[-1]
        p_off, self._off_keep = _lib.i64_array(offs)
        plen = L.choco_topk_segmented_plan_len(p_off, self.nseg)
        if plen < 0:
            raise RuntimeError(f"choco_topk_segmented_plan_len failed: {_lib.last_error()}")
        self._plan_host = (ctypes.c_int64 * int(plen))()
        self.plan_host = ctypes.cast(self._plan_host, ctypes.POINTER(ctypes.c_int64))
        total = L.choco_topk_segmented_plan(p_off, self.nseg, float(ratio), self.plan_host)
        if total < 0:
            raise RuntimeError(f"choco_topk_segmented_plan failed: {_lib.last_error()}")
        self.k_total = int(total)
        self.k_per_seg = [int(self._plan_host[8 * s + 2]) for s in range(self.nseg)]
        self.ntile = int(self._plan_host[6])
        self.plan_dev = torch.tensor(list(self._plan_host), dtype=torch.int64, device=device)
        self.ws_bytes = int(L.choco_topk_segmented_workspace_size(self.plan_host, self.nseg))
        self._base = None
        self._ws = {}

    def workspace(self, dev):
        """This plan's own zero-filled workspace per stream: the batched select keeps
        per-segment histograms there that every call leaves zeroed for the NEXT call of
        the same plan (include/choco_codec.h), so no other call may share it."""
        key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
        with _ws_lock:
            buf = self._ws.get(key)
            if buf is None:
                buf = self._ws[key] = _new_workspace(dev, max(self.ws_bytes, 256))
            return buf

    def __del__(self):
        # The plan's workspaces go with it, and so does the codec's host-side state keyed by
        # their addresses (warm windows, the pinned miss flag): a later workspace at the
        # same address must not inherit it.  The device may still write the miss flag, so
        # the devices are synchronised before it is freed.
        try:
            bufs = list(self._ws.values())
            self._ws.clear()
            if not bufs:
                return
            for d in {b.device.index for b in bufs}:
                torch.cuda.synchronize(d)
            L = lib()
            for buf in bufs:
                _status.pop(buf.data_ptr(), None)
                L.choco_topk_workspace_reset(_ptr(buf), buf.numel())
        except Exception:  # interpreter shutdown: the library or torch may be gone
            pass

    def drop_workspace(self, dev):
        """Forget this plan's workspace on the current stream of `dev` (after a failed
        call: its histograms may not be zeroed any more); the next call starts cold on
        a fresh zero-filled one."""
        key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
        with _ws_lock:
            buf = self._ws.pop(key, None)
        if buf is not None:
            _status.pop(buf.data_ptr(), None)
            lib().choco_topk_workspace_reset(_ptr(buf), buf.numel())

    def selected_base(self):
        """int32[K]: the segment start of every output slot (global -> local index)."""
        if self._base is None:
            offs = torch.tensor(self.seg_off[:-1], dtype=torch.int32, device=self.plan_dev.device)
            ks = torch.tensor(self.k_per_seg, dtype=torch.int64, device=self.plan_dev.device)
            self._base = torch.repeat_interleave(offs, ks)
        return self._base


def _seg_outputs(x, xhat, plan, out):
    _require(x, torch.float32, "x")
    if x.numel() != plan.n:
        raise RuntimeError(f"x holds {x.numel()} elements, the segment plan {plan.n}")
    if xhat is not None:
        _require(xhat, torch.float32, "xhat")
        if xhat.numel() != x.numel():
            raise RuntimeError("x and xhat must have the same number of elements")
    if out is not None:
        vals, idx = out
        _require(vals, torch.float32, "out values")
        _require(idx, torch.int32, "out indices")
        if vals.numel() != plan.k_total or idx.numel() != plan.k_total:
            raise RuntimeError("out buffers must hold exactly the plan's K elements")
        return vals, idx
    return (torch.empty(plan.k_total, dtype=torch.float32, device=x.device),
            torch.empty(plan.k_total, dtype=torch.int32, device=x.device))


def topk_segmented(x, plan, xhat=None, out=None, gossip=None):
    """Per-segment top-k (k_s of the plan), GLOBAL int32 indices; `out=(values, indices)`
    writes into caller buffers (e.g. the two halves of a wire message);
    `gossip=(memory, gamma)` fuses the consensus step."""
    vals, idx = _seg_outputs(x, xhat, plan, out)
    dev = x.device
    L = lib()
    ws = plan.workspace(dev)
    st = topk_status(ws)
    st.check()
    g = _gossip(gossip, x, xhat)
    try:
        if g is not None:
            _lib.check(L.choco_gossip_topk_compress_segmented(_ptr(x), _ptr(g[0]), _ptr(xhat), g[1],
                                                              _ptr(plan.plan_dev), plan.plan_host, plan.nseg,
                                                              _ptr(vals), _ptr(idx), _ptr(ws), ws.numel(),
                                                              _stream(dev)),
                       "choco_gossip_topk_compress_segmented")
        else:
            _lib.check(L.choco_topk_compress_segmented(_ptr(x), _ptr(xhat), _ptr(plan.plan_dev), plan.plan_host,
                                                       plan.nseg, _ptr(vals), _ptr(idx), _ptr(ws), ws.numel(),
                                                       _stream(dev)), "choco_topk_compress_segmented")
    except RuntimeError:
        # a call that failed part-way may leave the plan's histograms non-zero
        torch.cuda.synchronize(dev)
        plan.drop_workspace(dev)
        raise
    return vals, idx


# ----------------------------------------------------------------------------- random-k
def randk(x, k, seed, is_biased=True, xhat=None, offset=0, out=None):
    """Uniform random k-subset (include/choco_codec.h: the device sampler of (seed, offset)),
    values x[i] (- xhat[i]) (* n / k unbiased), int32 indices in ascending order;
    `out=(values f32[k], indices i32[k])` writes into caller buffers."""
    _require(x, torch.float32, "x")
    if xhat is not None:
        _require(xhat, torch.float32, "xhat")
        if xhat.numel() != x.numel():
            raise RuntimeError("x and xhat must have the same number of elements")
    n = x.numel()
    dev = x.device
    if out is not None:
        vals, idx = out
        _require(vals, torch.float32, "out values")
        _require(idx, torch.int32, "out indices")
        if vals.numel() != k or idx.numel() != k:
            raise RuntimeError("out buffers must hold exactly k elements")
    else:
        vals = torch.empty(k, dtype=torch.float32, device=dev)
        idx = torch.empty(k, dtype=torch.int32, device=dev)
    L = lib()
    ws = workspace(dev, "randk", L.choco_randk_workspace_size(n))
    _lib.check(L.choco_randk_compress(_ptr(x), _ptr(xhat), n, int(k), int(seed) & (2**64 - 1),
                                      int(offset) & (2**64 - 1), 1 if is_biased else 0, _ptr(vals), _ptr(idx),
                                      _ptr(ws), ws.numel(), _stream(dev)), "choco_randk_compress")
    return vals, idx


def randk_segmented(x, plan, seed, is_biased=True, xhat=None, out=None, gossip=None, offset=0):
    """Per-segment random-k over a SegmentPlan (k_s as top-k's), one batched call:
    segment s drawn with key derive(key(seed, offset), s); GLOBAL indices."""
    vals, idx = _seg_outputs(x, xhat, plan, out)
    dev = x.device
    L = lib()
    ws = plan.workspace(dev)
    g = _gossip(gossip, x, xhat)
    sd, off = int(seed) & (2**64 - 1), int(offset) & (2**64 - 1)
    if g is not None:
        _lib.check(L.choco_gossip_randk_compress_segmented(_ptr(x), _ptr(g[0]), _ptr(xhat), g[1],
                                                           _ptr(plan.plan_dev), plan.plan_host, plan.nseg, sd, off,
                                                           1 if is_biased else 0, _ptr(vals), _ptr(idx), _ptr(ws),
                                                           ws.numel(), _stream(dev)),
                   "choco_gossip_randk_compress_segmented")
    else:
        _lib.check(L.choco_randk_compress_segmented(_ptr(x), _ptr(xhat), _ptr(plan.plan_dev), plan.plan_host,
                                                    plan.nseg, sd, off, 1 if is_biased else 0, _ptr(vals), _ptr(idx),
                                                    _ptr(ws), ws.numel(), _stream(dev)),
                   "choco_randk_compress_segmented")
    return vals, idx


def gather(x, idx, scale=1.0, xhat=None):
    _require(x, torch.float32, "x")
    _require(idx, torch.int64, "idx")
    out = torch.empty(idx.numel(), dtype=torch.float32, device=x.device)
    _lib.check(lib().choco_gather(_ptr(x), _ptr(xhat), _ptr(idx), idx.numel(), float(scale), _ptr(out),
                                  _stream(x.device)), "choco_gather")
    return out


class IndexGuard:
    """Lazy check of the out-of-range index count that the sparse accumulate
    keeps in a device word (include/choco_codec.h): `arm()` queues a
    non-blocking copy of the word to pinned host memory behind the launches;
    `check()` raises RuntimeError -- the reference's index_put raises
    IndexError -- once that copy has landed with a count above what was already
    reported.  The count is cumulative (never reset on the device), so no error is
    lost between copies.  No host synchronisation on the hot path; callers check
    AFTER their own step's work is queued (a bad index of an earlier step must not
    stop this step's valid messages from being applied), and `check(wait=True)`
    copies and waits (teardown, checkpoints)."""

    def __init__(self, device):
        self.device = device
        self.word = torch.zeros(1, dtype=torch.int32, device=device)
        self.host = torch.zeros(1, dtype=torch.int32).pin_memory()
        self.event = None
        self.reported = 0

    def arm(self):
        self.host.copy_(self.word, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record(torch.cuda.current_stream(self.device))

    def check(self, wait=False):
        if wait and self.event is None:
            self.arm()
        if self.event is None:
            return
        if wait:
            self.event.synchronize()
        elif not self.event.query():
            return
        self.event = None
        bad = int(self.host.item()) & 0xFFFFFFFF
        if bad > self.reported:
            new, self.reported = bad - self.reported, bad
            raise RuntimeError(f"sparse accumulate: {new} received indices out of range or not ascending (corrupt "
                               "message or a peer with a different parameter layout); a corrupt message may already "
                               "have been applied")

    def check_then_arm(self):
        """End of a receiver step: report an EARLIER step's bad indices (this step's
        messages are already applied), then queue this step's copy."""
        try:
            self.check()
        finally:
            self.arm()


MAX_SPARSE_MSGS = 8  # messages per choco_sparse_accumulate_multi call


def sparse_accumulate_multi(messages, weights, memory, self_slot=-1, xhat_self=None, guard=None):
    """Every message of a receive step in ONE call (include/choco_codec.h
    choco_sparse_accumulate_multi): for m in order, x_hat[idx_m] += v_m (m == self_slot,
    xhat_self given) and memory[idx_m] += weights[m] * v_m -- bit-identical to one
    sparse_accumulate per message in that order (the per-message kernels run it).  messages: [(values f32, indices i32)];
    any count (chunks of MAX_SPARSE_MSGS, applied in order)."""
    _require(memory, torch.float32, "memory")
    if len(messages) != len(weights):
        raise RuntimeError("one weight per message")
    for v, i in messages:
        _require(v, torch.float32, "values")
        _require(i, torch.int32, "indices")
        if v.numel() != i.numel():
            raise RuntimeError("values and indices must have the same length")
    if xhat_self is not None:
        _require(xhat_self, torch.float32, "xhat_self")
        if xhat_self.numel() != memory.numel():
            raise RuntimeError("xhat_self and memory must have the same length")
    n = memory.numel()
    L = lib()
    dev = memory.device
    for c0 in range(0, len(messages), MAX_SPARSE_MSGS):
        part = messages[c0:c0 + MAX_SPARSE_MSGS]
        m = len(part)
        slot = self_slot - c0 if (xhat_self is not None and c0 <= self_slot < c0 + m) else -1
        nws = L.choco_sparse_accumulate_multi_workspace_size(n, m)
        ws = workspace(dev, "accm", nws) if nws else None
        vp, keep1 = _lib.ptr_array([v.data_ptr() for v, _ in part])
        ip, keep2 = _lib.ptr_array([i.data_ptr() for _, i in part])
        kp, keep3 = _lib.i64_array([v.numel() for v, _ in part])
        wp, keep4 = _lib.f32_array([float(w) for w in weights[c0:c0 + m]])
        _lib.check(L.choco_sparse_accumulate_multi(vp, ip, kp, wp, m, slot, _ptr(xhat_self if slot >= 0 else None),
                                                   _ptr(memory), n, _ptr(ws), ws.numel() if ws is not None else 0,
                                                   _ptr(guard.word) if guard is not None else ctypes.c_void_p(0),
                                                   _stream(dev)),
                   "choco_sparse_accumulate_multi")


def sparse_accumulate(values, indices, memory, weight, xhat_self=None, guard=None):
    """x_hat[idx] += v (xhat_self given); memory[idx] += weight * v.  Indices
    outside memory are skipped and counted into `guard` (an IndexGuard)."""
    _require(values, torch.float32, "values")
    _require(indices, torch.int32, "indices")
    _require(memory, torch.float32, "memory")
    if indices.numel() != values.numel():
        raise RuntimeError("values and indices must have the same length")
    if xhat_self is not None:
        _require(xhat_self, torch.float32, "xhat_self")
        if xhat_self.numel() != memory.numel():
            raise RuntimeError("xhat_self and memory must have the same length")
    _lib.check(lib().choco_sparse_accumulate(_ptr(values), _ptr(indices), values.numel(), _ptr(xhat_self),
                                             _ptr(memory), memory.numel(), float(weight),
                                             _ptr(guard.word) if guard is not None else ctypes.c_void_p(0),
                                             _stream(memory.device)),
               "choco_sparse_accumulate")


def sparse_extrapolate(values, indices, target, a, b, guard=None):
    """target[idx] = fmaf(b, v, target[idx] * a): ECD's replica update (ecd_psgd.py:299-303)."""
    _require(values, torch.float32, "values")
    _require(indices, torch.int32, "indices")
    _require(target, torch.float32, "target")
    if indices.numel() != values.numel():
        raise RuntimeError("values and indices must have the same length")
    _lib.check(lib().choco_sparse_extrapolate(_ptr(values), _ptr(indices), values.numel(), _ptr(target),
                                              target.numel(), float(a), float(b),
                                              _ptr(guard.word) if guard is not None else ctypes.c_void_p(0),
                                              _stream(target.device)), "choco_sparse_extrapolate")


# ----------------------------------------------------------------------------- sign
def sign_words(n):
    return int(lib().choco_sign_words(int(n)))


def _out_views(out, packed_n, packed_dtype, nseg, dev):
    """Caller-provided (packed, norms) buffers -- e.g. views into one wire message, so the
    kernels write the message in place instead of a torch.cat copying it afterwards."""
    packed, norms = out
    _require(packed, packed_dtype, "out packed")
    if packed.numel() != packed_n or packed.device != dev:
        raise RuntimeError(f"out packed must hold {packed_n} elements on {dev}")
    if norms is not None:
        _require(norms, torch.float32, "out norms")
        if norms.numel() != nseg or norms.device != dev:
            raise RuntimeError(f"out norms must hold {nseg} floats on {dev}")
    return packed, norms


def wire_header_words(nseg):
    """int32 words of a wire message's fp32 norms header (16-byte aligned)."""
    return (int(nseg) + 3) // 4 * 4


def sign_wire(n, nseg, dev):
    """One sign wire message [fp32 norms (16-B padded) | int32 words[N']] and the
    (packed, norms) views sign_compress(out=...) fills in place (header pad zeroed)."""
    hw = wire_header_words(nseg)
    msg = torch.empty(hw + sign_words(n), dtype=torch.int32, device=dev)
    msg[:hw].zero_()
    return msg, (msg[hw:], msg[:hw].view(torch.float32)[:nseg])


def sign_compress(x, xhat=None, seg_off=None, nseg=1, want_norms=True, gossip=None, out=None):
    """Pack sign bits in the (32, N') layout; optionally per-segment L1 norms (fp64-accumulated).
    `gossip=(memory, gamma)` fuses the consensus step; `out=(packed int32[N'], norms f32[nseg])`
    writes into caller buffers."""
    _require(x, torch.float32, "x")
    if xhat is not None:
        _require(xhat, torch.float32, "xhat")
    if seg_off is not None:
        _require(seg_off, torch.int64, "seg_off")
    n = x.numel()
    dev = x.device
    L = lib()
    if out is not None:
        packed, norms = _out_views(out, sign_words(n), torch.int32, nseg, dev)
    else:
        packed = torch.empty(sign_words(n), dtype=torch.int32, device=dev)
        norms = torch.empty(nseg, dtype=torch.float32, device=dev) if want_norms else None
    ws = workspace(dev, "acc", L.choco_sign_workspace_size(nseg))
    g = _gossip(gossip, x, xhat)
    if g is not None:
        _lib.check(L.choco_gossip_sign_compress(_ptr(x), _ptr(g[0]), _ptr(xhat), g[1], n, _ptr(seg_off), int(nseg),
                                                _ptr(packed), _ptr(norms), _ptr(ws), ws.numel(), _stream(dev)),
                   "choco_gossip_sign_compress")
        return packed, norms
    _lib.check(L.choco_sign_compress(_ptr(x), _ptr(xhat), n, _ptr(seg_off), int(nseg), _ptr(packed), _ptr(norms),
                                     _ptr(ws), ws.numel(), _stream(dev)), "choco_sign_compress")
    return packed, norms


SIGN_RANGE_ALIGN = 1024  # words per pack workgroup (sign.hip kSignCols)


def sign_chunks(n, chunks):
    """`chunks` word ranges [(w0, w1)] covering [0, N'), starts aligned to 1024 words."""
    words = sign_words(n)
    per = -(-words // max(1, int(chunks)))
    per = -(-per // SIGN_RANGE_ALIGN) * SIGN_RANGE_ALIGN
    return [(w, min(w + per, words)) for w in range(0, words, per)]


def sign_compress_range(x, w0, w1, finish, xhat=None, seg_off=None, nseg=1, gossip=None, out=None):
    """Pack the words [w0, w1) of sign_compress's layout into out=(packed int32[N'], norms
    f32[nseg] or None); the norms are written by the `finish` call, which must be the last
    range of the message on this stream (include/choco_codec.h "Chunked sign pack")."""
    _require(x, torch.float32, "x")
    if xhat is not None:
        _require(xhat, torch.float32, "xhat")
    if seg_off is not None:
        _require(seg_off, torch.int64, "seg_off")
    n = x.numel()
    dev = x.device
    L = lib()
    packed, norms = _out_views(out, sign_words(n), torch.int32, nseg, dev)
    ws = workspace(dev, "acc", L.choco_sign_workspace_size(nseg))
    g = _gossip(gossip, x, xhat)
    fin = 1 if finish else 0
    if g is not None:
        _lib.check(L.choco_gossip_sign_compress_range(_ptr(x), _ptr(g[0]), _ptr(xhat), g[1], n, _ptr(seg_off),
                                                      int(nseg), int(w0), int(w1), fin, _ptr(packed), _ptr(norms),
                                                      _ptr(ws), ws.numel(), _stream(dev)),
                   "choco_gossip_sign_compress_range")
    else:
        _lib.check(L.choco_sign_compress_range(_ptr(x), _ptr(xhat), n, _ptr(seg_off), int(nseg), int(w0), int(w1),
                                               fin, _ptr(packed), _ptr(norms), _ptr(ws), ws.numel(), _stream(dev)),
                   "choco_sign_compress_range")
    return packed, norms


def sign_unpack(packed, n):
    _require(packed, torch.int32, "packed")
    out = torch.empty(n, dtype=torch.float32, device=packed.device)
    _lib.check(lib().choco_sign_unpack(_ptr(packed), int(n), _ptr(out), _stream(packed.device)),
               "choco_sign_unpack")
    return out


MAX_FUSED_MSGS = 8  # messages one fused accumulate launch takes (sign.hip kMaxMsg, qsgd.hip kQMaxMsg)


def _msg_chunks(nmsg, self_slot):
    """Consecutive chunks of <= MAX_FUSED_MSGS messages, in order, with the local
    slot re-based into its chunk (-1 elsewhere).  memory is updated message by
    message, so chunked launches give the same fp32 sequence as one launch."""
    for c0 in range(0, nmsg, MAX_FUSED_MSGS):
        c1 = min(nmsg, c0 + MAX_FUSED_MSGS)
        yield c0, c1, (self_slot - c0) if c0 <= self_slot < c1 else -1


def _check_layout(memory, xhat_self, n, seg_off, nseg):
    if memory.numel() != n:
        raise RuntimeError(f"memory holds {memory.numel()} elements, the messages describe {n}")
    if xhat_self is not None:
        _require(xhat_self, torch.float32, "xhat_self")
        if xhat_self.numel() != n:
            raise RuntimeError("xhat_self and memory must have the same length")
    if nseg > 1:
        _require(seg_off, torch.int64, "seg_off")
        if seg_off.numel() != nseg + 1:
            raise RuntimeError("seg_off must hold nseg + 1 offsets")


def sign_accumulate(messages, weights, self_slot, n, memory, xhat_self=None, seg_off=None, nseg=1):
    """messages: list of (packed int32[N'], norms f32[nseg]) applied in order; any count
    (launched in fused chunks of MAX_FUSED_MSGS)."""
    _require(memory, torch.float32, "memory")
    _check_layout(memory, xhat_self, n, seg_off, nseg)
    if len(messages) != len(weights):
        raise RuntimeError("one weight per message")
    words = sign_words(n)
    for p, nm in messages:
        _require(p, torch.int32, "packed")
        _require(nm, torch.float32, "norms")
        if p.numel() != words or nm.numel() != nseg:
            raise RuntimeError(f"sign message must hold {words} words and {nseg} norms, got {p.numel()} / "
                               f"{nm.numel()}")
    for c0, c1, slot in _msg_chunks(len(messages), int(self_slot)):
        part = messages[c0:c1]
        pp, keep1 = _lib.ptr_array([p.data_ptr() for p, _ in part])
        nn, keep2 = _lib.ptr_array([nm.data_ptr() for _, nm in part])
        ww, keep3 = _lib.f32_array([float(w) for w in weights[c0:c1]])
        _lib.check(lib().choco_sign_decompress_accumulate(pp, nn, ww, len(part), slot, int(n), _ptr(seg_off),
                                                          int(nseg), _ptr(xhat_self if slot >= 0 else None),
                                                          _ptr(memory), ctypes.c_void_p(0), 0,
                                                          _stream(memory.device)),
                   "choco_sign_decompress_accumulate")


def sign_recv_gossip_compress(messages, weights, self_slot, x, memory, xhat, gamma, seg_off=None, nseg=1,
                              out=None):
    """The deferred receive fused into the next step's pass (include/choco_codec.h
    choco_sign_recv_gossip_compress): the previous step's messages [(packed, norms)] into
    x_hat (self_slot) and memory in order, then x += gamma (memory - x_hat), then this step's
    message (packed signs of x - x_hat, L1 norms) -- returned, or written to
    `out=(packed, norms)`, which must not be one of `messages`' buffers.  More than 8
    messages: the leading chunks are applied by sign_accumulate first (same order)."""
    _require(x, torch.float32, "x")
    _require(xhat, torch.float32, "xhat")
    _require(memory, torch.float32, "memory")
    n = x.numel()
    _check_layout(memory, xhat, n, seg_off, nseg)
    if len(messages) != len(weights) or not messages:
        raise RuntimeError("one weight per message, at least one message")
    words = sign_words(n)
    for p, nm in messages:
        _require(p, torch.int32, "packed")
        _require(nm, torch.float32, "norms")
        if p.numel() != words or nm.numel() != nseg:
            raise RuntimeError(f"sign message must hold {words} words and {nseg} norms")
    dev = x.device
    if out is not None:
        packed, norms = _out_views(out, words, torch.int32, nseg, dev)
    else:
        packed = torch.empty(words, dtype=torch.int32, device=dev)
        norms = torch.empty(nseg, dtype=torch.float32, device=dev)
    head = len(messages) - MAX_FUSED_MSGS
    if head > 0:  # leading messages first, in order
        sign_accumulate(messages[:head], weights[:head], self_slot, n, memory,
                        xhat_self=xhat if 0 <= self_slot < head else None, seg_off=seg_off, nseg=nseg)
        messages, weights, self_slot = messages[head:], weights[head:], self_slot - head
    slot = self_slot if 0 <= self_slot < len(messages) else -1
    L = lib()
    # (its own workspace: the accumulator block plus bit planes of the messages and the output)
    ws = workspace(dev, "signrecv", L.choco_sign_recv_workspace_size(n, nseg, len(messages)))
    pp, keep1 = _lib.ptr_array([p.data_ptr() for p, _ in messages])
    nn, keep2 = _lib.ptr_array([nm.data_ptr() for _, nm in messages])
    ww, keep3 = _lib.f32_array([float(w) for w in weights])
    _lib.check(L.choco_sign_recv_gossip_compress(pp, nn, ww, len(messages), slot, _ptr(x), _ptr(memory), _ptr(xhat),
                                                 float(gamma), n, _ptr(seg_off), int(nseg), _ptr(packed),
                                                 _ptr(norms), _ptr(ws), ws.numel(), _stream(dev)),
               "choco_sign_recv_gossip_compress")
    return packed, norms


def sign_axpy(messages, weights, n, target, seg_off=None, nseg=1, two_roundings=False):
    """target += w_m * decode(m) for each (packed, norms) message in order -- the receiver of
    the DCD / DeepSqueeze sign compressors; `two_roundings` selects torch's add_(w * u)
    over add_(u, alpha=w) (include/choco_codec.h)."""
    _require(target, torch.float32, "target")
    _check_layout(target, None, n, seg_off, nseg)
    if len(messages) != len(weights):
        raise RuntimeError("one weight per message")
    words = sign_words(n)
    for p, nm in messages:
        _require(p, torch.int32, "packed")
        _require(nm, torch.float32, "norms")
        if p.numel() != words or nm.numel() != nseg:
            raise RuntimeError(f"sign message must hold {words} words and {nseg} norms")
    for c0, c1, _ in _msg_chunks(len(messages), -1):
        part = messages[c0:c1]
        pp, keep1 = _lib.ptr_array([p.data_ptr() for p, _ in part])
        nn, keep2 = _lib.ptr_array([nm.data_ptr() for _, nm in part])
        ww, keep3 = _lib.f32_array([float(w) for w in weights[c0:c1]])
        _lib.check(lib().choco_sign_decompress_axpy(pp, nn, ww, len(part), int(n), _ptr(seg_off), int(nseg),
                                                    1 if two_roundings else 0, _ptr(target),
                                                    _stream(target.device)), "choco_sign_decompress_axpy")


def sign_extrapolate(packed, norms, n, target, a, b, seg_off=None, nseg=1):
    """target_s = target_s * a + ((b * norm_s) / numel_s) * sign: ECD (ecd_psgd.py:448-454)."""
    _require(packed, torch.int32, "packed")
    _require(norms, torch.float32, "norms")
    _require(target, torch.float32, "target")
    _check_layout(target, None, n, seg_off, nseg)
    _lib.check(lib().choco_sign_decompress_extrapolate(_ptr(packed), _ptr(norms), int(n), _ptr(seg_off), int(nseg),
                                                       float(a), float(b), _ptr(target), _stream(target.device)),
               "choco_sign_decompress_extrapolate")


def sign_local_decode(x, norms, seg_off=None, nseg=1):
    """(norm_s * torch.sign(x)) / numel_s: DeepSqueeze's local copy of its sign message."""
    _require(x, torch.float32, "x")
    _require(norms, torch.float32, "norms")
    out = torch.empty_like(x)
    _lib.check(lib().choco_sign_local_decode(_ptr(x), x.numel(), _ptr(seg_off), int(nseg), _ptr(norms), _ptr(out),
                                             _stream(x.device)), "choco_sign_local_decode")
    return out


# ----------------------------------------------------------------------------- QSGD
def qsgd_packed_bytes(n, q):
    return int(lib().choco_qsgd_packed_bytes(int(n), int(q)))


def qsgd_wire(n, q, nseg, dev):
    """One QSGD wire message [fp32 norms (16-B padded) | level plane | sign plane] (uint8)
    and the (packed, norms) views qsgd_compress(out=...) fills in place (header pad zeroed)."""
    hb = 4 * wire_header_words(nseg)
    msg = torch.empty(hb + qsgd_packed_bytes(n, q), dtype=torch.uint8, device=dev)
    msg[:hb].zero_()
    return msg, (msg[hb:], msg[:hb].view(torch.float32)[:nseg])


def qsgd_compress(x, q, is_biased=False, xhat=None, seg_off=None, nseg=1, norm_in=None, u_in=None,
                  seed=0, offset=0, want_dense=False, gossip=None, out=None):
    """QSGD with s = 2^q - 1.  Returns (packed uint8, norms f32[nseg], dense f32[n] or None).
    `gossip=(memory, gamma)` fuses the consensus step (device norms and uniforms only);
    `out=(packed uint8[qsgd_packed_bytes], norms f32[nseg])` writes into caller buffers."""
    _require(x, torch.float32, "x")
    if xhat is not None:
        _require(xhat, torch.float32, "xhat")
    if seg_off is not None:
        _require(seg_off, torch.int64, "seg_off")
    if norm_in is not None:
        _require(norm_in, torch.float32, "norm_in")
    if u_in is not None:
        _require(u_in, torch.float32, "u_in")
        if u_in.numel() != x.numel():
            raise RuntimeError("u_in must have one uniform per element")
    n = x.numel()
    dev = x.device
    L = lib()
    if out is not None:
        packed, norms = _out_views(out, qsgd_packed_bytes(n, q), torch.uint8, nseg, dev)
        if norms is None:
            raise RuntimeError("out norms is required")
    else:
        packed = torch.empty(qsgd_packed_bytes(n, q), dtype=torch.uint8, device=dev)
        norms = torch.empty(nseg, dtype=torch.float32, device=dev)
    dense = torch.empty(n, dtype=torch.float32, device=dev) if want_dense else None
    ws = workspace(dev, "acc", L.choco_qsgd_workspace_size(nseg))
    g = _gossip(gossip, x, xhat)
    if g is not None:
        if norm_in is not None or u_in is not None:
            raise RuntimeError("the fused gossip step takes the device norms and uniforms")
        _lib.check(L.choco_gossip_qsgd_compress(_ptr(x), _ptr(g[0]), _ptr(xhat), g[1], n, _ptr(seg_off), int(nseg),
                                                int(q), 1 if is_biased else 0, int(seed) & (2**64 - 1),
                                                int(offset) & (2**64 - 1), _ptr(packed), _ptr(norms), _ptr(dense),
                                                _ptr(ws), ws.numel(), _stream(dev)), "choco_gossip_qsgd_compress")
        return packed, norms, dense
    _lib.check(L.choco_qsgd_compress(_ptr(x), _ptr(xhat), n, _ptr(seg_off), int(nseg), int(q),
                                     1 if is_biased else 0, _ptr(norm_in), _ptr(u_in), int(seed) & (2**64 - 1),
                                     int(offset) & (2**64 - 1), _ptr(packed), _ptr(norms), _ptr(dense), _ptr(ws),
                                     ws.numel(), _stream(dev)), "choco_qsgd_compress")
    return packed, norms, dense


def qsgd_decode(packed, norms, n, q, is_biased=False, seg_off=None, nseg=1):
    _require(packed, torch.uint8, "packed")
    _require(norms, torch.float32, "norms")
    out = torch.empty(n, dtype=torch.float32, device=packed.device)
    _lib.check(lib().choco_qsgd_decode(_ptr(packed), _ptr(norms), int(n), _ptr(seg_off), int(nseg), int(q),
                                       1 if is_biased else 0, _ptr(out), _stream(packed.device)),
               "choco_qsgd_decode")
    return out


def qsgd_accumulate(messages, weights, self_slot, n, q, memory, xhat_self=None, is_biased=False, seg_off=None,
                    nseg=1):
    """messages: list of (packed uint8, norms f32[nseg]) applied in order; any count
    (launched in fused chunks of MAX_FUSED_MSGS)."""
    _require(memory, torch.float32, "memory")
    _check_layout(memory, xhat_self, n, seg_off, nseg)
    if len(messages) != len(weights):
        raise RuntimeError("one weight per message")
    nbytes = qsgd_packed_bytes(n, q)
    for p, nm in messages:
        _require(p, torch.uint8, "packed")
        _require(nm, torch.float32, "norms")
        if p.numel() != nbytes or nm.numel() != nseg:
            raise RuntimeError(f"QSGD message must hold {nbytes} bytes and {nseg} norms, got {p.numel()} / "
                               f"{nm.numel()}")
    for c0, c1, slot in _msg_chunks(len(messages), int(self_slot)):
        part = messages[c0:c1]
        pp, keep1 = _lib.ptr_array([p.data_ptr() for p, _ in part])
        nn, keep2 = _lib.ptr_array([nm.data_ptr() for _, nm in part])
        ww, keep3 = _lib.f32_array([float(w) for w in weights[c0:c1]])
        _lib.check(lib().choco_qsgd_decompress_accumulate(pp, nn, ww, len(part), slot, int(n), _ptr(seg_off),
                                                          int(nseg), int(q), 1 if is_biased else 0,
                                                          _ptr(xhat_self if slot >= 0 else None), _ptr(memory),
                                                          _stream(memory.device)),
                   "choco_qsgd_decompress_accumulate")


# ---- chunked QSGD wire (include/choco_codec.h "Chunked QSGD wire")
QSGD_RANGE_ALIGN = 8192


def qsgd_chunks(n, chunks):
    """`chunks` element ranges [(e0, e1)] covering [0, n), starts aligned to 8192."""
    per = -(-int(n) // max(1, int(chunks)))
    per = -(-per // QSGD_RANGE_ALIGN) * QSGD_RANGE_ALIGN
    return [(e, min(e + per, n)) for e in range(0, n, per)]


def qsgd_chunked_wire(n, q, nseg, chunks, dev):
    """One chunked QSGD message [fp32 norms (16-B padded) | range 0 | range 1 | ...], each
    range a self-contained [level plane | sign plane]; returns (message, norms view,
    [(e0, e1, range view)])."""
    hb = 4 * wire_header_words(nseg)
    ranges = qsgd_chunks(n, chunks)
    offs = [hb]
    for e0, e1 in ranges:
        offs.append(offs[-1] + qsgd_packed_bytes(e1 - e0, q))
    msg = torch.empty(offs[-1], dtype=torch.uint8, device=dev)
    msg[:hb].zero_()
    parts = [(e0, e1, msg[offs[i]:offs[i + 1]]) for i, (e0, e1) in enumerate(ranges)]
    return msg, msg[:hb].view(torch.float32)[:nseg], parts


def qsgd_norms(x, xhat=None, seg_off=None, nseg=1, gossip=None, out=None):
    """The QSGD norm pass alone (per-segment ||x - xhat||_2, fp64, rounded once);
    `gossip=(memory, gamma)` applies the consensus step to x in the same pass."""
    _require(x, torch.float32, "x")
    if xhat is not None:
        _require(xhat, torch.float32, "xhat")
    dev = x.device
    norms = out if out is not None else torch.empty(nseg, dtype=torch.float32, device=dev)
    _require(norms, torch.float32, "norms")
    L = lib()
    ws = workspace(dev, "acc", L.choco_qsgd_workspace_size(nseg))
    g = _gossip(gossip, x, xhat)
    if g is not None:
        _lib.check(L.choco_gossip_qsgd_norms(_ptr(x), _ptr(g[0]), _ptr(xhat), g[1], x.numel(), _ptr(seg_off),
                                             int(nseg), _ptr(norms), _ptr(ws), ws.numel(), _stream(dev)),
                   "choco_gossip_qsgd_norms")
    else:
        _lib.check(L.choco_qsgd_norms(_ptr(x), _ptr(xhat), x.numel(), _ptr(seg_off), int(nseg), _ptr(norms),
                                      _ptr(ws), ws.numel(), _stream(dev)), "choco_qsgd_norms")
    return norms


def qsgd_recv_gossip_norms(messages, weights, self_slot, x, memory, xhat, gamma, q, is_biased=False, seg_off=None,
                           nseg=1, out=None):
    """The deferred receive fused into the next step's first pass (include/choco_codec.h
    choco_qsgd_recv_gossip_norms): the previous step's messages [(packed, norms)] into x_hat
    (self_slot) and memory in order, then x += gamma (memory - x_hat), then this step's
    per-segment norms of x - x_hat (returned, or written to `out`).  More than 8 messages:
    the leading chunks are applied by qsgd_accumulate first (same order, same results)."""
    _require(x, torch.float32, "x")
    _require(xhat, torch.float32, "xhat")
    _check_layout(memory, xhat, x.numel(), seg_off, nseg)
    n = x.numel()
    if len(messages) != len(weights) or not messages:
        raise RuntimeError("one weight per message, at least one message")
    nbytes = qsgd_packed_bytes(n, q)
    for p, nm in messages:
        _require(p, torch.uint8, "packed")
        _require(nm, torch.float32, "norms")
        if p.numel() != nbytes or nm.numel() != nseg:
            raise RuntimeError(f"QSGD message must hold {nbytes} bytes and {nseg} norms")
    dev = x.device
    norms = out if out is not None else torch.empty(nseg, dtype=torch.float32, device=dev)
    _require(norms, torch.float32, "norms")
    head = len(messages) - MAX_FUSED_MSGS
    if head > 0:  # leading messages first, in order
        qsgd_accumulate(messages[:head], weights[:head], self_slot, n, q, memory, xhat_self=xhat,
                        is_biased=is_biased, seg_off=seg_off, nseg=nseg)
        messages, weights, self_slot = messages[head:], weights[head:], self_slot - head
    slot = self_slot if 0 <= self_slot < len(messages) else -1
    L = lib()
    ws = workspace(dev, "acc", L.choco_qsgd_workspace_size(nseg))
    pp, keep1 = _lib.ptr_array([p.data_ptr() for p, _ in messages])
    nn, keep2 = _lib.ptr_array([nm.data_ptr() for _, nm in messages])
    ww, keep3 = _lib.f32_array([float(w) for w in weights])
    _lib.check(L.choco_qsgd_recv_gossip_norms(pp, nn, ww, len(messages), slot, _ptr(x), _ptr(memory), _ptr(xhat),
                                              float(gamma), n, _ptr(seg_off), int(nseg), int(q),
                                              1 if is_biased else 0, _ptr(norms), _ptr(ws), ws.numel(),
                                              _stream(dev)), "choco_qsgd_recv_gossip_norms")
    return norms


def qsgd_quantize_range(x, q, norms, e0, e1, packed_range, is_biased=False, xhat=None, seg_off=None, nseg=1,
                        seed=0, offset=0):
    """Quantize elements [e0, e1) into `packed_range` (qsgd_packed_bytes(e1 - e0, q) bytes)."""
    _require(x, torch.float32, "x")
    _require(norms, torch.float32, "norms")
    _require(packed_range, torch.uint8, "packed_range")
    if packed_range.numel() != qsgd_packed_bytes(e1 - e0, q):
        raise RuntimeError("packed_range must hold qsgd_packed_bytes(e1 - e0, q) bytes")
    _lib.check(lib().choco_qsgd_quantize_range(_ptr(x), _ptr(xhat), x.numel(), _ptr(seg_off), int(nseg), int(q),
                                               1 if is_biased else 0, _ptr(norms), int(seed) & (2**64 - 1),
                                               int(offset) & (2**64 - 1), int(e0), int(e1), _ptr(packed_range),
                                               _stream(x.device)), "choco_qsgd_quantize_range")


def qsgd_accumulate_range(messages, weights, self_slot, n, q, memory, e0, e1, xhat_self=None, is_biased=False,
                          seg_off=None, nseg=1):
    """qsgd_accumulate over elements [e0, e1); messages: list of (range message, norms)."""
    _require(memory, torch.float32, "memory")
    _check_layout(memory, xhat_self, n, seg_off, nseg)
    if len(messages) != len(weights):
        raise RuntimeError("one weight per message")
    nbytes = qsgd_packed_bytes(e1 - e0, q)
    for p, nm in messages:
        _require(p, torch.uint8, "packed")
        _require(nm, torch.float32, "norms")
        if p.numel() != nbytes or nm.numel() != nseg:
            raise RuntimeError(f"QSGD range message must hold {nbytes} bytes and {nseg} norms")
    for c0, c1, slot in _msg_chunks(len(messages), int(self_slot)):
        part = messages[c0:c1]
        pp, keep1 = _lib.ptr_array([p.data_ptr() for p, _ in part])
        nn, keep2 = _lib.ptr_array([nm.data_ptr() for _, nm in part])
        ww, keep3 = _lib.f32_array([float(w) for w in weights[c0:c1]])
        _lib.check(lib().choco_qsgd_decompress_accumulate_range(
            pp, nn, ww, len(part), slot, int(n), _ptr(seg_off), int(nseg), int(q), 1 if is_biased else 0, int(e0),
            int(e1), _ptr(xhat_self if slot >= 0 else None), _ptr(memory), _stream(memory.device)),
            "choco_qsgd_decompress_accumulate_range")


def qsgd_extrapolate(packed, norms, n, q, target, a, b, is_biased=False, seg_off=None, nseg=1):
    """target = fmaf(b, decode(m), target * a): ECD (ecd_psgd.py:415-423)."""
    _require(packed, torch.uint8, "packed")
    _require(norms, torch.float32, "norms")
    _require(target, torch.float32, "target")
    _check_layout(target, None, n, seg_off, nseg)
    _lib.check(lib().choco_qsgd_decompress_extrapolate(_ptr(packed), _ptr(norms), int(n), _ptr(seg_off), int(nseg),
                                                       int(q), 1 if is_biased else 0, float(a), float(b),
                                                       _ptr(target), _stream(target.device)),
               "choco_qsgd_decompress_extrapolate")


# ----------------------------------------------------------------------------- gossip
def gossip_step(x, memory, xhat, gamma):
    for t, nm in ((x, "x"), (memory, "memory"), (xhat, "xhat")):
        _require(t, torch.float32, nm)
    _lib.check(lib().choco_gossip_step(_ptr(x), _ptr(memory), _ptr(xhat), float(gamma), x.numel(),
                                       _stream(x.device)), "choco_gossip_step")


# ----------------------------------------------------------------------------- profiling
def profile_enable(on=True):
    lib().choco_profile_enable(1 if on else 0)


def profile_filter(names=None):
    """Time only the launches named in `names` (a name or a list; None = all)."""
    if isinstance(names, (list, tuple)):
        names = ",".join(names)
    lib().choco_profile_filter(names.encode() if names else None)


def profile_read(name):
    total = ctypes.c_double(0.0)
    cnt = ctypes.c_int64(0)
    lib().choco_profile_read(name.encode(), ctypes.byref(total), ctypes.byref(cnt))
    return total.value, cnt.value


def profile_reset():
    lib().choco_profile_reset()


def launch_count(name):
    """Launches of kernel `name` since the library was loaded (counted with profiling off)."""
    return int(lib().choco_launch_count(name.encode()))


def topk_workspace_word(off, dev=None, plan=None):
    """Diagnostic: the uint32 at byte `off` of this stream's flat top-k workspace (or of
    `plan`'s segmented one); include/choco_codec.h CHOCO_TOPK_*_OFFSET.  Synchronises."""
    dev = torch.device(dev) if dev is not None else torch.device("cuda", torch.cuda.current_device())
    if plan is not None:
        ws = plan.workspace(dev)
    else:
        with _ws_lock:
            ws = _ws_cache.get((dev.index, torch.cuda.current_stream(dev).cuda_stream, "topk"))
        if ws is None:
            return 0
    torch.cuda.current_stream(dev).synchronize()
    return int(ws[off:off + 4].view(torch.int32).item())


def is_pow2_minus1(s):
    return s >= 1 and (s + 1) & s == 0 and int(math.log2(s + 1)) <= 16
