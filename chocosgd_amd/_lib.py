"""ctypes binding of libchoco_codec.so (the C ABI declared in include/choco_codec.h).

This is the same binding a maintainer would add to the reference (see
INTEGRATION.md).  There is no fallback: if the HIP library is missing or a
call fails, a RuntimeError is raised -- the reference's compressor pipelines
catch exactly RuntimeError (dl_code/pcode/optim/parallel_choco_v.py:226-227).
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# CHOCO_CODEC_LIB: another build of the same ABI (the A/B variants of tools/build_variants.py)
LIB_PATH = os.environ.get("CHOCO_CODEC_LIB") or os.path.join(_HERE, "lib", "libchoco_codec.so")

TOPK_STATUS_OFFSET = 0        # CHOCO_TOPK_STATUS_OFFSET
TOPK_FALLBACKS_OFFSET = 4     # CHOCO_TOPK_FALLBACKS_OFFSET
TOPK_COLD_LEFT_OFFSET = 8     # CHOCO_TOPK_COLD_LEFT_OFFSET
TOPK_K2_SAMPLES_OFFSET = 16   # CHOCO_TOPK_K2_SAMPLES_OFFSET
TOPK_STATUS_POLL_TIMEOUT = 1  # CHOCO_TOPK_STATUS_POLL_TIMEOUT

_c_i32, _c_i64, _c_u64, _c_f32, _c_f64 = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64,
                                           ctypes.c_float, ctypes.c_double)
_c_sz, _vp = ctypes.c_size_t, ctypes.c_void_p
_pp = ctypes.POINTER(ctypes.c_void_p)
_p_i64 = ctypes.POINTER(ctypes.c_int64)
_p_f32 = ctypes.POINTER(ctypes.c_float)

# name -> (restype, argtypes); mirrors include/choco_codec.h one to one
SIGNATURES = {
    "choco_version": (_c_i32, []),
    "choco_last_error": (_c_i32, [ctypes.c_char_p, _c_sz]),
    "choco_topk_k": (_c_i64, [_c_i64, _c_f64]),
    "choco_topk_workspace_size": (_c_sz, [_c_i64]),
    "choco_topk_workspace_reset": (_c_i32, [_vp, _c_sz]),
    "choco_topk_set_warm_start": (_c_i32, [_c_i32]),
    "choco_topk_host_status": (_c_i32, [_vp, _c_i32, _vp]),
    "choco_topk_compress": (_c_i32, [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_topk_compress_accumulate": (_c_i32, [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_f32, _vp, _c_sz,
                                                _vp]),
    "choco_topk_segmented_plan_len": (_c_i64, [_p_i64, _c_i32]),
    "choco_topk_segmented_plan": (_c_i64, [_p_i64, _c_i32, _c_f64, _p_i64]),
    "choco_topk_segmented_workspace_size": (_c_sz, [_p_i64, _c_i32]),
    "choco_topk_compress_segmented": (_c_i32, [_vp, _vp, _vp, _p_i64, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_randk_workspace_size": (_c_sz, [_c_i64]),
    "choco_randk_compress": (_c_i32, [_vp, _vp, _c_i64, _c_i64, _c_u64, _c_u64, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_randk_compress_segmented": (_c_i32, [_vp, _vp, _vp, _p_i64, _c_i32, _c_u64, _c_u64, _c_i32, _vp, _vp, _vp,
                                                _c_sz, _vp]),
    "choco_gather": (_c_i32, [_vp, _vp, _vp, _c_i64, _c_f32, _vp, _vp]),
    "choco_sparse_accumulate": (_c_i32, [_vp, _vp, _c_i64, _vp, _vp, _c_i64, _c_f32, _vp, _vp]),
    "choco_sparse_accumulate_multi_workspace_size": (_c_sz, [_c_i64, _c_i32]),
    "choco_sparse_accumulate_multi": (_c_i32, [_pp, _pp, _p_i64, _p_f32, _c_i32, _c_i32, _vp, _vp, _c_i64, _vp,
                                               _c_sz, _vp, _vp]),
    "choco_sign_words": (_c_i64, [_c_i64]),
    "choco_sign_workspace_size": (_c_sz, [_c_i32]),
    "choco_sign_compress": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_sign_compress_range": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i32, _c_i64, _c_i64, _c_i32, _vp, _vp, _vp,
                                           _c_sz, _vp]),
    "choco_sign_unpack": (_c_i32, [_vp, _c_i64, _vp, _vp]),
    "choco_sign_decompress_accumulate": (_c_i32, [_pp, _pp, _p_f32, _c_i32, _c_i32, _c_i64, _vp, _c_i32,
                                                  _vp, _vp, _vp, _c_sz, _vp]),
    "choco_sign_recv_workspace_size": (_c_sz, [_c_i64, _c_i32, _c_i32]),
    "choco_sign_recv_gossip_compress": (_c_i32, [_pp, _pp, _p_f32, _c_i32, _c_i32, _vp, _vp, _vp, _c_f32, _c_i64,
                                                 _vp, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_sign_decompress_axpy": (_c_i32, [_pp, _pp, _p_f32, _c_i32, _c_i64, _vp, _c_i32, _c_i32, _vp, _vp]),
    "choco_sign_decompress_extrapolate": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i32, _c_f32, _c_f32, _vp, _vp]),
    "choco_qsgd_decompress_extrapolate": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i32, _c_i32, _c_i32, _c_f32, _c_f32,
                                                   _vp, _vp]),
    "choco_sparse_extrapolate": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i64, _c_f32, _c_f32, _vp, _vp]),
    "choco_sign_local_decode": (_c_i32, [_vp, _c_i64, _vp, _c_i32, _vp, _vp, _vp]),
    "choco_qsgd_packed_bytes": (_c_i64, [_c_i64, _c_i32]),
    "choco_qsgd_workspace_size": (_c_sz, [_c_i32]),
    "choco_qsgd_compress": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i32, _c_i32, _c_i32, _vp, _vp, _c_u64, _c_u64,
                                     _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_qsgd_decode": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i32, _c_i32, _c_i32, _vp, _vp]),
    "choco_qsgd_decompress_accumulate": (_c_i32, [_pp, _pp, _p_f32, _c_i32, _c_i32, _c_i64, _vp, _c_i32,
                                                  _c_i32, _c_i32, _vp, _vp, _vp]),
    "choco_qsgd_norms": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i32, _vp, _vp, _c_sz, _vp]),
    "choco_qsgd_recv_gossip_norms": (_c_i32, [_pp, _pp, _p_f32, _c_i32, _c_i32, _vp, _vp, _vp, _c_f32, _c_i64, _vp,
                                              _c_i32, _c_i32, _c_i32, _vp, _vp, _c_sz, _vp]),
    "choco_gossip_qsgd_norms": (_c_i32, [_vp, _vp, _vp, _c_f32, _c_i64, _vp, _c_i32, _vp, _vp, _c_sz, _vp]),
    "choco_qsgd_quantize_range": (_c_i32, [_vp, _vp, _c_i64, _vp, _c_i32, _c_i32, _c_i32, _vp, _c_u64, _c_u64,
                                           _c_i64, _c_i64, _vp, _vp]),
    "choco_qsgd_decompress_accumulate_range": (_c_i32, [_pp, _pp, _p_f32, _c_i32, _c_i32, _c_i64, _vp, _c_i32,
                                                        _c_i32, _c_i32, _c_i64, _c_i64, _vp, _vp, _vp]),
    "choco_gossip_step": (_c_i32, [_vp, _vp, _vp, _c_f32, _c_i64, _vp]),
    "choco_gossip_topk_compress": (_c_i32, [_vp, _vp, _vp, _c_f32, _c_i64, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_gossip_topk_compress_accumulate": (_c_i32, [_vp, _vp, _vp, _c_f32, _c_i64, _c_i64, _vp, _vp, _c_i32,
                                                       _c_f32, _vp, _c_sz, _vp]),
    "choco_gossip_topk_compress_segmented": (_c_i32, [_vp, _vp, _vp, _c_f32, _vp, _p_i64, _c_i32, _vp, _vp, _vp,
                                                      _c_sz, _vp]),
    "choco_gossip_randk_compress_segmented": (_c_i32, [_vp, _vp, _vp, _c_f32, _vp, _p_i64, _c_i32, _c_u64, _c_u64,
                                                       _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_gossip_sign_compress": (_c_i32, [_vp, _vp, _vp, _c_f32, _c_i64, _vp, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_gossip_sign_compress_range": (_c_i32, [_vp, _vp, _vp, _c_f32, _c_i64, _vp, _c_i32, _c_i64, _c_i64,
                                                  _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_gossip_qsgd_compress": (_c_i32, [_vp, _vp, _vp, _c_f32, _c_i64, _vp, _c_i32, _c_i32, _c_i32, _c_u64,
                                            _c_u64, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "choco_profile_enable": (_c_i32, [_c_i32]),
    "choco_profile_filter": (_c_i32, [ctypes.c_char_p]),
    "choco_profile_read": (_c_i32, [ctypes.c_char_p, ctypes.POINTER(_c_f64), ctypes.POINTER(_c_i64)]),
    "choco_profile_reset": (_c_i32, []),
    "choco_launch_count": (_c_i64, [ctypes.c_char_p]),
}

_lib = None
_lock = threading.Lock()


def load(path=LIB_PATH):
    """Load (once) and type the shared library; raises RuntimeError if absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"chocosgd_amd: HIP codec library not found at {path}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error():
    lib = load()
    buf = ctypes.create_string_buffer(1024)
    lib.choco_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (status {rc}): {last_error()}")
    return rc


def ptr_array(ptrs):
    arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
    return ctypes.cast(arr, _pp), arr


def f32_array(vals):
    arr = (ctypes.c_float * len(vals))(*vals)
    return ctypes.cast(arr, _p_f32), arr


def i64_array(vals):
    arr = (ctypes.c_int64 * len(vals))(*vals)
    return ctypes.cast(arr, _p_i64), arr
