"""Back-to-back top-k stream kernel (K2) alone vs inside the full call, for a few
ratios (CHOCO_STAMPS diagnostic build only)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import _lib, codec  # noqa: E402

_lp = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else "chocosgd_amd/lib/variants/lib_stamps.so"
lib = _lib.load(os.path.join(ROOT, _lp))
fn = lib.choco_dbg_stream_only
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32,
               ctypes.POINTER(ctypes.c_double), ctypes.c_void_p]
dev = torch.device("cuda", 0)
n = 100_000_000
for dist in ("randn", "zeros+1"):
    d = torch.randn(n, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    for ratio in (0.99999999, 0.99, 0.9):
        k = codec.topk_k(n, ratio)
        codec.topk(d, k)
        torch.cuda.synchronize()
        ws = codec.workspace(dev, "topk", lib.choco_topk_workspace_size(n))
        ms = ctypes.c_double()
        rc = fn(d.data_ptr(), n, k, ws.data_ptr(), ws.numel(), 20, ctypes.byref(ms),
                torch.cuda.current_stream().cuda_stream)
        assert rc == 0, _lib.last_error()
        print(f"{dist:8s} ratio {ratio}: stream kernel alone, back to back: {ms.value * 1e3:7.1f} us "
              f"({4 * n / ms.value / 1e6:6.0f} GB/s)", flush=True)
    break
