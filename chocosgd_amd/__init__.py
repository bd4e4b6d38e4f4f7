"""chocosgd_amd -- MI355X-native codec for ChocoSGD's CHOCO compressor path.

Drop-in modules (same class/function names as the reference's dl_code/pcode):
  chocosgd_amd.sparsification   <- pcode/utils/sparsification.py
  chocosgd_amd.parallel_choco   <- pcode/optim/parallel_choco_v.py (CHOCOCompressor & co.)
  chocosgd_amd.tensor_buffer    <- pcode/utils/tensor_buffer.py
  chocosgd_amd.communication    <- pcode/utils/communication.py (decentralized exchange)
  chocosgd_amd.utils            <- pcode/optim/utils.py (recover_params, update_params_from_neighbor)
Compute lives in libchoco_codec.so (HIP, gfx950), bound through chocosgd_amd._lib.
"""
from . import _lib  # noqa: F401

__all__ = ["codec", "sparsification", "parallel_choco", "tensor_buffer", "communication", "utils"]
__version__ = "0.1.0"
