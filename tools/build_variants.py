"""Build diagnostic variants of the codec (K2 ablations / tuning knobs) into
chocosgd_amd/lib/variants/ for tools/diag_stream.py.  Never loaded by the product."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import build  # noqa: E402

VARIANTS = {
    "stamps": ["CHOCO_STAMPS=1"],
    "stream_nt": ["CHOCO_STREAM_NT=1"],
    "chunk4k": ["CHOCO_K2_CHUNK=4096"],
    "nopf": ["CHOCO_K34_PREFETCH=0"],
    "earlypf": ["CHOCO_K34_PREFETCH=1"],
    "qn_plain": ["CHOCO_QNORM_NT=0"],
    "sign_plain": ["CHOCO_SIGN_NT=0"],
    "qq_nt": ["CHOCO_QQUANT_NT=1"],
    "acc_u4": ["CHOCO_ACC_U=4"],
    "acc_u8": ["CHOCO_ACC_U=8"],
    "acc_u16": ["CHOCO_ACC_U=16"],
    "s32k": ["CHOCO_SAMPLE_RUNS=128"],
    "s32k_nopf": ["CHOCO_SAMPLE_RUNS=128", "CHOCO_K34_PREFETCH=0"],
    "stamps_s32k": ["CHOCO_STAMPS=1", "CHOCO_SAMPLE_RUNS=128"],
    "stamps4k": ["CHOCO_STAMPS=1", "CHOCO_K2_CHUNK=4096"],
    "nob1": ["CHOCO_STAMPS=1", "CHOCO_DIAG_NOBURST=1"],
    "nob2": ["CHOCO_STAMPS=1", "CHOCO_DIAG_NOBURST=2"],
    "nob3": ["CHOCO_STAMPS=1", "CHOCO_DIAG_NOBURST=3"],
    "k2st_nt": ["CHOCO_K2_STORE=1"],
    "k2st_sc1": ["CHOCO_K2_STORE=2"],
}


def main(names):
    out = os.path.join(build.LIBDIR, "variants")
    names = names or list(VARIANTS)

    def one(nm):
        return build.build_library(force=True, defines=VARIANTS[nm], lib=os.path.join(out, f"lib_{nm}.so"), jobs=2)
    with ThreadPoolExecutor(4) as ex:
        for p in ex.map(one, names):
            print(p)


if __name__ == "__main__":
    main(sys.argv[1:])
