"""Build diagnostic variants of the codec (K2 ablations / tuning knobs) into
chocosgd_amd/lib/variants/ for tools/diag_stream.py.  Never loaded by the product."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import build  # noqa: E402

VARIANTS = {
    "stamps": ["CHOCO_STAMPS=1"],
    "acc_elem": ["CHOCO_ACC_MODE=0"],
    "acc_seg8": ["CHOCO_ACC_SEGF=8"],
    "acc_seg32": ["CHOCO_ACC_SEGF=32"],
    "qq_nt": ["CHOCO_QQUANT_NT=1"],
    "qq_fwd": ["CHOCO_QQUANT_REV=0"],
    "rk_q2": ["CHOCO_RK_Q=2"],
    "rk_q8": ["CHOCO_RK_Q=8"],
    "rk_q16": ["CHOCO_RK_Q=16"],
    "seg_wnt0": ["CHOCO_SEG_WARM_NT=0"],
    "acc_nt1": ["CHOCO_ACC_NT=1"],
    "acc_next0": ["CHOCO_ACC_NEXT=0"],
    "acc_nt2": ["CHOCO_ACC_NT=2"],
    "qn_t48k": ["CHOCO_QNORM_TILE=49152"],
    "qn_t64k": ["CHOCO_QNORM_TILE=65536"],
    "seg512_w6": ["CHOCO_SEG_THREADS=512", "CHOCO_SEG_WPE=6"],
    "seg512_w5": ["CHOCO_SEG_THREADS=512", "CHOCO_SEG_WPE=5"],
    "seg512_w4": ["CHOCO_SEG_THREADS=512", "CHOCO_SEG_WPE=4"],
    "qq_fwd_nt": ["CHOCO_QQUANT_REV=0", "CHOCO_QQUANT_NT=1"],
    "qn_plain": ["CHOCO_QNORM_NT=0"],
    "sign_acc1": ["CHOCO_SIGN_ACC1=1"],
    "g_form0": ["CHOCO_GOSSIP_FORM=0"],
    "gs_st_plain": ["CHOCO_GS_STORE_NT=0"],
    "wide_debug": ["CHOCO_WIDE_DEBUG=1"],
    "qdec_nt": ["CHOCO_QDEC_ST_NT=1"],
    "qn_plain_qdec_nt": ["CHOCO_QNORM_NT=0", "CHOCO_QDEC_ST_NT=1"],
    "s1_c2": ["CHOCO_S1_COPIES=2"],
    "s1_c4": ["CHOCO_S1_COPIES=4"],
    "s4_1024": ["CHOCO_S4_THREADS=1024"],
    "s1_lc2": ["CHOCO_S1_LANEC=2"],
    "s1_lc4": ["CHOCO_S1_LANEC=4"],
    "s1_lc8": ["CHOCO_S1_LANEC=8"],
    "k2st_nt": ["CHOCO_K2_STORE=1"],
    "k2st_wt": ["CHOCO_K2_STORE=2"],
    "k34st_nt": ["CHOCO_K34_STORE=1"],
    "k34st_wt": ["CHOCO_K34_STORE=2"],
    "s4_128": ["CHOCO_S4_THREADS=128"],
    "s4_64": ["CHOCO_S4_THREADS=64"],
    "s3_128": ["CHOCO_S3_THREADS=128"],
    "s3_64": ["CHOCO_S3_THREADS=64"],
    "sacc_rg32": ["CHOCO_SIGN_ACC_RG=32"],
    "sacc_rg16": ["CHOCO_SIGN_ACC_RG=16"],
    "sacc_rg4": ["CHOCO_SIGN_ACC_RG=4"],
    "sgs_ru4": ["CHOCO_SIGN_GS_RU=4"],
    "sgs_split": ["CHOCO_SIGN_GS_FUSE=0"],
    "k2t384": ["CHOCO_K2_TARGET=384"],
    "k2t512": ["CHOCO_K2_TARGET=512"],
    "k2t768": ["CHOCO_K2_TARGET=768"],
    "k2t1024": ["CHOCO_K2_TARGET=1024"],
    # every bounded wait of the exact fallback gives up at once: tools/status_probe.py
    "poll1": ["CHOCO_POLL_BUDGET=1"],
    "qq_loop1": ["CHOCO_QQ_LOOP=1"],
    "qq_loop1_g512": ["CHOCO_QQ_LOOP=1", "CHOCO_QQ_GRID=512"],
    "qq_loop1_g2048": ["CHOCO_QQ_LOOP=1", "CHOCO_QQ_GRID=2048"],
    "qcheck0": ["CHOCO_QCHECK=0"],
    "seg_loop1": ["CHOCO_SEG_LOOP=1"],
    "seg_sf0": ["CHOCO_SEG_SMALL_FIRST=0"],
    "k2wf0": ["CHOCO_K2_WINDOW_FIRST=0"],
    "k34ws1": ["CHOCO_K34_WAVE_SELECT=1"],
    "seg_loop1_g512": ["CHOCO_SEG_LOOP=1", "CHOCO_SEG_LOOP_GRID=512"],
    "qq_h0": ["CHOCO_QQ_HALF=0"],
    # timing diagnostics only, WRONG results (never in a parity run)
    "qqdiag_coal": ["CHOCO_QQ_DIAG_COAL=1"],
    "qqdiag_nomath": ["CHOCO_QQ_DIAG_NOMATH=1"],
    "qqdiag_coal_nomath": ["CHOCO_QQ_DIAG_COAL=1", "CHOCO_QQ_DIAG_NOMATH=1"],
    "qqdiag_loadonly": ["CHOCO_QQ_DIAG_NOMATH=2"],
    "qqdiag_nomath_nt": ["CHOCO_QQ_DIAG_NOMATH=1", "CHOCO_QQUANT_NT=1"],
    "qqdiag_nomath_fwd": ["CHOCO_QQ_DIAG_NOMATH=1", "CHOCO_QQUANT_REV=0"],
    "qqdiag_nomath_h0": ["CHOCO_QQ_DIAG_NOMATH=1", "CHOCO_QQ_HALF=0"],
    "qq_nt_h": ["CHOCO_QQUANT_NT=1"],
    "qn_plain_qq_nt": ["CHOCO_QNORM_NT=0", "CHOCO_QQUANT_NT=1"],
    "qq_loop_asm": ["CHOCO_QQ_LOOP=1", "CHOCO_QQ_LOOP_ASM=1"],
    "qq_loop_asm_g512": ["CHOCO_QQ_LOOP=1", "CHOCO_QQ_LOOP_ASM=1", "CHOCO_QQ_GRID=512"],
    "qq_fwd_h": ["CHOCO_QQUANT_REV=0"],
    "qq_ring_d3w3": ["CHOCO_QQ_RING=1", "CHOCO_QQ_RING_D=3", "CHOCO_QQ_RING_WGS=3"],
    "qq_ring_d2w4": ["CHOCO_QQ_RING=1", "CHOCO_QQ_RING_D=2", "CHOCO_QQ_RING_WGS=4"],
    "qq_hw8": ["CHOCO_QQ_HWAVES=8"],
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
