"""Build diagnostic variants of the codec (K2 ablations / tuning knobs) into
chocosgd_amd/lib/variants/ for tools/diag_stream.py.  Never loaded by the product."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chocosgd_amd import build  # noqa: E402

# (Round 5 removed the measured-slower and wrong-result knobs from the product sources;
# the variants that built them live in git history, r02-r04.)
VARIANTS = {
    "stamps": ["CHOCO_STAMPS=1"],
    # every bounded wait of the exact fallback gives up at once: tools/status_probe.py
    "poll1": ["CHOCO_POLL_BUDGET=1"],
    # round 6 A/B: the fused sign pack's x store with the row offset as soffset (round 5)
    "st_soff": ["CHOCO_AB_SIGN_ST_SOFF=1"],
    # round 6 A/B (timing only, unordered output): K2 streams strided 32768-element blocks
    "k2strided": ["CHOCO_AB_K2_STRIDED=1"],
    # round 6 A/B: K2's tile-end burst (pairs, side list) with non-temporal stores
    "k2ntst": ["CHOCO_AB_K2_NTST=1"],
    # round 6 A/B (timing only, wrong output): K34B without the per-block loads / the block search
    "k34b_nogt": ["CHOCO_AB_K34B_NOGT=1"],
    "k34b_nosearch": ["CHOCO_AB_K34B_NOSEARCH=1"],
    "k34b_both": ["CHOCO_AB_K34B_NOGT=1", "CHOCO_AB_K34B_NOSEARCH=1"],
    "k2strided_ntst": ["CHOCO_AB_K2_STRIDED=1", "CHOCO_AB_K2_NTST=1"],
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
