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
