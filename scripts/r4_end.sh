#!/bin/bash
# End of round: the whole -m gpu suite + smoke on the final tree, then the random-k row re-measured.
cd $GRAFT_REPO_ROOT
bash scripts/r4_full.sh || exit $?
WLS="randk" R=r04 bash scripts/gpu_measure.sh
