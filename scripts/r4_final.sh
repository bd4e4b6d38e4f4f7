#!/bin/bash
# Final tree: the whole -m gpu suite + smoke, then the QSGD workloads re-measured (quantize changed).
cd $GRAFT_REPO_ROOT
bash scripts/r4_full.sh || exit $?
WLS="qsgd step_qsgd" R=r04 bash scripts/gpu_measure.sh
