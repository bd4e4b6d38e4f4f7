#!/bin/bash
# Multi-rank rehearsal on one card (gloo, ranks share cuda:0), then the QSGD rows re-measured.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4x; mkdir -p $O
for spec in "topk 2" "topk 3" "topk_r50 2" "qsgd 2" "sign 2" "step_topk 2" "step_qsgd 2" "randk 2"; do
  set -- $spec
  timeout -k 10 240 python bench.py --workload $1 --gpus $2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/$1_$2.json 2> $O/$1_$2.err \
    || { echo "FAIL $1 $2"; tail -20 $O/$1_$2.err; exit 1; }
  echo "$1 x$2: $(tail -1 $O/$1_$2.json | cut -c1-220)"
done
WLS="qsgd step_qsgd" R=r04 bash scripts/gpu_measure.sh
