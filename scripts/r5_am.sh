#!/bin/bash
# Round-5 GPU pass AM: per-tensor (ResNet-50) random-k beside flat random-k at 25.6M and 100M.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5am; mkdir -p $O
for spec in randk_r50 "randk --n 25557032" randk; do
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec', d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
