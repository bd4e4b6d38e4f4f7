#!/bin/bash
# Round-5 GPU pass AF: the fused top-k step on ResNet-50's per-tensor layout (the drop-in's CHOCO top-k path),
# fused and unfused, beside the flat 100M step.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5af; mkdir -p $O
for rep in 1 2; do
for spec in "step_topk_r50" "step_topk_r50 --unfused" "topk_r50" "step_topk"; do
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec', d['ms_per_step'], d['roofline']['frac'], d['kernels_us'], d.get('cold_start'))"
done
done
