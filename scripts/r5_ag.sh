#!/bin/bash
# Round-5 GPU pass AG: the full GPU suite + smoke on the current tree, then the per-tensor (ResNet-50) compress /
# decompress rounds of sign and QSGD without the consensus step.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5ag; mkdir -p $O
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for spec in sign_r50 qsgd_r50 topk_r50; do
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec', d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
