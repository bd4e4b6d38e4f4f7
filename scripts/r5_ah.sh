#!/bin/bash
# Round-5 GPU pass AH: sign / QSGD compress at 25.6M -- per-tensor layout against a flat buffer of the same size.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5ah; mkdir -p $O
for spec in "sign_r50" "sign --n 25557032" "qsgd_r50" "qsgd --n 25557032" "step_sign --n 25557032" "step_qsgd --n 25557032"; do
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec', d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
