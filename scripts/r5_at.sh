#!/bin/bash
# Round-5 GPU pass AT: sign accumulate, non-temporal loads + stores (saccnt2) against plain, more passes.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5at; mkdir -p $O; V=chocosgd_amd/lib/variants
for rep in 1 2 3 4; do
for v in base saccnt2; do
for spec in sign step_sign sign_r50; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec $v', d['ms_per_step'], d['kernels_us'])"
done
done
done
