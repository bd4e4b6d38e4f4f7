#!/bin/bash
# Round-5 GPU pass AV: the QSGD decode's loads + stores non-temporal (variant qdecnt2), whole steps.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5av; mkdir -p $O; V=chocosgd_amd/lib/variants
for rep in 1 2 3; do
for v in base qdecnt2; do
for spec in qsgd step_qsgd qsgd_r50; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec $v', d['ms_per_step'], d['kernels_us'])"
done
done
done
