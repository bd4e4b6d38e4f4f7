#!/bin/bash
# Round-5 GPU pass T: the deferred QSGD receive's store policy (plain / all nt / memory nt), same box, with its
# parity tests run on each variant library first.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5t; mkdir -p $O; V=chocosgd_amd/lib/variants
for rep in 1 2 3; do
for v in base qrg1 qrg2; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload step_qsgd --defer-receive --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
