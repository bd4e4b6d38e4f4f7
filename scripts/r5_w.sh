#!/bin/bash
# Round-5 GPU pass W: row-run sign receive knobs (cache policy, grid-stride vs one workgroup per run) A/B on
# step_sign --defer-receive, against the column-tile receive (signcols).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5w; mkdir -p $O; V=chocosgd_amd/lib/variants
for rep in 1 2; do
for v in base rows_plain rows_one rows_one_plain rows_g1024 signcols; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload step_sign --defer-receive --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('step_sign+defer $v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
