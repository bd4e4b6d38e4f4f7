#!/bin/bash
# QSGD quantize timing diagnostics (variants with WRONG results, bench timing only).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4y; mkdir -p $O
summ() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', d['kernels_us'])"; }
for rep in 1 2; do
  for v in default qqdiag_nomath qqdiag_loadonly qqdiag_nomath_nt qqdiag_nomath_fwd qqdiag_nomath_h0 qq_nt_h qq_fwd_h; do
    L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
    timeout -k 10 120 python bench.py --workload qsgd --steps 10 --warmup 4 --no-cpu-baseline --no-e2e $L > $O/qsgd_$v.json 2>$O/qsgd_$v.err || { tail -5 $O/qsgd_$v.err; exit 1; }
    summ $O/qsgd_$v.json qsgd_$v
  done
done
