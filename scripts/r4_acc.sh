#!/bin/bash
# Sparse accumulate store policy in the top-k step (write-back placement): plain / nt / write-through.
# (prepared at the end of round 4; the pool was busy, not yet run -- next round)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4acc; mkdir -p $O
summ() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', d['ms_per_step'], d['kernels_us'])"; }
for rep in 1 2 3; do
  for wl in topk step_topk; do
    for v in default acc_nt1 acc_nt2; do
      L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
      timeout -k 10 120 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e $L > $O/${wl}_$v.json 2>$O/${wl}_$v.err || { tail -5 $O/${wl}_$v.err; exit 1; }
      summ $O/${wl}_$v.json ${wl}_$v
    done
  done
done
