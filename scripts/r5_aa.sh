#!/bin/bash
# Round-5 GPU pass AA: the sparse accumulate's segment write-back non-temporal (stores; loads + stores) -- whole
# step times on randk / topk / topk_r50 (the next step's gathers and stream run behind the write-back).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5aa; mkdir -p $O; V=chocosgd_amd/lib/variants
for rep in 1 2 3; do
for wl in randk topk topk_r50; do
for v in base acc_ntst acc_ntldst; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$wl $v', d['ms_per_step'], d['kernels_us'])"
done
done
done
