#!/bin/bash
# fold + QSGD occupancy: parity first, then same-box A/B
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topk_fold.py tests/test_gpu_qsgd_sign.py tests/test_gpu_topk.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -40 $O/tests.log; exit $rc; }
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['stage'], r['frac'], d['kernels_us'])"; }
for rep in 1 2; do
  for v in nofold fold; do
    F=""; [ $v = fold ] && F="--fold"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e $F > $O/topk_$v.json 2>$O/topk_$v.err || { tail -5 $O/topk_$v.err; exit 1; }
    summ $O/topk_$v.json topk_$v
  done
  for v in default qq_w4 qq_w6 qcheck0; do
    L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
    timeout -k 10 200 python bench.py --workload qsgd --no-cpu-baseline --no-e2e $L > $O/qsgd_$v.json 2>$O/qsgd_$v.err || { tail -5 $O/qsgd_$v.err; exit 1; }
    summ $O/qsgd_$v.json qsgd_$v
  done
done
for v in nofold fold; do
  F=""; [ $v = fold ] && F="--fold"
  timeout -k 10 200 python bench.py --workload step_topk --no-cpu-baseline --no-e2e $F > $O/step_$v.json 2>$O/step_$v.err || { tail -5 $O/step_$v.err; exit 1; }
  summ $O/step_$v.json step_topk_$v
done
