#!/bin/bash
# Random-k R2: workgroups per tile 4 (default) vs 8 / 16: parity with each build, then A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4rk; mkdir -p $O
for v in rk_q8 rk_q16; do
  CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_consumers.py tests/test_gpu_choco_api.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "randk or random" > $O/tests_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests_$v.log | head -30; tail -30 $O/tests_$v.log; exit $rc; }
done
summ() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', d['ms_per_step'], d['kernels_us'])"; }
for rep in 1 2 3; do
  for v in default rk_q8 rk_q16; do
    L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
    timeout -k 10 120 python bench.py --workload randk --steps 10 --warmup 4 --no-cpu-baseline --no-e2e $L > $O/randk_$v.json 2>$O/randk_$v.err || { tail -5 $O/randk_$v.err; exit 1; }
    summ $O/randk_$v.json randk_$v
  done
done
