#!/bin/bash
# Looping quantize with the prefetch hidden from the compiler's wait pass: parity, then A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4z; mkdir -p $O
for v in qq_loop_asm; do
  CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_baseline_sizes.py tests/test_gpu_consumers.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "qsgd or dgc" > $O/tests_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests_$v.log | head -30; tail -30 $O/tests_$v.log; exit $rc; }
done
summ() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', d['ms_per_step'], d['kernels_us'])"; }
for rep in 1 2 3; do
  for v in default qq_loop_asm qq_loop_asm_g512 qn_plain qn_plain_qq_nt qq_nt_h; do
    L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
    timeout -k 10 120 python bench.py --workload qsgd --steps 10 --warmup 4 --no-cpu-baseline --no-e2e $L > $O/qsgd_$v.json 2>$O/qsgd_$v.err || { tail -5 $O/qsgd_$v.err; exit 1; }
    summ $O/qsgd_$v.json qsgd_$v
  done
done
