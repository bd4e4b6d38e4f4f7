#!/bin/bash
# QSGD ring quantize (LDS-DMA per-wave ring): parity with each ring build, then A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4v; mkdir -p $O
for v in qq_ring_d3w3 qq_ring_d2w4; do
  CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_baseline_sizes.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "qsgd" > $O/tests_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests_$v.log | head -30; tail -30 $O/tests_$v.log; exit $rc; }
done
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['stage'], r['frac'], d['kernels_us'])"; }
for rep in 1 2 3; do
  for v in default qq_ring_d3w3 qq_ring_d2w4; do
    L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
    timeout -k 10 120 python bench.py --workload qsgd --steps 10 --warmup 4 --no-cpu-baseline --no-e2e $L > $O/qsgd_$v.json 2>$O/qsgd_$v.err || { tail -5 $O/qsgd_$v.err; exit 1; }
    summ $O/qsgd_$v.json qsgd_$v
  done
done
