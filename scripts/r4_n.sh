#!/bin/bash
# Combined pass: parity of the r04 kernels (r04_all build: looping QSGD quantize, looping
# segmented W2, K2 window-first), then same-box A/Bs against the default build.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4n; mkdir -p $O
CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_r04_all.so timeout -k 10 700 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_baseline_sizes.py tests/test_gpu_topk.py tests/test_gpu_topk_fold.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -40 $O/tests.log; exit $rc; }
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['stage'], r['frac'], d['kernels_us'])"; }
ab() {  # workload variant...
  wl=$1; shift
  for v in "$@"; do
    L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
    timeout -k 10 120 python bench.py --workload $wl --steps 10 --warmup 4 --no-cpu-baseline --no-e2e $L > $O/${wl}_$v.json 2>$O/${wl}_$v.err || { tail -5 $O/${wl}_$v.err; exit 1; }
    summ $O/${wl}_$v.json ${wl}_$v
  done
}
for rep in 1 2; do
  ab topk default k2wf1
  ab topk25m default k2wf1
  ab qsgd default qq_loop1 qq_loop1_g512 qq_loop1_g2048
  ab topk_r50 default seg_loop1 seg_loop1_g512
done
for v in stamps stamps_wf1; do
  timeout -k 10 120 python -u tools/stamps.py --lib chocosgd_amd/lib/variants/lib_$v.so > $O/$v.txt 2>&1; echo "$v rc=$?"; grep -v amdgpu.ids $O/$v.txt | head -24
done
