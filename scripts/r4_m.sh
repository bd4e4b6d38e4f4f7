#!/bin/bash
# K2 window-first: top-k parity, stamps, same-box A/B (100M and 25M)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_topk_fold.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -40 $O/tests.log; exit $rc; }
timeout -k 10 120 python -u tools/stamps.py > $O/stamps.txt 2>&1; echo "stamps rc=$?"; grep -v amdgpu.ids $O/stamps.txt | head -48
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['stage'], r['frac'], d['kernels_us'])"; }
for rep in 1 2; do
  for wl in topk topk25m; do
    for v in default k2wf0; do
      L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
      timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-e2e $L > $O/${wl}_$v.json 2>$O/${wl}_$v.err || { tail -5 $O/${wl}_$v.err; exit 1; }
      summ $O/${wl}_$v.json ${wl}_$v
    done
  done
done
