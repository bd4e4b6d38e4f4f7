#!/bin/bash
# 16-element uniform streams: every QSGD parity test + smoke, then quantize A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_baseline_sizes.py tests/test_gpu_gossip_fused.py tests/test_gpu_consumers.py tests/test_gpu_multiproc.py tests/test_gpu_choco_api.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -40 $O/tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['stage'], r['frac'], d['kernels_us'])"; }
for rep in 1 2 3; do
  for wl in qsgd step_qsgd; do
    for v in default qq_h0; do
      L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
      timeout -k 10 120 python bench.py --workload $wl --steps 10 --warmup 4 --no-cpu-baseline --no-e2e $L > $O/${wl}_$v.json 2>$O/${wl}_$v.err || { tail -5 $O/${wl}_$v.err; exit 1; }
      summ $O/${wl}_$v.json ${wl}_$v
    done
  done
done
