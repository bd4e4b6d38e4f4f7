#!/bin/bash
# Round-5 GPU pass M: the wave index as an SGPR (sign packs without readfirstlane loops) -- sign / deferred /
# fused-step suites; same-box A/B against the round-4 form (wfall) on sign, step_sign, step_sign --defer-receive.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5m; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_deferred_receive.py tests/test_gpu_gossip_fused.py \
  tests/test_gpu_baseline_sizes.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do
for wl in sign step_sign step_sign+defer; do
for v in base wfall; do
  w=${wl%%+*}; F=""; [ "$wl" != "$w" ] && F="--defer-receive"
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $w $F --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$wl $v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
done
