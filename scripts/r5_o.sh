#!/bin/bash
# Round-5 GPU pass O: sign column tiles with VGPR row offsets (no readfirstlane loops) -- oracle diagnostic, sign /
# deferred / fused-step / baseline-size suites, then sign, step_sign, step_sign --defer-receive bench lines.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 200 python tools/debug_sign_fused.py > $O/debug.log 2>&1; grep -v amdgpu.ids $O/debug.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_deferred_receive.py tests/test_gpu_gossip_fused.py \
  tests/test_gpu_baseline_sizes.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do
for wl in sign step_sign step_sign+defer; do
  w=${wl%%+*}; F=""; [ "$wl" != "$w" ] && F="--defer-receive"
  timeout -k 10 300 python bench.py --workload $w $F --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$wl', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
