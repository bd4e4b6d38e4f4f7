#!/bin/bash
# Round-5 GPU pass Z: LDS-staged plane transposes -- the deferred-receive and sign/API tests, the
# multi-process deferred tests, the oracle diagnostic, then the round measurement of step_sign+defer.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred_receive.py tests/test_gpu_choco_api.py tests/test_gpu_qsgd_sign.py \
  tests/test_gpu_gossip_fused.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py -x -q -k deferred -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $O/mp.log 2>&1; rc=$?; tail -2 $O/mp.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/debug_sign_fused.py > $O/debug.log 2>&1 || { tail -20 $O/debug.log; exit 1; }
echo "debug mismatches: $(grep -c differ $O/debug.log)"
WLS="step_sign+defer" bash scripts/gpu_measure.sh
