#!/bin/bash
# Round-5 GPU pass AB: the row-run sign receive for per-tensor layouts -- the deferred-receive tests (segmented
# cases: ResNet-20, 300 tiny segments, ragged), the multi-process deferred rounds, sign / API tests, full sizes.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred_receive.py tests/test_gpu_choco_api.py tests/test_gpu_qsgd_sign.py \
  tests/test_gpu_gossip_fused.py tests/test_gpu_baseline_sizes.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py -x -q -k deferred -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $O/mp.log 2>&1; rc=$?; tail -2 $O/mp.log; exit $rc
