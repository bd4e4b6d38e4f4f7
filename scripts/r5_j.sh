#!/bin/bash
# Round-5 GPU pass J: the flat warm gossip sequence step by step (diagnostic), then test_gpu_topk.py again.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 200 python tools/debug_gossip_seq.py 3 > $O/debug.log 2>&1; rc=$?; cat $O/debug.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "warm_start" > $O/tests2.log 2>&1; rc=$?; tail -3 $O/tests2.log; exit $rc
