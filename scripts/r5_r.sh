#!/bin/bash
# Round-5 GPU pass R: the whole GPU suite on the committed tree, then smoke().
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  --durations=10 > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -3 $O/smoke.log; exit $rc
