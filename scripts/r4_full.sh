#!/bin/bash
# Round-end rehearsal: the whole -m gpu suite as the driver runs it, then smoke().
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4full; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/gpu_tests.log | tail -3; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -60 $O/gpu_tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -3 $O/smoke.log; exit $rc
