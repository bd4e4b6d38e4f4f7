#!/bin/bash
# Round-5 GPU pass A: rings > 3 (world 4 / 8 CHOCO rounds, ring-8 replay vs the reference),
# fold vs oracle, fallback under load; known-T floor at 25M and 100M; gloo 4-rank bench line.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_choco_api.py tests/test_gpu_topk_fold.py \
  "tests/test_gpu_topk.py::test_topk_wide_fallback_under_concurrent_load" -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|error" $O/tests.log | head -30; tail -60 $O/tests.log; exit $rc; }
timeout -k 10 150 tools/probe_floor 25000000 > $O/probe_floor_25m.txt 2>&1 || { echo "probe rc=$?"; tail -20 $O/probe_floor_25m.txt; exit 1; }
sed -n 1,25p $O/probe_floor_25m.txt
timeout -k 10 150 tools/probe_floor > $O/probe_floor_100m.txt 2>&1 || { echo "probe rc=$?"; tail -20 $O/probe_floor_100m.txt; exit 1; }
sed -n 13,22p $O/probe_floor_100m.txt
timeout -k 10 300 python bench.py --gpus 4 --backend gloo --no-cpu-baseline --steps 10 --warmup 3 > $O/b_gloo4.json 2> $O/b_gloo4.err; rc=$?
tail -c 600 $O/b_gloo4.json; [ $rc -ne 0 ] && tail -20 $O/b_gloo4.err
exit $rc
