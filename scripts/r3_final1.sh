# r3: top-k GPU tests, then the measurement pass for the top-k / random-k workloads
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/final1_tests.log 2>&1
rc=$?; tail -3 $O/final1_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/final1_tests.log | head -30; exit $rc; }
WLS="topk topk25m topk_r50 randk step_topk" R=r03 bash scripts/gpu_measure.sh
