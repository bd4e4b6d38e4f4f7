# Wide exact fallback: parity at 100M (ties / all-equal / zeros), the flat top-k suite, timing.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/fallback; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_topk.py -m gpu -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^E |FAILED|Timeout" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/fallback_time.py > $O/time.txt 2>&1 || { tail -5 $O/time.txt; exit 1; }
cat $O/time.txt
