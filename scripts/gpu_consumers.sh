# DCD / DeepSqueeze drop-ins + the sign receiver's rounding modes (-m gpu).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/consumers; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_consumers.py tests/test_gpu_qsgd_sign.py tests/test_gpu_choco_api.py \
  -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head -40; exit $rc; }
exit 0
