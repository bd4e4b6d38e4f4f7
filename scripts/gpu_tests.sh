# GPU parity suite on one MI355X (gpurun): every -m gpu test through the C ABI.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/tests; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/gpu_tests.log | tail -3
[ $rc -ne 0 ] && tail -60 $O/gpu_tests.log
exit $rc
