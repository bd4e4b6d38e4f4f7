# GPU parity tests, stamps timeline, top-k ratio sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/quick; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -x > gpurun_out/quick/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/quick/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/stamps.py --save gpurun_out/quick/stamps.npy > gpurun_out/quick/stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/quick/stamps.log
timeout -k 10 200 python tools/diag_stream.py --only topk --modes hot --ratios 0.99999999,0.999,0.99,0.9,0.5 > gpurun_out/quick/ratios.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/quick/ratios.log
for v in ${VARIANTS:-}; do
  timeout -k 10 120 python tools/diag_stream.py --lib chocosgd_amd/lib/variants/lib_$v.so --only topk --modes hot \
    --ratios 0.99999999,0.99 > gpurun_out/quick/$v.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/quick/$v.log
done
