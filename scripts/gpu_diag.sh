# GPU parity tests + stream-kernel diagnostics on one MI355X.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/diag; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -x > gpurun_out/diag/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/diag/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -f chocosgd_amd/lib/variants/lib_stamps.so ]; then
  timeout -k 10 120 python tools/stamps.py > gpurun_out/diag/stamps.log 2>&1 || exit $?
  cat gpurun_out/diag/stamps.log
fi
for v in ${VARIANTS:-}; do
  timeout -k 10 120 python tools/diag_stream.py --lib chocosgd_amd/lib/variants/lib_$v.so --only topk \
    > gpurun_out/diag/$v.log 2>&1 || exit $?
  cat gpurun_out/diag/$v.log
done
for m in hot cold; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/diag/prof_$m -o run --output-format csv -- \
    python tools/diag_stream.py --modes $m > gpurun_out/diag/prof_$m.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/diag/prof_$m.log
  python tools/kstats.py $(find gpurun_out/diag/prof_$m -name "*kernel_stats.csv")
done
