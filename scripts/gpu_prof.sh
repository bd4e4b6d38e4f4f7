set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/prof6; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -x > gpurun_out/gpu_tests6.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests6.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for wl in topk qsgd sign; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6/$wl -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --workload $wl --no-cpu-baseline > gpurun_out/bench6_$wl.log 2>&1
echo "bench $wl rc=$?"
done
