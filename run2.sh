set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 > gpurun_out/gpu_tests2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/topk -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_topk.log 2>&1
echo "prof rc=$?"
for wl in qsgd sign topk25m; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --workload $wl --no-cpu-baseline > gpurun_out/bench_$wl.log 2>&1
echo "bench $wl rc=$?"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_topk_cpu.log 2>&1
echo "bench topk+cpu rc=$?"
