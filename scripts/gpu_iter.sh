# Iteration loop on one MI355X: top-k parity tests, phase stamps, stream-only timing, bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/iter; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/${TESTS:-test_gpu_topk.py} -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python tools/stamps.py --save $O/stamps.npy > $O/stamps.log 2>&1 || { tail $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
timeout -k 10 120 python tools/stream_only.py > $O/stream_only.log 2>&1 || { tail $O/stream_only.log; exit 1; }
grep -v amdgpu.ids $O/stream_only.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/bench_topk.json 2> $O/bench_topk.err || { tail $O/bench_topk.err; exit 1; }
cat $O/bench_topk.json
