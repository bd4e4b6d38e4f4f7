# top-k parity tests, stamps + stream-only timing for the given variants, product bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/iter; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ${VARIANTS:-stamps}; do
  echo "=== $v"
  timeout -k 10 120 python tools/stamps.py --lib chocosgd_amd/lib/variants/lib_$v.so > $O/$v.log 2>&1 || { tail $O/$v.log; exit 1; }
  grep -v amdgpu.ids $O/$v.log | grep -v "subsample\|keys >=\|tile entries\|(key loads"
  timeout -k 10 120 python tools/stream_only.py --lib chocosgd_amd/lib/variants/lib_$v.so > $O/so_$v.log 2>&1 || { tail $O/so_$v.log; exit 1; }
  grep "0.99:" $O/so_$v.log
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > $O/bench_topk.json 2> $O/bench_topk.err || { tail $O/bench_topk.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_topk.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
