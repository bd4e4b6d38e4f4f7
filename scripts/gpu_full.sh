# Full GPU parity suite + bench lines for every workload (no cpu baseline / e2e).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/full; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for wl in ${WLS:-topk topk25m qsgd sign}; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-e2e > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail $O/bench_$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$wl.json')); print('$wl', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
