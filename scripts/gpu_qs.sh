# QSGD / sign kernels: parity tests, then their bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/qs; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "qsgd or sign or baseline or multiproc or more_than" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wl in qsgd sign; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-e2e > $O/bench_$wl.json || exit 1
  python -c "import json;d=json.load(open('$O/bench_$wl.json'));print('$wl',d['value'],d['ms_per_step'],d['kernels_us'])"
done
