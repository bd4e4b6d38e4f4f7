set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/qq; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "qsgd or multiproc" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py --workload qsgd --no-cpu-baseline --no-e2e > $O/bench_qsgd.json || exit 1
python -c "import json;d=json.load(open('$O/bench_qsgd.json'));print(d['value'],d['ms_per_step'],d['kernels_us'])"
