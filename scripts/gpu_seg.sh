# Segmented top-k / random-k: parity tests, then the ResNet-50 layout bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/seg; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "segmented or randk or choco or multiproc" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python bench.py --workload topk_r50 --no-cpu-baseline --no-e2e > $O/bench_r50.json || exit 1
python -c "import json;d=json.load(open('$O/bench_r50.json'));print(d['value'],d['ms_per_step'],d['kernels_us'])"
