# Fused top-k: parity first (every flat / segmented top-k test), then A/B bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/fused; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "topk or randk or choco or smoke" > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in default topk3 default; do
  L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e $L > $O/bench_$v.json || exit 1
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v',d['value'],d['ms_per_step'],d['kernels_us'])"
done
