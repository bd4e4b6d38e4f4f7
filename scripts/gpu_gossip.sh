# Fused CHOCO step (consensus step inside the compressor's first pass): parity tests,
# the top-k / sign / QSGD regression suites, then fused vs unfused step bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/gossip; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gossip_fused.py tests/test_gpu_topk.py tests/test_gpu_qsgd_sign.py \
  tests/test_gpu_choco_api.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -40 $O/tests.log; exit $rc; }
for wl in step_topk step_sign step_qsgd; do
  for mode in "" "--unfused"; do
    timeout -k 10 300 python bench.py --workload $wl $mode --no-cpu-baseline --steps 10 --warmup 4 \
      > $O/bench_${wl}${mode}.json 2> $O/bench_${wl}${mode}.err || { tail -20 $O/bench_${wl}${mode}.err; exit 1; }
  done
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/gossip/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["kernels_us"])
PY
