# r3: top-k + random-k GPU parity tests, then the randk / topk_r50 / topk bench lines
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_choco_api.py tests/test_gpu_consumers.py tests/test_gpu_gossip_fused.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/seg2_tests.log 2>&1
rc=$?; tail -3 $O/seg2_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/seg2_tests.log | head -30; exit $rc; }
for wl in randk topk_r50 topk; do
  timeout -k 10 200 python3 bench.py --workload $wl --no-cpu-baseline --no-e2e > $O/b_$wl.json 2> $O/b_$wl.err || { tail -5 $O/b_$wl.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$wl.json').read().splitlines()[-1])
print('$wl', d['ms_per_step'], round(d['roofline']['frac'], 4), {k: round(v, 1) for k, v in d['kernels_us'].items()})"
done
timeout -k 10 120 python tools/rk_stamps.py > $O/rk_stamps.txt 2>&1; tail -14 $O/rk_stamps.txt
