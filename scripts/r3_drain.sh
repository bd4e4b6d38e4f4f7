# r3: the warm-start drain tests + all top-k tests, then the fused-step and top-k bench lines
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_gossip_fused.py tests/test_gpu_choco_api.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/drain_tests.log 2>&1
rc=$?; tail -3 $O/drain_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/drain_tests.log | head -30; exit $rc; }
for wl in step_topk topk topk_r50 topk25m; do
  timeout -k 10 200 python3 bench.py --workload $wl --no-cpu-baseline --no-e2e > $O/b_$wl.json 2> $O/b_$wl.err || { tail -5 $O/b_$wl.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$wl.json').read().splitlines()[-1])
print('$wl', d['ms_per_step'], round(d['roofline']['frac'], 4), {k: round(v, 1) for k, v in d['kernels_us'].items()})"
done
