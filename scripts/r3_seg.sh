cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_gossip_fused.py tests/test_gpu_choco_api.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/t_seg.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/t_seg.log | tail -3; [ $rc -ne 0 ] && { grep -E "FAILED|Error|^E " $O/t_seg.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --workload topk_r50 --no-cpu-baseline --no-e2e > $O/b_r50.json 2> $O/b_r50.err; rc=$?
python -c "import json; d=json.load(open('$O/b_r50.json')); print(d['value'], d['ms_per_step'], d['kernels_us'], [ (s['stage'], s['us_per_step'], s['frac']) for s in d['stages']])"
exit $rc
