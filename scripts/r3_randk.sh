cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -k "randk or gather" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/t_randk.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/t_randk.log | tail -3; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/t_randk.log | head -20; tail -30 $O/t_randk.log; exit $rc; }
timeout -k 10 300 python bench.py --workload randk --no-cpu-baseline --no-e2e > $O/b_randk.json 2> $O/b_randk.err; rc=$?
python -c "import json; d=json.load(open('$O/b_randk.json')); print(d['value'], d['ms_per_step'], d['kernels_us'], [ (s['stage'], s['frac']) for s in d['stages']])"
exit $rc
