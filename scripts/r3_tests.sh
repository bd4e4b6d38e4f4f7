# r3: GPU tests of the given files (default: all), then the top-k bench line
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
FILES=${FILES:-tests}
timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/tests.log | tail -3; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -30 $O/tests.log; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $O/b_topk.json 2> $O/b_topk.err; rc=$?
python -c "import json; d=json.load(open('$O/b_topk.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
exit $rc
