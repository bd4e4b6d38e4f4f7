# r3: random-k GPU parity tests, the random-k bench line, and the phase stamps
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "randk or random" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/rk_tests.log 2>&1
rc=$?; tail -3 $O/rk_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/rk_tests.log | head -20; exit $rc; }
timeout -k 10 200 python3 bench.py --workload randk --no-cpu-baseline --no-e2e > $O/b_randk.json 2> $O/b_randk.err || { tail -5 $O/b_randk.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/b_randk.json').read().splitlines()[-1])
print('randk', d['ms_per_step'], round(d['roofline']['frac'], 4), {k: round(v, 1) for k, v in d['kernels_us'].items()})"
timeout -k 10 120 python tools/rk_stamps.py > $O/rk_stamps.txt 2>&1; cat $O/rk_stamps.txt
