#!/bin/bash
# Round-5 GPU pass B: the whole GPU suite (rings > 3, multi-message receive, the purged
# sources), known-T floor at 25M / 100M, gloo 4-rank bench line, ring-3 loopback A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=15 > $O/tests.log 2>&1
rc=$?; tail -25 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|error" $O/tests.log | head -30; exit $rc; }
timeout -k 10 150 tools/probe_floor 25000000 > $O/probe_floor_25m.txt 2>&1 || { echo "probe rc=$?"; tail -20 $O/probe_floor_25m.txt; exit 1; }
sed -n 13,22p $O/probe_floor_25m.txt
for acc in multi per_message multi per_message; do
  timeout -k 10 300 python bench.py --ring3-loopback --accumulate $acc --no-cpu-baseline --no-e2e > $O/b_loop_$acc.json 2> $O/b_loop_$acc.err || { tail -20 $O/b_loop_$acc.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_loop_$acc.json')); s=[x for x in d['stages'] if x['stage']=='decompress'][0]; print('$acc', d['ms_per_step'], s['us_per_step'], s['kernels'], s.get('granule_bytes'), s.get('line_tx_rate'))"
done
timeout -k 10 300 python bench.py --gpus 4 --backend gloo --no-cpu-baseline --steps 10 --warmup 3 > $O/b_gloo4.json 2> $O/b_gloo4.err; rc=$?
tail -c 400 $O/b_gloo4.json; [ $rc -ne 0 ] && tail -20 $O/b_gloo4.err
exit $rc
