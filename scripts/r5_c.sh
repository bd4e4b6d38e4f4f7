#!/bin/bash
# Round-5 GPU pass C: the whole GPU suite, known-T floor at 25M, ring-3 loopback A/B
# (multi sweep vs per message), gloo 4-rank bench line, K34 j* hint A/B (top-k).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=10 > $O/tests.log 2>&1
rc=$?; tail -14 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|error" $O/tests.log | head -30; exit $rc; }
timeout -k 10 150 tools/probe_floor 25000000 > $O/probe_floor_25m.txt 2>&1 || { echo "probe rc=$?"; tail -20 $O/probe_floor_25m.txt; exit 1; }
sed -n 13,22p $O/probe_floor_25m.txt
for acc in multi per_message multi per_message; do
  timeout -k 10 300 python bench.py --ring3-loopback --accumulate $acc --no-cpu-baseline --no-e2e > $O/b_loop_$acc.json 2> $O/b_loop_$acc.err || { tail -20 $O/b_loop_$acc.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_loop_$acc.json')); s=[x for x in d['stages'] if x['stage']=='decompress'][0]; print('$acc', d['ms_per_step'], s['us_per_step'], {k: v['us_per_launch'] for k, v in s['kernels'].items()}, s.get('granule_bytes'), s.get('line_tx_rate'))"
done
for v in main k34_nohint main k34_nohint main k34_nohint; do
  L=""; [ "$v" != main ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e $L > $O/b_topk_$v.json 2> $O/b_topk_$v.err || { tail -20 $O/b_topk_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_topk_$v.json')); r=d['roofline']; print('$v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
timeout -k 10 300 python bench.py --gpus 4 --backend gloo --no-cpu-baseline --steps 10 --warmup 3 > $O/b_gloo4.json 2> $O/b_gloo4.err; rc=$?
tail -c 300 $O/b_gloo4.json; [ $rc -ne 0 ] && tail -20 $O/b_gloo4.err
exit $rc
