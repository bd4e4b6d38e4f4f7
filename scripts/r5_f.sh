#!/bin/bash
# Round-5 GPU pass F: deferred receive (QSGD, sign) -- parity, step A/B (sequence vs fused), rocprof stats.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_deferred_receive.py tests/test_gpu_qsgd_sign.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for wl in step_qsgd step_sign; do
for v in plain defer plain defer; do
  F=""; [ $v = defer ] && F="--defer-receive"
  timeout -k 10 300 python bench.py --workload $wl $F --no-cpu-baseline > $O/b_${wl}_$v.json 2> $O/b_${wl}_$v.err || { tail -20 $O/b_${wl}_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${wl}_$v.json')); r=d['roofline']; print('$wl $v', d['value'], d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
for wl in step_qsgd step_sign; do
rm -rf /tmp/pk
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk -o k -- python3 bench.py --workload $wl \
  --defer-receive --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/prof_$wl.json 2> $O/prof_$wl.err || { tail -5 $O/prof_$wl.err; exit 1; }
cp $(find /tmp/pk -name "*kernel_stats.csv" | head -1) $O/r05_${wl}_deferred_kernel_stats.csv && python3 tools/kstats.py $O/r05_${wl}_deferred_kernel_stats.csv
done
