#!/bin/bash
# Round-5 GPU pass E: multi sweep v2 -- parity, ring-3 loopback rocprof stats + line traffic, A/B.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_multi.py tests/test_gpu_choco_api.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/tests.log | head; exit $rc; }
for acc in multi per_message; do
  B="bench.py --workload topk --ring3-loopback --accumulate $acc --steps 3 --warmup 2 --no-cpu-baseline --no-e2e"
  rm -rf /tmp/pf /tmp/pw /tmp/pk
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o f -- python3 $B > $O/pmcf_$acc.log 2>&1 || { tail -5 $O/pmcf_$acc.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o w -- python3 $B > $O/pmcw_$acc.log 2>&1 || { tail -5 $O/pmcw_$acc.log; exit 1; }
  python3 tools/step_traffic.py /tmp/pf /tmp/pw 8 sparse_acc_seg_kernel sparse_split_kernel sparse_acc_multi_kernel > $O/traffic_$acc.txt || exit 1
  echo "== $acc"; cat $O/traffic_$acc.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk -o k -- python3 bench.py --workload topk \
    --ring3-loopback --accumulate $acc --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/prof_$acc.json 2> $O/prof_$acc.err || { tail -5 $O/prof_$acc.err; exit 1; }
  cp $(find /tmp/pk -name "*kernel_stats.csv" | head -1) $O/r05_ring3_${acc}_kernel_stats.csv || exit 1
  python3 tools/kstats.py $O/r05_ring3_${acc}_kernel_stats.csv | grep -E "sparse|topk"
done
