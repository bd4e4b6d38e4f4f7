#!/bin/bash
# Round-5 GPU pass D: ring-3 loopback receive, merged sweep vs per message -- rocprofv3 kernel
# stats and FETCH/WRITE line traffic per step; top-k default line (one message).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5d; mkdir -p $O
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
  python3 tools/kstats.py $O/r05_ring3_${acc}_kernel_stats.csv 2>/dev/null | head -12 || grep -E "sparse|topk" $O/r05_ring3_${acc}_kernel_stats.csv | cut -c1-160
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $O/b_topk.json 2> $O/b_topk.err || { tail -20 $O/b_topk.err; exit 1; }
python -c "import json; d=json.load(open('$O/b_topk.json')); r=d['roofline']; print('topk', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
