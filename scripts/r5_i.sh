#!/bin/bash
# Round-5 GPU pass I: warm segmented tail v2 (S3w one-trip loads + per-tile kept keys; S4w with segment window
# workgroups) -- segmented parity suites, then same-box A/B against the round-4 tail (segw0).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5i; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_choco_api.py tests/test_gpu_gossip_fused.py \
  tests/test_gpu_consumers.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for rep in 1 2 3; do
for v in base segw0; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 200 python bench.py --workload topk_r50 --no-cpu-baseline --no-e2e $L > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$v.json')); r=d['roofline']; print('$v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
rm -rf /tmp/pk
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk -o k -- python3 bench.py --workload topk_r50 \
  --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
cp $(find /tmp/pk -name "*kernel_stats.csv" | head -1) $O/r05_topk_r50_w3_kernel_stats.csv && python3 tools/kstats.py $O/r05_topk_r50_w3_kernel_stats.csv | grep seg
