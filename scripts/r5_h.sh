#!/bin/bash
# Round-5 GPU pass H: warm segmented tail S3w + S4w (product) -- parity suites; then same-box A/B against the
# round-4 tail (segw0) and the tile-size variants (seg5 / seg6, parity-checked first).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5h; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_choco_api.py tests/test_gpu_gossip_fused.py \
  tests/test_gpu_consumers.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for v in seg5 seg6; do
  timeout -k 10 300 python tools/seg_variant_check.py $V/lib_$v.so > $O/check_$v.log 2>&1 || { tail -5 $O/check_$v.log; exit 1; }
  tail -1 $O/check_$v.log
done
for rep in 1 2 3; do
for v in base segw0 seg5 seg6; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 200 python bench.py --workload topk_r50 --no-cpu-baseline --no-e2e $L > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$v.json')); r=d['roofline']; print('$v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
