#!/bin/bash
# Round-5 GPU pass AP: the sign accumulate's buffer-load fast path (A/B: saccold, the realigned loads) -- sign /
# consumer / fused / deferred tests, then sign, step_sign, sign_r50, step_sign_r50 (twice).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5ap; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_gossip_fused.py tests/test_gpu_deferred_receive.py \
  tests/test_gpu_choco_api.py tests/test_gpu_consumers.py tests/test_gpu_baseline_sizes.py -x -q -p no:cacheprovider \
  --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do
for v in base saccold; do
for spec in sign step_sign sign_r50; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec $v', d['ms_per_step'], d['kernels_us'])"
done
done
done
