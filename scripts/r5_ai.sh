#!/bin/bash
# Round-5 GPU pass AI: LDS-staged segment lookups (sign pack, QSGD quantize), quantize loads before the lookup,
# vectorized boundary tiles -- the QSGD / sign / consumer tests, then per-tensor and flat compress rounds.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5ai; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_gossip_fused.py tests/test_gpu_deferred_receive.py \
  tests/test_gpu_choco_api.py tests/test_gpu_consumers.py tests/test_gpu_baseline_sizes.py -x -q -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for spec in sign_r50 qsgd_r50 step_sign_r50 step_qsgd_r50 "step_qsgd_r50 --defer-receive" qsgd sign step_qsgd; do
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec', d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
