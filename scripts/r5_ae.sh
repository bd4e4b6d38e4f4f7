#!/bin/bash
# Round-5 GPU pass AE: adaptive QSGD norm tiles; the fused sign pack in 4-row groups on small grids (A/B: packru8)
# -- the sign / QSGD / fused / deferred / consumer tests, then the ResNet-50-layout and flat steps.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5ae; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_gossip_fused.py tests/test_gpu_deferred_receive.py \
  tests/test_gpu_choco_api.py tests/test_gpu_consumers.py tests/test_gpu_baseline_sizes.py -x -q -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do
for spec in "step_sign_r50" "step_sign_r50 --lib $V/lib_packru8.so" "step_sign_r50 --defer-receive" \
            "step_sign_r50 --defer-receive --lib $V/lib_signseg2k.so" "step_qsgd_r50" "step_qsgd_r50 --defer-receive" \
            "step_sign" "step_qsgd" "qsgd" "sign"; do
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec'.replace('$V/',''), d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
done
