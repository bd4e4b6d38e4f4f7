#!/bin/bash
# Round-5 GPU pass AN: the sign pack's row split on small grids (A/B: packrs1) -- sign / fused / deferred / consumer
# tests, the per-layout diagnostic on both builds, then the ResNet-50 and flat 25.6M sign steps.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5an; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_gossip_fused.py tests/test_gpu_deferred_receive.py \
  tests/test_gpu_choco_api.py tests/test_gpu_consumers.py -x -q -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for v in base packrs1; do
  L=""; [ $v != base ] && L="$V/lib_$v.so"
  echo "== $v"; timeout -k 10 300 python -u tools/diag_seg_layouts.py $L 2>&1 | grep -v amdgpu.ids || exit 1
done
for rep in 1 2; do
for v in base packrs1; do
for spec in step_sign_r50 "step_sign --n 25557032" sign_r50; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec $v', d['ms_per_step'], d['kernels_us'])"
done
done
done
