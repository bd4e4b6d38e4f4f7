#!/bin/bash
# Round-5 GPU pass V: the deferred sign receive over row runs of bit planes -- its tests and the oracle
# diagnostic, then a same-box A/B against the column-tile receive (variant signcols) on step_sign --defer-receive.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5v; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred_receive.py tests/test_gpu_choco_api.py -x -q \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/debug_sign_fused.py > $O/debug.log 2>&1 || { tail -20 $O/debug.log; exit 1; }
grep -c differ $O/debug.log
for rep in 1 2 3; do
for v in base signcols; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload step_sign --defer-receive --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('step_sign+defer $v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py -x -q -k deferred -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $O/mp.log 2>&1; rc=$?; tail -3 $O/mp.log; exit $rc
