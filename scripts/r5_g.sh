#!/bin/bash
# Round-5 GPU pass G: deferred receive tests (kernels + drop-in), same-box A/B of the fused sign kernel's knobs.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_deferred_receive.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
V=chocosgd_amd/lib/variants
for rep in 1 2; do
for v in base srp_nts0 srp_nt00 srp_ru2 srp_ru2_nts0 srp_wpe3 srp_ru8; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 200 python bench.py --workload step_sign --defer-receive --steps 10 --warmup 4 --no-cpu-baseline --no-e2e $L \
    > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$v.json')); r=d['roofline']; print('$v', d['ms_per_step'], r['kernel_us'], r['frac'])"
done
done
