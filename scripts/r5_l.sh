#!/bin/bash
# Round-5 GPU pass L: segmented warm tail v3 (hist2 prefetched by the window workgroups, fewer barriers) --
# segmented suites, A/B against segw0; the sign access-pattern probe.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5l; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_choco_api.py tests/test_gpu_gossip_fused.py \
  -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "segment or choco or fused or gossip" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for rep in 1 2 3; do
for v in base segw0; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 200 python bench.py --workload topk_r50 --no-cpu-baseline --no-e2e $L > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$v.json')); r=d['roofline']; print('$v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
timeout -k 10 150 tools/probe_sign_rw > $O/probe_sign_rw.txt 2>&1 || { echo "probe rc=$?"; tail -5 $O/probe_sign_rw.txt; exit 1; }
cat $O/probe_sign_rw.txt
