#!/bin/bash
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_choco_api.py tests/test_gpu_consumers.py tests/test_gpu_gossip_fused.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -40 $O/tests.log; exit $rc; }
timeout -k 10 120 python -u tools/seg_stamps.py > $O/seg_stamps.txt 2>&1; echo "stamps rc=$?"; grep -v amdgpu.ids $O/seg_stamps.txt | head -14
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['stage'], r['frac'], d['kernels_us'])"; }
for rep in 1 2 3; do
  for v in default seg_sf0; do
    L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
    timeout -k 10 120 python bench.py --workload topk_r50 --steps 10 --warmup 4 --no-cpu-baseline --no-e2e $L > $O/r50_$v.json 2>$O/r50_$v.err || { tail -5 $O/r50_$v.err; exit 1; }
    summ $O/r50_$v.json r50_$v
  done
done
