#!/bin/bash
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topk.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/t_topk.log 2>&1
rc=$?; tail -2 $O/t_topk.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/t_topk.log | head -30; tail -60 $O/t_topk.log; exit $rc; }
CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_stamps.so timeout -k 10 120 python -u tools/one_stamps.py --calls 2 --loop 10 --acc --seed 1000 > $O/one_stamps_i.txt 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/one_stamps_i.txt | cut -c1-200
for v in default one0 one_rot0 default one0 one_rot0; do
  if [ $v = default ]; then L=""; else L="--lib chocosgd_amd/lib/variants/lib_$v.so"; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e $L > $O/ab_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/ab_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'], 'fallbacks', d['topk_fallbacks'])"
done
