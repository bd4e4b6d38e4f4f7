#!/bin/bash
# Round-4 GPU pass B: one-launch top-k timeline (stamps build) and a same-box A/B of the bench.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4; mkdir -p $O
CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_stamps.so timeout -k 10 120 python -u tools/one_stamps.py > $O/one_stamps.txt 2>&1; echo "stamps rc=$?"; cat $O/one_stamps.txt | grep -v amdgpu.ids
for v in one0 default one0 default; do
  if [ $v = default ]; then L=""; else L="--lib chocosgd_amd/lib/variants/lib_$v.so"; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e $L > $O/ab_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/ab_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
