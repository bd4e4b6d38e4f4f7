#!/bin/bash
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4; mkdir -p $O
for v in stamps_one0 stamps; do
CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_$v.so timeout -k 10 120 python -u tools/one_stamps.py --calls 1 --loop 10 --acc --seed 1000 --trace > $O/one_stamps_e.txt 2>&1; echo "== $v rc=$?"; grep -v amdgpu.ids $O/one_stamps_e.txt | grep -E "warm-up|fallbacks|Error|error" | cut -c1-250
done
