#!/bin/bash
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4; mkdir -p $O
for opt in "--loop 10" "--loop 10 --acc"; do
CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_stamps.so timeout -k 10 120 python -u tools/one_stamps.py --calls 2 $opt > $O/one_stamps_d.txt 2>&1; echo "== $opt rc=$?"; grep -v amdgpu.ids $O/one_stamps_d.txt | grep -E "call|start  |window|streamed|ticket|record|emitted|last work|Error|error"
done
