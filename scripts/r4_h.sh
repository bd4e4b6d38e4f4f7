#!/bin/bash
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4; mkdir -p $O
CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_stamps.so timeout -k 10 120 python -u tools/one_stamps.py --calls 2 --loop 10 --acc --seed 1000 > $O/one_stamps_h.txt 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/one_stamps_h.txt | cut -c1-200
