#!/bin/bash
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4o; mkdir -p $O
for i in 1 2; do
timeout -k 10 120 python -u tools/stamps.py --lib chocosgd_amd/lib/variants/lib_stamps.so > $O/stamps$i.txt 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/stamps$i.txt | sed -n 20,45p
done
