#!/bin/bash
# Round-5 GPU pass N: diagnostic -- sign pack with the fused step and the deferred receive vs the oracle, on the
# product library (wave index as SGPR) and on the round-4 form (wfall).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5n; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 200 python tools/debug_sign_fused.py > $O/base.log 2>&1; cat $O/base.log | grep -v amdgpu.ids
timeout -k 10 200 python tools/debug_sign_fused.py $V/lib_wfall.so > $O/wfall.log 2>&1; cat $O/wfall.log | grep -v amdgpu.ids
