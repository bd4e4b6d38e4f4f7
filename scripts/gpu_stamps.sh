# Phase-stamp timelines of one top-k call for the stamp variants (tools/stamps.py).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/stamps; export TMPDIR=/tmp
for v in ${VARIANTS:-stamps}; do
  echo "=== $v"
  timeout -k 10 120 python tools/stamps.py --lib chocosgd_amd/lib/variants/lib_$v.so \
    --save gpurun_out/stamps/$v.npy > gpurun_out/stamps/$v.log 2>&1 || { tail gpurun_out/stamps/$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps/$v.log
  timeout -k 10 120 python tools/stream_only.py --lib chocosgd_amd/lib/variants/lib_$v.so > gpurun_out/stamps/so_$v.log 2>&1 || { tail gpurun_out/stamps/so_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps/so_$v.log
done
