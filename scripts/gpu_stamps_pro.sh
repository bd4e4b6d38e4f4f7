set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/stamps; export TMPDIR=/tmp
for v in ${VARIANTS}; do
  echo "=== $v"
  timeout -k 10 120 python tools/stamps.py --lib chocosgd_amd/lib/variants/lib_$v.so > gpurun_out/stamps/$v.log 2>&1 || { tail gpurun_out/stamps/$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps/$v.log | head -14
done
