# Stamps at two ratios for one variant.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/stamps; export TMPDIR=/tmp
for v in ${VARIANTS:-stamps}; do
for r in 0.99999999 0.99; do
  echo "=== $v ratio $r"
  timeout -k 10 120 python tools/stamps.py --ratio $r --lib chocosgd_amd/lib/variants/lib_$v.so \
    > gpurun_out/stamps/${v}_$r.log 2>&1 || { tail gpurun_out/stamps/${v}_$r.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps/${v}_$r.log
done
done
