set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/quick
timeout -k 10 120 python tools/stamps.py --save gpurun_out/quick/stamps.npy 2>&1 | grep -v amdgpu.ids
