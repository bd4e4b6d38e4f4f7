set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/fused2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "topk and not segmented" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/fused_stamps.py 2>&1 | grep -v amdgpu.ids | head -12 || exit 1
timeout -k 10 120 python tools/fused_stamps.py --lib chocosgd_amd/lib/variants/lib_stamps_pre1.so 2>&1 | grep -v amdgpu.ids | head -12 || exit 1
for v in default fpre1 topk3 default; do
  L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e $L > $O/bench_$v.json || exit 1
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v',d['value'],d['ms_per_step'],d['kernels_us'])"
done
