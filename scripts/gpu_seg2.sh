# Segmented top-k select rework: parity + the ResNet-50 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/seg2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_gossip_fused.py tests/test_gpu_choco_api.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^E |FAILED" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --workload topk_r50 --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print(d['ms_per_step'], d['kernels_us'])"
