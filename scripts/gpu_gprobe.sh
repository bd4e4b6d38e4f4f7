# A/B of the fused consensus-step kernels (tools/build_variants.py sgs_* / qgs_*).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/gprobe; mkdir -p $O; export TMPDIR=/tmp
V=chocosgd_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_gossip_fused.py tests/test_gpu_qsgd_sign.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/gossip_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
b() {  # workload lib [flags]
  timeout -k 10 300 python bench.py --workload $1 --no-cpu-baseline --no-e2e --steps 10 --warmup 4 --lib $2 $3 \
    > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print('$1 $3', '$2'.split('/')[-1], d['ms_per_step'], d['kernels_us'])"
}
L=chocosgd_amd/lib/libchoco_codec.so
b step_sign $L && b step_sign $V/lib_sgs_ru4.so && b step_sign $V/lib_sgs_split.so && b step_sign $L --unfused \
  && b step_qsgd $L && b sign $L
