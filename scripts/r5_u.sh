#!/bin/bash
# Round-5 GPU pass U: K2 writing each wave's pairs at its stream end (k2early, round 4's DESIGN 9.2) -- the top-k
# suite on the variant library, then a same-box A/B against the product on topk, topk25m and step_topk.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5u; mkdir -p $O; V=chocosgd_amd/lib/variants
CHOCO_CODEC_LIB=$V/lib_k2early.so timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_topk_fold.py -x -q \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
for rep in 1 2 3; do
for wl in topk topk25m step_topk; do
for v in base k2early; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$wl $v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
done
