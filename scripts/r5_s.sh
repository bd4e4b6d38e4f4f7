#!/bin/bash
# Round-5 GPU pass S: the round-4 warm tail purged (S3a / S3b / S4 cold-only) -- top-k / drop-in / fused-step /
# consumer / multiprocess suites (random warm layouts included); segmented bench line.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_choco_api.py tests/test_gpu_gossip_fused.py \
  tests/test_gpu_consumers.py tests/test_gpu_multiproc.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --workload topk_r50 --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('topk_r50', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'], d['cold_start']['compress_us'])"
