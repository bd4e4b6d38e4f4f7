#!/bin/bash
# Round-5 GPU pass AU: the sign accumulate non-temporal on large buffers (n >= 2^25) -- tests, then the round
# measurement of sign and step_sign, and sign_r50 (plain policy).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5au; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd_sign.py tests/test_gpu_baseline_sizes.py tests/test_gpu_deferred_receive.py \
  tests/test_gpu_consumers.py tests/test_gpu_choco_api.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --workload sign_r50 --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || exit 1
python -c "import json; d=json.load(open('$O/b.json')); print('sign_r50', d['ms_per_step'], d['kernels_us'])"
WLS="sign step_sign" bash scripts/gpu_measure.sh
