#!/bin/bash
# Round-5 GPU pass Y: the sparse accumulate as return-less float atomics (agent / workgroup scope) -- parity on
# the variants, then a same-box A/B against the segment-owner kernel on topk and randk (decompress stage).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5y; mkdir -p $O; V=chocosgd_amd/lib/variants
for v in acc_atom_agent acc_atom_wg; do
  CHOCO_CODEC_LIB=$V/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse_multi.py tests/test_gpu_choco_api.py \
    tests/test_gpu_multiproc.py -k "topk and not deferred" -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests_$v.log | head -20; }
done
for rep in 1 2; do
for wl in topk randk; do
for v in base acc_atom_agent acc_atom_wg; do
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$wl $v', d['ms_per_step'], d['kernels_us'])"
done
done
done
