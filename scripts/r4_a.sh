#!/bin/bash
# Round-4 GPU pass A: floor probe, top-k parity (one-launch path), status probe, top-k bench.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4; mkdir -p $O
timeout -k 10 150 tools/probe_floor > $O/probe_floor.txt 2>&1 || { echo "probe rc=$?"; tail -20 $O/probe_floor.txt; }
tail -45 $O/probe_floor.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_topk.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/t_topk.log 2>&1
rc=$?; tail -4 $O/t_topk.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|error" $O/t_topk.log | head -30; tail -60 $O/t_topk.log; exit $rc; }
CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_poll1.so timeout -k 10 120 python -u tools/status_probe.py > $O/status_probe.txt 2>&1; echo "status probe rc=$?"; cat $O/status_probe.txt | tail -5
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $O/b_topk.json 2> $O/b_topk.err; rc=$?
python -c "import json; d=json.load(open('$O/b_topk.json')); print(d['value'], d['ms_per_step'], d['roofline'], d.get('kernels_us'), d.get('cold_start'))"
exit $rc
