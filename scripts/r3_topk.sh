cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/t_topk.log 2>&1
rc=$?; tail -5 $O/t_topk.log; [ $rc -ne 0 ] && { tail -40 $O/t_topk.log; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $O/b_topk.json 2> $O/b_topk.err; rc=$?
cat $O/b_topk.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
exit $rc
