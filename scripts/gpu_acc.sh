set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/acc; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "accumulate or round_trip or choco or multiproc" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in default chocosgd_amd/lib/variants/lib_acc_elem.so chocosgd_amd/lib/variants/lib_acc_seg8.so chocosgd_amd/lib/variants/lib_acc_seg32.so; do
  L=""; [ $v != default ] && L="--lib $v"
  for m in 1 3; do timeout -k 10 120 python tools/acc_bench.py $L --msgs $m || exit 1; done
done
timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e > $O/bench_topk.json || exit 1
python -c "import json;d=json.load(open('$O/bench_topk.json'));print(d['value'],d['ms_per_step'],d['kernels_us'])"
