set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/qqv; mkdir -p $O; export TMPDIR=/tmp
for v in default qq_form0 qq_form0_nt qq_nt default; do
  L=""; [ $v != default ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
  timeout -k 10 200 python bench.py --workload qsgd --no-cpu-baseline --no-e2e $L > $O/bench_$v.json || exit 1
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v',d['value'],d['ms_per_step'],d['kernels_us'])"
done
