# Bench step time (top-k workload) for the product lib and each given variant.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/vb; mkdir -p $O; export TMPDIR=/tmp
for v in product ${VARIANTS}; do
  L=""; [ "$v" != product ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 50 $L > $O/b_$v.json 2> $O/b_$v.err || { tail $O/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$v.json')); print('%-10s'%'$v', d['value'], d['ms_per_step'], d['kernels_us'])"
done
