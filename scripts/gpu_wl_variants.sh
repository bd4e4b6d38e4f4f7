# Bench lines of the given workloads for the product lib and each given variant.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/wv; mkdir -p $O; export TMPDIR=/tmp
for wl in ${WLS:-qsgd sign}; do
for v in product ${VARIANTS}; do
  L=""; [ "$v" != product ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-e2e $L ${BARGS} > $O/b_${wl}_$v.json 2> $O/b_${wl}_$v.err || { tail $O/b_${wl}_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${wl}_$v.json')); print('%-6s %-10s'%('$wl','$v'), d['value'], d['ms_per_step'], d['kernels_us'])"
done
done
