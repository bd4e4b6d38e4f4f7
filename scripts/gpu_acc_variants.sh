# Bench the top-k step with accumulate store-policy variants.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/accv; mkdir -p $O; export TMPDIR=/tmp
for v in product acc_nt acc_sc1; do
  L=""; [ $v = product ] || L="--lib chocosgd_amd/lib/variants/lib_$v.so"
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e $L > $O/$v.json 2> $O/$v.err || { tail $O/$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$v.json')); print('$v', d['ms_per_step'], d['kernels_us'])"
done
