set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/nt; mkdir -p $O; export TMPDIR=/tmp
for v in product stream_nt; do
  L=""; [ $v = product ] || L="--lib chocosgd_amd/lib/variants/lib_$v.so"
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e $L > $O/$v.json 2> $O/$v.err || { tail $O/$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$v.json')); print('$v', d['ms_per_step'], d['kernels_us'])"
  timeout -k 10 200 python tools/diag_stream.py --only topk --modes hot,cold --ratios 0.99 $L > $O/diag_$v.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/diag_$v.log
done
