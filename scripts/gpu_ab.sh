# A/B of library variants (chocosgd_amd/lib/variants/lib_<name>.so; "main" = the product
# library) on bench workloads: one line per (workload, variant) with the step time and the
# per-kernel event times.  LIBS="main old ..." WLS="qsgd step_qsgd" bash scripts/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/ab; mkdir -p $O; export TMPDIR=/tmp
for wl in $WLS; do
  for v in $LIBS; do
    L=""; [ "$v" != main ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
    timeout -k 10 200 python3 bench.py --workload $wl --no-cpu-baseline --no-e2e $L $EXTRA > $O/${wl}_$v.json 2> $O/${wl}_$v.err \
      || { tail -5 $O/${wl}_$v.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${wl}_$v.json').read().splitlines()[-1])
print('$wl', '$v', d['ms_per_step'], {k: round(v, 1) for k, v in d['kernels_us'].items()})"
  done
done
