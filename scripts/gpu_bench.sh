# Bench lines for every workload on one MI355X (gpurun); the default (top-k) line
# carries the e2e leg and the CPU baseline.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/bench; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench_topk.json 2> $O/bench_topk.err || { tail -20 $O/bench_topk.err; exit 1; }
for wl in ${WLS:-topk25m topk_r50 randk qsgd sign}; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err \
    || { tail -20 $O/bench_$wl.err; exit 1; }
done
cat $O/bench_*.json
