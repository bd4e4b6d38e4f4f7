# Round measurement on one MI355X: parity tests, PMC traffic, kernel-trace stats, bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/round; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -x > $O/gpu_tests.log 2>&1 \
  || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e"
for wl in topk qsgd sign; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f_$wl -o run --output-format csv -- $B --workload $wl \
    > $O/pmc_f_$wl.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w_$wl -o run --output-format csv -- $B --workload $wl \
    > $O/pmc_w_$wl.log 2>&1 || exit $?
done
python tools/pmc_traffic.py $O/pmc_f_topk $O/pmc_w_topk topk_stream_kernel topk:100000000 && \
python tools/pmc_traffic.py $O/pmc_f_topk $O/pmc_w_topk topk_finish_kernel topk_finish:100000000 && \
python tools/pmc_traffic.py $O/pmc_f_topk $O/pmc_w_topk sparse_acc_kernel sparse_acc:1000000 && \
python tools/pmc_traffic.py $O/pmc_f_qsgd $O/pmc_w_qsgd qsgd_quant_kernel qsgd:100000000 && \
python tools/pmc_traffic.py $O/pmc_f_sign $O/pmc_w_sign sign_pack sign:345000000 && \
cp profiles/pmc_traffic.json $O/ || exit 1
for wl in topk topk25m qsgd sign; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$wl -o run --output-format csv -- \
    python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/prof_$wl.log 2>&1 || exit $?
  python tools/kstats.py $(find $O/prof_$wl -name "*kernel_stats.csv") | head -8
done
timeout -k 10 500 python bench.py > $O/bench_topk.json 2> $O/bench_topk.err || exit $?
for wl in topk25m qsgd sign; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || exit $?
done
cat $O/bench_*.json
