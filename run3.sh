cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 ./tools/probe_hbm > gpurun_out/probe_hbm.log 2>&1; echo "probe rc=$?"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --workload sign --no-cpu-baseline > gpurun_out/bench_sign.log 2>&1; echo "sign rc=$?"
