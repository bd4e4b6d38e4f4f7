# Round measurement for the workloads in $WLS: PMC FETCH/WRITE passes (-> profiles/
# pmc_traffic.json), a rocprofv3 --kernel-trace --stats run, then the bench line (CPU
# baseline included).  Summaries land in gpurun_out/measure/; copy what is judged
# into profiles/.  A workload spec is name[+mode...]: "+defer" runs with --defer-receive,
# "+ring3" with --ring3-loopback, "+nograd" with
# --grad-lr 0 (round 5's synthetic step state); the PMC key is bench.traffic_key of the same
# flags; R names the round (default r06).  PMC medians and the *_kernel_stats_tail.csv
# summary keep each kernel's last dispatches (the step workloads' 200 burn-in steps run in
# the profiled process; rocprofv3's own kernel_stats.csv averages over them too).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/measure; mkdir -p $O; export TMPDIR=/tmp
for spec in $WLS; do
  wl=${spec%%+*}; F=""; tag=$wl
  rest=$spec
  while [ "$rest" != "${rest#*+}" ]; do
    rest=${rest#*+}; mode=${rest%%+*}
    case $mode in
      defer) F="$F --defer-receive"; tag=${tag}_deferred ;;
      ring3) F="$F --ring3-loopback"; tag=${tag}_ring3 ;;
      nograd) F="$F --grad-lr 0"; tag=${tag}_nograd ;;
      *) echo "unknown mode $mode"; exit 1 ;;
    esac
  done
  key=$(python3 -c "import bench; print(bench.traffic_key(bench.parse('--workload $wl $F'.split())))") || exit 1
  B="bench.py --workload $wl $F --steps 3 --warmup 2 --no-cpu-baseline --no-e2e"
  rm -rf /tmp/pf /tmp/pw
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o f -- python3 $B > $O/pmcf_$tag.log 2>&1 \
    || { tail -5 $O/pmcf_$tag.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o w -- python3 $B > $O/pmcw_$tag.log 2>&1 \
    || { tail -5 $O/pmcw_$tag.log; exit 1; }
  N=$(python3 -c "import bench; print(bench.WORKLOADS['$wl'][1] if not '$wl'.endswith('_r50') else 25557032)")
  # the last 10 dispatches per kernel: the step workloads' burn-in runs in the same process
  python3 tools/pmc_traffic.py /tmp/pf /tmp/pw $key $N --tail 10 > $O/pmc_$tag.txt || exit 1
  rm -rf /tmp/pk
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk -o k -- python3 bench.py --workload $wl $F \
    --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/prof_$tag.json 2> $O/prof_$tag.err || { tail -5 $O/prof_$tag.err; exit 1; }
  cp $(find /tmp/pk -name "*kernel_stats.csv" | head -1) $O/${R:-r06}_${tag}_kernel_stats.csv || exit 1
  # the same run's last 20 dispatches per kernel (the timed steps; the stats above include the burn-in)
  python3 tools/kstats_tail.py $(find /tmp/pk -name "*kernel_trace.csv" | head -1) 20 > $O/${R:-r06}_${tag}_kernel_stats_tail.csv || exit 1
  timeout -k 10 300 python3 bench.py --workload $wl $F > $O/bench_$tag.json 2> $O/bench_$tag.err \
    || { tail -5 $O/bench_$tag.err; exit 1; }
  echo "$tag done: $(python3 -c "import json; d=json.loads(open('$O/bench_$tag.json').read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['stage'], r['frac'], r['traffic'], (d.get('warm_start') or {}).get('warm_call_share'))")"
done
cp profiles/pmc_traffic.json $O/pmc_traffic.json
