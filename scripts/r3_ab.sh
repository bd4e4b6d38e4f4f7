# r3: optional GPU test files ($FILES), then a same-box A/B of library variants on bench
# workloads, two alternating passes: LIBS="main k2late" WLS="topk" FILES=tests/test_gpu_topk.py
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
if [ -n "$FILES" ]; then
  timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/ab_tests.log 2>&1
  rc=$?; tail -3 $O/ab_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/ab_tests.log | head -20; exit $rc; }
fi
for pass in 1 2; do
  for wl in $WLS; do
    for v in $LIBS; do
      L=""; [ "$v" != main ] && L="--lib chocosgd_amd/lib/variants/lib_$v.so"
      timeout -k 10 200 python3 bench.py --workload $wl --no-cpu-baseline --no-e2e $L $EXTRA > $O/ab_${wl}_$v.json 2> $O/ab_${wl}_$v.err \
        || { tail -5 $O/ab_${wl}_$v.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/ab_${wl}_$v.json').read().splitlines()[-1])
print('$wl', '$v', d['ms_per_step'], round(d['roofline']['frac'], 4), {k: round(v, 1) for k, v in d['kernels_us'].items()})"
    done
  done
done
