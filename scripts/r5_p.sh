#!/bin/bash
# Round-5 GPU pass P: same-box A/B of the sign packs' row offsets (VGPR offsets, product) against round 4's form
# (sgn_old: a VGPR-derived scalar offset, readfirstlane loops) on sign, step_sign, step_sign --defer-receive;
# the fused-gossip pack in 4-row groups (sgs4) on step_sign.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5p; mkdir -p $O; V=chocosgd_amd/lib/variants
timeout -k 10 200 python tools/debug_sign_fused.py $V/lib_sgn_old.so > $O/debug.log 2>&1; grep -c ": ok" $O/debug.log
timeout -k 10 200 python tools/debug_sign_fused.py $V/lib_sgs4.so > $O/debug4.log 2>&1; grep -c ": ok" $O/debug4.log
for rep in 1 2; do
for wl in sign step_sign step_sign+defer; do
for v in base sgn_old sgs4; do
  [ $v = sgs4 ] && [ $wl != step_sign ] && continue
  w=${wl%%+*}; F=""; [ "$wl" != "$w" ] && F="--defer-receive"
  L=""; [ $v != base ] && L="--lib $V/lib_$v.so"
  timeout -k 10 300 python bench.py --workload $w $F --no-cpu-baseline --no-e2e $L > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); r=d['roofline']; print('$wl $v', d['ms_per_step'], r['kernel_us'], r['frac'], d['kernels_us'])"
done
done
done
