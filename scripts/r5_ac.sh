#!/bin/bash
# Round-5 GPU pass AC: the per-tensor (ResNet-50, 161 tensors) CHOCO steps -- sign and QSGD, plain and deferred --
# and a same-box A/B of the deferred sign receive: row runs with per-segment scales / sums (product) against the
# receive + fused pack as two kernels (variant signseg2k).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5ac; mkdir -p $O; V=chocosgd_amd/lib/variants
for rep in 1 2; do
for spec in "step_sign_r50" "step_sign_r50 --defer-receive" "step_sign_r50 --defer-receive --lib $V/lib_signseg2k.so" \
            "step_qsgd_r50" "step_qsgd_r50 --defer-receive"; do
  timeout -k 10 300 python bench.py --workload $spec --no-cpu-baseline --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$spec'.replace('$V/',''), d['ms_per_step'], d['roofline']['frac'], d['kernels_us'])"
done
done
