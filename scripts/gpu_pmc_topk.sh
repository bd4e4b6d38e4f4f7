# SQ counters of the top-k kernels at k ~ 1 and k = 1 %.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/pmc_topk; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
P2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM"
for r in 0.99999999 0.99; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $O/r${r}_p$i -o run --output-format csv -- python tools/topk_loop.py --ratio $r \
      > $O/r${r}_p$i.log 2>&1 || { tail -5 $O/r${r}_p$i.log; echo "pass failed"; }
  done
done
ls -R $O | head -30
