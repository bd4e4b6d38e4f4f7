#!/bin/bash
# SQ counter passes: QSGD quantize, segmented W2; then the poll1 status probe.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4sq; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1; echo "list rc=$?"
for c in SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE; do
  grep -q "\b$c\b" $O/avail.txt && echo "have $c" || echo "MISSING $c"
done
P1="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for wl in qsgd topk_r50; do
  B="bench.py --workload $wl --steps 3 --warmup 2 --no-cpu-baseline --no-e2e"
  for p in 1 2; do
    eval P0=\$P$p; P=""
    for c in $P0; do grep -q "\b$c\b" $O/avail.txt && P="$P $c"; done
    [ -z "$P" ] && continue
    rm -rf /tmp/ps$p
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d /tmp/ps$p -o s -- python3 $B > $O/pmc${p}_$wl.log 2>&1 || { tail -5 $O/pmc${p}_$wl.log; exit 1; }
    python3 tools/pmc_sq.py /tmp/ps$p qsgd_ seg_ sparse_acc > $O/sq${p}_$wl.txt || exit 1
  done
  echo "== $wl"; cat $O/sq1_$wl.txt $O/sq2_$wl.txt
done
CHOCO_CODEC_LIB=chocosgd_amd/lib/variants/lib_poll1.so timeout -k 10 120 python3 tools/status_probe.py > $O/status_probe.txt 2>&1; echo "status probe rc=$?"; tail -5 $O/status_probe.txt
