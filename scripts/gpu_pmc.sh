# PMC counters for the top-k stream kernel (separate passes; no sys/runtime trace).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d gpurun_out/pmc/$name -o run --output-format csv -- \
    python tools/diag_stream.py --only ${WHAT:-topk} --modes hot --ratios 0.99 --reps 3 > gpurun_out/pmc/$name.log 2>&1
}
run p1 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM && \
run p2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run p3 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE && \
run p4 FETCH_SIZE && \
run p5 WRITE_SIZE && \
python tools/pmc_summary.py gpurun_out/pmc
