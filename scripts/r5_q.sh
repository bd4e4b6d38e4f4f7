#!/bin/bash
# Round-5 measurement, part 3: the workloads whose kernels changed after parts 1-2 (segmented warm tail; the
# fused-gossip K1 on cold runs) and the deferred sign step's PMC (its kernel now mapped).
R=r05 WLS="topk_r50 step_topk step_sign+defer" bash scripts/gpu_measure.sh
