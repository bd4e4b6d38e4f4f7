#!/bin/bash
# Round-5 measurement, part 2: the gossip steps (plain and deferred receive) and the ring-3 loopback receive
R=r05 WLS="step_topk step_sign step_qsgd step_sign+defer step_qsgd+defer topk+ring3" bash scripts/gpu_measure.sh
