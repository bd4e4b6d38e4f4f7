#!/bin/bash
# Round-5 measurement, part 1: the codec workloads
R=r05 WLS="topk topk25m topk_r50 randk qsgd sign" bash scripts/gpu_measure.sh
