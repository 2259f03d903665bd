#!/bin/bash
# Round 5: dual-accumulator GEMM micro-benchmark v2, then the val-Dice oracle golden (per seed pair + spread).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05b}; mkdir -p $O; cd $R
timeout -k 10 120 ./scripts/micro/gemm8d > $O/gemm8d.log 2>&1 || { tail -20 $O/gemm8d.log; exit 1; }
cat $O/gemm8d.log
TAG=${TAG:-r05b} STEP=oracle bash scripts/gpu_valdice_golden.sh || exit 1
