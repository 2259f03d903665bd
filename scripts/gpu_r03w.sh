#!/bin/bash
# PMC passes over the 8192^3 GEMM: gemm4x (fast path 25) vs the default 8-phase kernel.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03w}; mkdir -p $O
for F in 25 1; do
  FAST=$F TAG=r03w/f$F ARGS="8192 8192 8192" bash $R/scripts/gemm_pmc.sh > $O/f$F.log 2>&1 || { cat $O/f$F.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $O/f$F gemm > $O/f$F.summary.txt
  cat $O/f$F.summary.txt
  rm -rf $O/f$F/kt $O/f$F/p1 $O/f$F/p2 $O/f$F/p3 $O/f$F/p4
done
