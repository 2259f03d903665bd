#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04m}; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/gemm_skew_ab.py > $O/gemm_skew_ab.log 2>&1 || { tail -20 $O/gemm_skew_ab.log; exit 1; }
cat $O/gemm_skew_ab.log
