#!/bin/bash
# Small-problem GEMM with the epilogue operands prefetched: parity tests, per-launch A/B against the build without
# (ab_libs/liboctsam_small_nopre.so), same-box step A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-smallpre}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q -k "small or token_side or small_problem" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/tok_gemm_ab.py > $O/ab_pre.log 2>&1 || { tail -20 $O/ab_pre.log; exit 1; }
OCTSAM_LIB=$R/ab_libs/liboctsam_small_nopre.so timeout -k 10 200 python -u scripts/tok_gemm_ab.py > $O/ab_nopre.log 2>&1 || { tail -20 $O/ab_nopre.log; exit 1; }
paste -d'\n' <(grep '^{' $O/ab_pre.log | cut -c1-200) <(grep '^{' $O/ab_nopre.log | cut -c1-200)
TAG=${TAG}/step LIB_B=ab_libs/liboctsam_small_nopre.so bash scripts/step_lib_ab.sh
