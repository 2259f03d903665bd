#!/bin/bash
# Round 5: the fused-pp fallback tests, the dual-accumulator GEMM micro-benchmark, GEMM calibration on this box
# (variants, stamps), the oracle-made val-Dice warm start.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05a}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fused_pp.py > $O/pytest_fused_pp.log 2>&1 || { tail -30 $O/pytest_fused_pp.log; exit 1; }
tail -2 $O/pytest_fused_pp.log
timeout -k 10 120 ./scripts/micro/gemm8d > $O/gemm8d.log 2>&1 || { tail -20 $O/gemm8d.log; exit 1; }
cat $O/gemm8d.log
GEMM_SHAPES=qkv_glob,proj,fc1,fc2 GEMM_VARIANTS=default,single,p1tile,p_nostore,noepi,noloop,blaslt timeout -k 10 300 python -u scripts/gemm_variants.py > $O/gemm_variants.log 2>&1 || { tail -5 $O/gemm_variants.log; exit 1; }
cat $O/gemm_variants.log | grep name
timeout -k 10 200 python -u scripts/gemm_stamps.py > $O/gemm_stamps.log 2>&1 || { tail -5 $O/gemm_stamps.log; exit 1; }
cut -c1-400 $O/gemm_stamps.log
TAG=${TAG:-r05a} STEP=warm bash scripts/gpu_valdice_golden.sh || exit 1
