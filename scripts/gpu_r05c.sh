#!/bin/bash
# Round 5: the LDS-staged fp32 residual epilogue A/B (bit-identity + time), the GEMM tests, the multi-seed val-Dice test
# (oracle-made warm start), then the default bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05c}; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/gemm_ab_res.py > $O/gemm_ab_res.log 2>&1 || { tail -20 $O/gemm_ab_res.log; exit 1; }
grep name $O/gemm_ab_res.log
grep -q '"bit_identical": false' $O/gemm_ab_res.log && { echo "NOT BIT-IDENTICAL"; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py > $O/pytest_gemm.log 2>&1 || { tail -30 $O/pytest_gemm.log; exit 1; }
tail -2 $O/pytest_gemm.log
OCTSAM_VALDICE_HIP_OUT=$O/valdice_hip.json timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_val_dice.py > $O/pytest_valdice.log 2>&1 || { grep -E "^pair|mean over|FAIL|Error|assert" $O/pytest_valdice.log | tail -30; exit 1; }
grep -E "^pair|mean over|passed|failed" $O/pytest_valdice.log
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
