#!/bin/bash
# octsam_wgrad_tok parity; decoder / step tests; step A/B token-side fused dW on/off (pipelined + sequential).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03p}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "wgrad" > $O/pytest_wgrad.log 2>&1 || { tail -30 $O/pytest_wgrad.log; exit 1; }
tail -1 $O/pytest_wgrad.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py tests/test_gpu_step_oracle.py tests/test_gpu_vitl.py tests/test_gpu_vith.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
STEP_VARIANTS=default,tok_off timeout -k 10 250 python -u scripts/step_ab3.py > $O/step_ab_tok.log 2>&1 || exit 1
tail -1 $O/step_ab_tok.log
STEP_PIPELINE=0 STEP_VARIANTS=default,tok_off timeout -k 10 250 python -u scripts/step_ab3.py > $O/step_ab_tok_seq.log 2>&1 || exit 1
tail -1 $O/step_ab_tok_seq.log
