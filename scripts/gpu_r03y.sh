#!/bin/bash
# LayerNorm2d + GELU backward fused into the mask-head backward: parity, decoder tests, step A/B, kernel times.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03y}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_upmask.py > $O/pytest_upmask.log 2>&1 || { tail -30 $O/pytest_upmask.log; exit 1; }
tail -1 $O/pytest_upmask.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_graph_step.py tests/test_gpu_step_oracle.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
STEP_VARIANTS=default,ln_sep timeout -k 10 250 python -u scripts/step_ab3.py > $O/step_ab_ln.log 2>&1 || { tail -20 $O/step_ab_ln.log; exit 1; }
tail -1 $O/step_ab_ln.log
STEP_PIPELINE=0 STEP_VARIANTS=default,ln_sep timeout -k 10 250 python -u scripts/step_ab3.py > $O/step_ab_ln_seq.log 2>&1 || { tail -20 $O/step_ab_ln_seq.log; exit 1; }
tail -1 $O/step_ab_ln_seq.log
