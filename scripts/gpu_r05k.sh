#!/bin/bash
# Round 5: grouped token-side weight gradients: tests, step A/B (pipelined and sequential).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05k}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_graph_step.py \
  tests/test_gpu_model.py tests/test_gpu_step_oracle.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
STEP_VARIANTS=default,tokgroup_off,dkeys_two timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab.log 2>&1 || { tail -5 $O/step_ab.log; exit 1; }
tail -1 $O/step_ab.log
STEP_PIPELINE=0 STEP_VARIANTS=default,tokgroup_off timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab_seq.log 2>&1 || { tail -5 $O/step_ab_seq.log; exit 1; }
tail -1 $O/step_ab_seq.log
