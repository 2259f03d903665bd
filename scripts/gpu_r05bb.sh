#!/bin/bash
# Round 5: the decoder's token-side GEMMs on hipBLASLt (bit 262144 = off): GEMM + step tests, step A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05bb}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $O/tests_gemm.log 2>&1; grep -E "passed|failed|FAILED" $O/tests_gemm.log | tail -15
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py \
  tests/test_gpu_model.py tests/test_gpu_step_oracle.py tests/test_gpu_dp.py tests/test_gpu_dec_attn.py > $O/tests_step.log 2>&1 || { tail -30 $O/tests_step.log; exit 1; }
tail -1 $O/tests_step.log
STEP_VARIANTS=default,blaslt_tok_off timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab.log 2>&1 || { tail -5 $O/step_ab.log; exit 1; }
tail -1 $O/step_ab.log
STEP_PIPELINE=0 STEP_VARIANTS=default,blaslt_tok_off timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab_seq.log 2>&1 || { tail -5 $O/step_ab_seq.log; exit 1; }
tail -1 $O/step_ab_seq.log
