#!/bin/bash
# Round 5: last-wave K split of the encoder GEMMs: GEMM tests, kernel A/B, same-process step A/B (pipelined and
# sequential), graph-step tests.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05i}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_graph_step.py \
  tests/test_gpu_model.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u scripts/ksplit_ab.py > $O/ksplit_ab.log 2>&1 || { tail -5 $O/ksplit_ab.log; exit 1; }
cat $O/ksplit_ab.log
ROUNDS=3 timeout -k 10 500 python -u scripts/step_ab2.py 1:1 8193:1 1:0 8193:0 > $O/step_ab.log 2>&1 || { tail -5 $O/step_ab.log; exit 1; }
tail -6 $O/step_ab.log
