#!/bin/bash
# 256x192 ping-pong tiles: parity tests, isolated A/B on the encoder shapes, same-process step A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-n192w}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q -k "pingpong or small_oneshot or token_side" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VARIANTS=native,w256,gemm8 SHAPES=qkv,proj,fc1,fc2,fc2e16 timeout -k 10 300 python -u scripts/gemm8w_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep '^{' $O/ab.log | cut -c1-330
ROUNDS=3 timeout -k 10 400 python -u scripts/step_ab2.py 1:1 131073:1 1:0 131073:0 > $O/step_ab.log 2>&1 || { tail -20 $O/step_ab.log; exit 1; }
tail -5 $O/step_ab.log
