#!/bin/bash
# Round 5: scalar vs packed f32 softmax arithmetic in the ViT attention (bit-identity, kernel times, step A/B), layer
# tests; the GEMM call list of one step.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05l}; mkdir -p $O; cd $R
for rnd in 1 2; do
  ATTN_GLOB=-1,2 timeout -k 10 200 python -u scripts/attn_lib_ab.py run scalar$rnd > $O/ab_scalar$rnd.log 2>&1 || { tail -5 $O/ab_scalar$rnd.log; exit 1; }
  OCTSAM_LIB=$R/ab_libs/liboctsam_attn_pk.so ATTN_GLOB=-1,2 timeout -k 10 200 python -u scripts/attn_lib_ab.py run pk$rnd > $O/ab_pk$rnd.log 2>&1 || { tail -5 $O/ab_pk$rnd.log; exit 1; }
done
python scripts/attn_lib_ab.py cmp pk1 scalar1; python scripts/attn_lib_ab.py cmp pk2 scalar2
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_layers.py > $O/layers.log 2>&1; tail -1 $O/layers.log
TOP=120 timeout -k 10 300 python -u scripts/gemm_calls.py > $O/gemm_calls.log 2>&1; head -3 $O/gemm_calls.log
