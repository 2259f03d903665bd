#!/bin/bash
# Round 5: decoder attention precision (fp32 delta, P / dO / dS hi + lo) and the ViT attention asm-read A/B:
# kernel tests, attention old-vs-new library A/B, layer tests, gradient diagnostics, val-Dice.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05f}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_dec_attn.py \
  > $O/dec_attn.log 2>&1; rc=$?
grep "rel-Frob\|passed\|failed" $O/dec_attn.log | cut -c1-330
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u scripts/attn_lib_ab.py run new_a > $O/attn_new_a.log 2>&1 || { tail -5 $O/attn_new_a.log; exit 1; }
OCTSAM_LIB=$R/ab_libs/liboctsam_old_attn.so timeout -k 10 200 python -u scripts/attn_lib_ab.py run old > $O/attn_old.log 2>&1 || { tail -5 $O/attn_old.log; exit 1; }
ATTN_WIN=100,101 timeout -k 10 200 python -u scripts/attn_lib_ab.py run new_b > $O/attn_new_b.log 2>&1 || { tail -5 $O/attn_new_b.log; exit 1; }
grep differs $O/attn_new_b.log
timeout -k 10 100 python -u scripts/attn_lib_ab.py cmp old new_b > $O/attn_cmp.log 2>&1; cat $O/attn_cmp.log
timeout -k 10 100 python -u scripts/attn_lib_ab.py cmp old new_a > $O/attn_cmp_a.log 2>&1; cat $O/attn_cmp_a.log
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_graph_step.py \
  > $O/layers.log 2>&1; tail -2 $O/layers.log
timeout -k 10 600 python -u scripts/grad_diag.py > $O/grad_diag.log 2>&1 || { tail -20 $O/grad_diag.log; exit 1; }
grep state $O/grad_diag.log | cut -c1-600
OCTSAM_VALDICE_HIP_OUT=$O/valdice_hip.json timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 \
  --timeout-method thread tests/test_gpu_val_dice.py > $O/valdice.log 2>&1; rc=$?
tail -25 $O/valdice.log
exit $rc
