#!/bin/bash
# Round 5: mask-head kernels, packed vs scalar GELU arithmetic (same-box library A/B, alternating).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05m}; mkdir -p $O; cd $R
for rnd in 1 2; do
  for lib in default ab_libs/liboctsam_um_scalar.so ab_libs/liboctsam_um_noslp.so; do
    n=$(basename $lib .so)_$rnd
    if [ $lib = default ]; then unset OCTSAM_LIB; else export OCTSAM_LIB=$R/$lib; fi
    timeout -k 10 200 python -u scripts/upmask_ab.py run $n > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
    tail -1 $O/$n.log
  done
done
unset OCTSAM_LIB
python scripts/upmask_ab.py cmp default_2 liboctsam_um_scalar_2
python scripts/upmask_ab.py cmp default_2 liboctsam_um_noslp_2
# global attention: exp2 partly from a polynomial on the FMA pipe (ATTN_POLY_EXP 1 / 2 of 8 pairs)
for rnd in 1 2; do
  for lib in default ab_libs/liboctsam_polyexp1.so ab_libs/liboctsam_polyexp2.so; do
    n=$(basename $lib .so)_$rnd
    if [ $lib = default ]; then unset OCTSAM_LIB; else export OCTSAM_LIB=$R/$lib; fi
    ATTN_GLOB=-1 timeout -k 10 200 python -u scripts/attn_lib_ab.py run $n > $O/attn_$n.log 2>&1 || { tail -5 $O/attn_$n.log; exit 1; }
    grep '"variant": -1' $O/attn_$n.log
  done
done
# accuracy of the polynomial variant against fp32 (the layer tests' tolerance)
OCTSAM_LIB=$R/ab_libs/liboctsam_polyexp2.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_gpu_layers.py -k "test_vit_attention and not token_ordered" > $O/attn_poly2_tests.log 2>&1; tail -3 $O/attn_poly2_tests.log
python scripts/attn_lib_ab.py cmp default_2 liboctsam_polyexp1_2 | grep '"variant": -1'
python scripts/attn_lib_ab.py cmp default_2 liboctsam_polyexp2_2 | grep '"variant": -1'
