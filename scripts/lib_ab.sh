#!/bin/bash
# A/B of two builds of liboctsam_hip.so on one box (outputs under gpurun_out/$TAG): GEMM variant times and the
# pipelined step, alternating processes. usage: TAG=x LIB_B=path bash scripts/lib_ab.sh
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-libab}; mkdir -p $O; cd $R
for rnd in 1 2; do
  for lib in default $LIB_B; do
    if [ $lib = default ]; then unset OCTSAM_LIB; else export OCTSAM_LIB=$R/$lib; fi
    GEMM_SHAPES=qkv_glob,fc1,fc2,proj GEMM_VARIANTS=default timeout -k 10 200 python scripts/gemm_variants.py \
      > $O/gv_${rnd}_$(basename $lib).log 2>&1 || exit $?
    echo "== $lib round $rnd"; grep '^{' $O/gv_${rnd}_$(basename $lib).log | cut -c1-120
    ROUNDS=2 timeout -k 10 300 python scripts/step_ab2.py 1:1 > $O/st_${rnd}_$(basename $lib).log 2>&1 || exit $?
    tail -1 $O/st_${rnd}_$(basename $lib).log
  done
done
