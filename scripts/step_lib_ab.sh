#!/bin/bash
# Same-box A/B of two builds of liboctsam_hip.so on the training step (pipelined and sequential), alternating
# processes. usage: TAG=x LIB_B=ab_libs/name.so bash scripts/step_lib_ab.sh
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-steplibab}; mkdir -p $O; cd $R
for rnd in 1 2 3; do
  for lib in default $LIB_B; do
    if [ $lib = default ]; then unset OCTSAM_LIB; else export OCTSAM_LIB=$R/$lib; fi
    ROUNDS=2 timeout -k 10 300 python -u scripts/step_ab2.py 1:1 1:0 > $O/st_${rnd}_$(basename $lib).log 2>&1 || { tail -5 $O/st_${rnd}_$(basename $lib).log; exit 1; }
    echo "$lib round $rnd: $(tail -1 $O/st_${rnd}_$(basename $lib).log)"
  done
done
