#!/bin/bash
# Makes the val-Dice protocol's fixtures with the fp32 oracle alone (tests/golden/make_valdice_golden.py): the
# oracle-made warm start (--warm) and the per-seed-pair oracle values + perturbation spread (--oracle), into
# gpurun_out/$TAG (copied into tests/golden/ by hand after the run). Depends on no HIP kernel, so it runs once.
# STEP=extend: only the seed pairs the committed golden lacks (--keep), then tests/test_gpu_val_dice.py against it.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-valdice_golden}; mkdir -p $O; cd $R
STEP=${STEP:-both}
if [ "$STEP" = warm ] || [ "$STEP" = both ]; then
  timeout -k 10 600 python -u tests/golden/make_valdice_golden.py --warm --warm-out $O/valdice_warm_oracle.safetensors > $O/warm.log 2>&1 || { tail -20 $O/warm.log; exit 1; }
  tail -2 $O/warm.log
  cp $O/valdice_warm_oracle.safetensors tests/golden/valdice_warm_oracle.safetensors
fi
if [ "$STEP" = oracle ] || [ "$STEP" = both ]; then
  timeout -k 10 1000 python -u tests/golden/make_valdice_golden.py --oracle --oracle-out $O/valdice_oracle.json > $O/oracle.log 2>&1 || { tail -20 $O/oracle.log; exit 1; }
  tail -4 $O/oracle.log
fi
if [ "$STEP" = extend ]; then  # run only the pairs the committed golden lacks, then the val-Dice test against it
  cp tests/golden/valdice_oracle.json $O/valdice_oracle.json
  timeout -k 10 900 python -u tests/golden/make_valdice_golden.py --oracle --keep --perturb ${PERTURB:-2} --oracle-out $O/valdice_oracle.json > $O/oracle.log 2>&1 || { tail -20 $O/oracle.log; exit 1; }
  tail -4 $O/oracle.log | cut -c1-300
  cp $O/valdice_oracle.json tests/golden/valdice_oracle.json
  OCTSAM_VALDICE_HIP_OUT=$O/valdice_hip.json timeout -k 10 500 python -u -m pytest -x -v -s --timeout 490 \
    --timeout-method thread tests/test_gpu_val_dice.py > $O/valdice.log 2>&1; rc=$?
  grep "mean over\|passed\|failed\|Error" $O/valdice.log | cut -c1-300
  exit $rc
fi
