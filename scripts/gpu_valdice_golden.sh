#!/bin/bash
# Regenerates the oracle side of the val-Dice protocol (tests/golden/valdice_oracle.json) after a change to the HIP
# step's numerics: the protocol's warm start is 64 HIP steps, so the oracle's trajectory starts from the HIP code's
# own warm state. Runs tests/test_gpu_val_dice.py (which asserts every epoch within +-0.005) and writes its values.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-valdice}; mkdir -p $O; cd $R
OCTSAM_VALDICE_OUT=$O/valdice_oracle_run.json timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_val_dice.py > $O/pytest_valdice.log 2>&1 || { tail -30 $O/pytest_valdice.log; exit 1; }
grep -E "after|fingerprint|passed|failed" $O/pytest_valdice.log
cat $O/valdice_oracle_run.json
