#!/bin/bash
# The val-Dice parity test alone (96 seed pairs against the committed oracle golden), its HIP column kept as JSON.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-valdice}; mkdir -p $O; cd $R
export OCTSAM_VALDICE_HIP_OUT=$O/hip.json
t0=$(date +%s)
timeout -k 10 ${LIMIT:-1000} python -u -m pytest tests/test_gpu_val_dice.py -m gpu -x -s -q --timeout 950 \
  --timeout-method thread > $O/pytest_valdice.log 2>&1
rc=$?
grep -E "mean over pairs|^\{\"step|passed|failed" $O/pytest_valdice.log | tail -12
echo "elapsed $(( $(date +%s) - t0 )) s"
exit $rc
