#!/bin/bash
# Reproducibility of the val-Dice oracle: the test after other GPU tests in the same process (as the round-end suite
# runs it) and standalone; both write their values (the oracle's must agree).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-valrepro}; mkdir -p $O; cd $R
OCTSAM_VALDICE_OUT=$O/after_model.json timeout -k 10 900 python -u -m pytest -x -q -s --timeout 800 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_upmask.py tests/test_gpu_val_dice.py > $O/pytest_a.log 2>&1; echo "rc_a=$?"
grep -E "after|fingerprint|passed|failed" $O/pytest_a.log | tail -8
OCTSAM_VALDICE_OUT=$O/alone.json timeout -k 10 900 python -u -m pytest -x -q -s --timeout 800 --timeout-method thread tests/test_gpu_val_dice.py > $O/pytest_b.log 2>&1; echo "rc_b=$?"
grep -E "after|fingerprint|passed|failed" $O/pytest_b.log | tail -8
