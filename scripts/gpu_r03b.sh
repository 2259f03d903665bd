#!/bin/bash
# The configs[3]/[4] step-vs-oracle test, then val-Dice trajectories on the 128/32 protocol: a long fp32-oracle vs
# HIP run (saving two oracle decoder start points, bf16) and the oracle under bf16 autocast.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03b}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_step_oracle.py tests/test_gpu_model.py > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/val_dice_traj.py --epochs 24 --seed 1 --save-at 256,384 --save-dir $O/start --out $O/traj_long.jsonl > $O/traj_long.log 2>&1 || exit $?
timeout -k 10 500 python -u scripts/val_dice_traj.py --epochs 16 --no-hip --ref-autocast --out $O/traj_autocast.jsonl > $O/traj_autocast.log 2>&1 || exit $?
