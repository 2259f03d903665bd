#!/bin/bash
# Pipelined global attention A/B + parity, per-call step breakdown, and an fp32-oracle start point for the
# val-Dice test (seed-0 data, saved after the oracle leaves the all-foreground regime).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03c}; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/attn_ab.py > $O/attn_ab.log 2>&1 || exit $?
cat $O/attn_ab.log | grep side
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layers.py > $O/pytest_layers.log 2>&1 || exit $?
tail -2 $O/pytest_layers.log
timeout -k 10 300 python -u scripts/step_breakdown.py > $O/breakdown.log 2>&1 || exit $?
timeout -k 10 500 python -u scripts/val_dice_traj.py --epochs 16 --seed 0 --no-hip --save-at 192,256 --save-dir $O/start --out $O/traj_oracle0.jsonl > $O/traj_oracle0.log 2>&1 || exit $?
