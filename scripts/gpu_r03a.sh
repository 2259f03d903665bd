#!/bin/bash
# Round-3 first call: headline bench at HEAD + val-Dice trajectory on the 128/32 protocol.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03a}; mkdir -p $O; cd $R
timeout -k 10 420 python -u scripts/val_dice_traj.py --epochs ${EPOCHS:-8} --out $O/traj.jsonl > $O/traj.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.err
