#!/bin/bash
# Val-Dice protocol: oracle spread under bf16-sized perturbations (round-3 cold-Adam protocol), warm start
# (weights + Adam state) generation, HIP vs oracle trajectory from the warm start.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04a}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_topo_w2.py tests/test_gpu_ph.py > $O/pytest_w2.log 2>&1 || { tail -30 $O/pytest_w2.log; exit 1; }
tail -1 $O/pytest_w2.log
timeout -k 10 420 python -u scripts/val_dice_warm.py --mode spread --every 4 --out $O/spread.jsonl > $O/spread.log 2>&1 || { tail -30 $O/spread.log; exit 1; }
timeout -k 10 240 python -u scripts/val_dice_warm.py --mode warm --steps 64 --every 8 --save $O/valdice_start_warm.safetensors --out $O/warm.jsonl > $O/warm.log 2>&1 || { tail -30 $O/warm.log; exit 1; }
timeout -k 10 300 python -u scripts/val_dice_warm.py --mode traj --warm $O/valdice_start_warm.safetensors --epochs 4 --every 8 --out $O/traj.jsonl > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
cat $O/traj.jsonl
