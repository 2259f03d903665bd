#!/bin/bash
# Round 4: graph-step tests at the reverted attention, the warm-start val-Dice trajectory, and a default bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04e}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_graph_step.py > $O/graph.log 2>&1 || { tail -30 $O/graph.log; exit 1; }
tail -1 $O/graph.log
timeout -k 10 200 python -u scripts/val_dice_warm.py --mode warm --steps 64 --every 16 --save $O/valdice_start_warm.safetensors --out $O/warm.jsonl > $O/warm.log 2>&1 || { tail -30 $O/warm.log; exit 1; }
timeout -k 10 400 python -u scripts/val_dice_warm.py --mode traj --warm $O/valdice_start_warm.safetensors --epochs 4 --every 8 --out $O/traj.jsonl > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
cat $O/traj.jsonl
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
