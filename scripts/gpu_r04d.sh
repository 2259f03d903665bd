#!/bin/bash
# Round 4: graph-step variant test with the current and the HEAD attention libraries, window-attention timing of
# both, then the val-Dice diagnostics (oracle spread under bf16-sized perturbations; warm start; warm trajectory).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04d}; mkdir -p $O; cd $R
HEADLIB=$R/dilabhelmholtzoct_amd/liboctsam_hip_head.so
OCTSAM_LIB=$HEADLIB timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_graph_step.py > $O/graph_head.log 2>&1; echo "head rc=$?"; tail -1 $O/graph_head.log
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_graph_step.py > $O/graph_cur.log 2>&1; echo "cur rc=$?"; tail -1 $O/graph_cur.log
grep -E "PASSED|FAILED" $O/graph_head.log $O/graph_cur.log | cut -c1-150
OCTSAM_LIB=$HEADLIB timeout -k 10 200 python -u scripts/attn_time.py > $O/attn_head.log 2>&1 || { tail -5 $O/attn_head.log; exit 1; }
timeout -k 10 200 python -u scripts/attn_time.py > $O/attn_cur.log 2>&1 || { tail -5 $O/attn_cur.log; exit 1; }
grep side $O/attn_head.log $O/attn_cur.log
timeout -k 10 420 python -u scripts/val_dice_warm.py --mode spread --variants base,ulp1,ulp2,emb_bf16,hip --every 4 --out $O/spread.jsonl > $O/spread.log 2>&1 || { tail -30 $O/spread.log; exit 1; }
timeout -k 10 200 python -u scripts/val_dice_warm.py --mode warm --steps 64 --every 16 --save $O/valdice_start_warm.safetensors --out $O/warm.jsonl > $O/warm.log 2>&1 || { tail -30 $O/warm.log; exit 1; }
timeout -k 10 300 python -u scripts/val_dice_warm.py --mode traj --warm $O/valdice_start_warm.safetensors --epochs 4 --every 8 --out $O/traj.jsonl > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
cat $O/traj.jsonl
