#!/bin/bash
# Round 4: PH phase split, stream-priority A/B (no host sync inside the step since round 3), the oracle's own spread
# along the warm-start trajectory, and the per-epoch val-Dice test.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04f}; mkdir -p $O; cd $R
timeout -k 10 60 ./scripts/micro/ph_timing_probe > $O/ph_timing.log 2>&1 || { tail -5 $O/ph_timing.log; exit 1; }
cat $O/ph_timing.log
VARS=2:0,2:-1 timeout -k 10 300 python -u scripts/prio_ab.py > $O/prio_ab.log 2>&1 || { tail -5 $O/prio_ab.log; exit 1; }
tail -2 $O/prio_ab.log
timeout -k 10 200 python -u scripts/val_dice_warm.py --mode warm --steps 64 --every 64 --save $O/warm.safetensors --out $O/warm.jsonl > $O/warm.log 2>&1 || { tail -30 $O/warm.log; exit 1; }
timeout -k 10 600 python -u scripts/val_dice_warm.py --mode spread --warm $O/warm.safetensors --epochs 4 --every 8 --variants base,ulp1,ulp2,ulp3,emb_bf16,hip --out $O/spread_warm.jsonl > $O/spread_warm.log 2>&1 || { tail -30 $O/spread_warm.log; exit 1; }
rm -f $O/warm.safetensors
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_gpu_val_dice.py > $O/valdice.log 2>&1; echo "valdice rc=$?"
grep -E "after|specificity|PASS|FAIL|Error" $O/valdice.log | head -20
