#!/bin/bash
# Round 5: residual-through-LDS A/B incl. gemm4w proj, then the val-Dice diagnostics (fp16 encoder; oracle decoder on
# HIP embeddings; oracle with bf16-rounded embeddings).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05d}; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/gemm_ab_res.py > $O/gemm_ab_res.log 2>&1 || { tail -20 $O/gemm_ab_res.log; exit 1; }
grep name $O/gemm_ab_res.log
grep -q '"bit_identical": false' $O/gemm_ab_res.log && { echo "NOT BIT-IDENTICAL"; exit 1; }
timeout -k 10 1000 python -u scripts/val_dice_diag.py > $O/valdice_diag.log 2>&1 || { tail -20 $O/valdice_diag.log; exit 1; }
grep variant $O/valdice_diag.log
