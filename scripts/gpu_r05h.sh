#!/bin/bash
# Round 5: val-Dice protocol variants (fp16 encoder, fused keys-gradient product) and the step's per-kernel issue profile.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05h}; mkdir -p $O; cd $R
timeout -k 10 600 python -u scripts/valdice_variants.py fp16,dkeys > $O/valdice_variants.log 2>&1 || { tail -5 $O/valdice_variants.log; exit 1; }
grep mean_diff $O/valdice_variants.log
TAG=r05h/pmc bash scripts/step_pmc.sh
