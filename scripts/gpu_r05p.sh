#!/bin/bash
# Round 5: persistence + transport forked beside the DiceCE backward (fork_topo) against the default, step A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05p}; mkdir -p $O; cd $R
STEP_VARIANTS=default,fork_topo timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab.log 2>&1 || { tail -5 $O/step_ab.log; exit 1; }
tail -1 $O/step_ab.log
STEP_PIPELINE=0 STEP_VARIANTS=default,fork_topo timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab_seq.log 2>&1 || { tail -5 $O/step_ab_seq.log; exit 1; }
tail -1 $O/step_ab_seq.log
