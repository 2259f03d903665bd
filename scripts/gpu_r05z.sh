#!/bin/bash
# Round 5: the encoder's QKV on hipBLASLt too (fast path bit 131072), step A/B pipelined + sequential.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05z}; mkdir -p $O; cd $R
STEP_VARIANTS=default,blaslt_qkv timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab.log 2>&1 || { tail -5 $O/step_ab.log; exit 1; }
tail -1 $O/step_ab.log
STEP_PIPELINE=0 STEP_VARIANTS=default,blaslt_qkv timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab_seq.log 2>&1 || { tail -5 $O/step_ab_seq.log; exit 1; }
tail -1 $O/step_ab_seq.log
