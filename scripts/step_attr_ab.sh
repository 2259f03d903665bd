#!/bin/bash
# Same-box A/B of a mask-decoder attribute setting on the training step, alternating processes (three rounds).
# usage: TAG=x ATTRS_B="tok_flush_block=0" [STEP_ATTRS_B="fork_topo=0"] [VARIANTS="1:1 513:1"] bash scripts/step_attr_ab.sh
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-stepattr}; mkdir -p $O; cd $R
for rnd in 1 2 3; do
  for arm in A B; do
    if [ $arm = A ]; then export DEC_ATTRS="" STEP_ATTRS=""; else export DEC_ATTRS="${ATTRS_B:-}" STEP_ATTRS="${STEP_ATTRS_B:-}"; fi
    ROUNDS=2 timeout -k 10 300 python -u scripts/step_ab2.py ${VARIANTS:-1:1 1:0} > $O/st_${rnd}_$arm.log 2>&1 || { tail -5 $O/st_${rnd}_$arm.log; exit 1; }
    echo "$arm ($DEC_ATTRS $STEP_ATTRS) round $rnd: $(tail -1 $O/st_${rnd}_$arm.log)"
  done
done
