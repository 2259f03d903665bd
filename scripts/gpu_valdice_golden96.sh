#!/bin/bash
# Extends the val-Dice oracle golden (tests/golden/valdice_oracle.json) to valdice_protocol.SEEDS with the fp32 oracle
# alone: new pairs get one bf16-sized perturbed run, kept pairs without one get it (--fill 1). The file is rewritten
# after every pair and the run stops starting pairs after DEADLINE seconds, so several calls continue each other
# (copy gpurun_out/$TAG/valdice_oracle.json into tests/golden/ between calls).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-vg}; mkdir -p $O; cd $R
cp tests/golden/valdice_oracle.json $O/valdice_oracle.json
timeout -k 10 ${LIMIT:-1080} python -u tests/golden/make_valdice_golden.py --oracle --keep --perturb 1 --fill 1 \
  --deadline ${DEADLINE:-960} --oracle-out $O/valdice_oracle.json > $O/oracle.log 2>&1; rc=$?
tail -3 $O/oracle.log | cut -c1-300
exit $rc
