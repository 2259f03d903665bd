#!/bin/bash
# Same-process step A/B over octsam_gemm fast-path settings (pipelined and sequential).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-stepflags}; mkdir -p $O; cd $R
ROUNDS=${ROUNDS:-3} timeout -k 10 ${LIMIT:-600} python -u scripts/step_ab2.py ${VARIANTS} > $O/step_ab.log 2>&1 || { tail -20 $O/step_ab.log; exit 1; }
tail -1 $O/step_ab.log
