#!/bin/bash
# Per-kernel tables of the training step alone (sequential and pipelined), rocprofv3 kernel trace.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03o}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for P in 0 1; do
  PIPE=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$P -o run -- python3 $R/scripts/step_prof.py > $O/p$P.log 2>&1 || { tail -5 $O/p$P.log; exit 1; }
  python3 $R/scripts/prof_summary.py $O/p$P $O/step_kernels_pipe$P.csv --delete-trace || exit 1
  grep ms/step $O/p$P.log
done
