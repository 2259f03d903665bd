#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04i}; mkdir -p $O; cd $R
timeout -k 10 200 python -u scripts/resid_ab.py > $O/resid_ab.log 2>&1 || { tail -20 $O/resid_ab.log; exit 1; }
cat $O/resid_ab.log
