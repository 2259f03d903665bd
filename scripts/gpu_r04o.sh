#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04o}; mkdir -p $O; cd $R
CU_VARIANTS=default,all:def,def:all,def:q1,def:h1,q3:def,def:even timeout -k 10 500 python -u scripts/cumask_step_ab.py > $O/cumask_ab.log 2>&1 || { tail -20 $O/cumask_ab.log; exit 1; }
tail -1 $O/cumask_ab.log
