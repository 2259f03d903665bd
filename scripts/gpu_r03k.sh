#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03k}; mkdir -p $O; cd $R
timeout -k 10 120 python -u scripts/wgrad_debug.py > $O/wgrad_debug.log 2>&1; rc=$?
cat $O/wgrad_debug.log | grep -v amdgpu.ids; exit $rc
