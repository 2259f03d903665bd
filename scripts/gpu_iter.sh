#!/bin/bash
# Quick GPU iteration: selected GPU tests, bench (no CPU baseline / val), rocprofv3 kernel stats.
# usage: TAG=x bash scripts/gpu_iter.sh tests/test_a.py tests/test_b.py
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-it}
mkdir -p $O
cd $R
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/t.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --cpu-baseline 0 --val 0 > $O/b.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $O/b.log | cut -c1-220
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --cpu-baseline 0 --val 0 > $O/prof.log 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
