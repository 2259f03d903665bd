#!/bin/bash
# GPU box: bench.py (default config) then a rocprofv3 kernel-trace/stats pass of the same command.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r01}
mkdir -p $O
cd $R
timeout -k 10 500 python bench.py "$@" > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -3 $O/bench.err; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --cpu-baseline 0 --val 0 > $O/prof.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -2 $O/prof.log
exit $rc
