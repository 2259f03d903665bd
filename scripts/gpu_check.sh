#!/bin/bash
# GPU-box check used each round: smoke, pytest -m gpu, bench, rocprofv3 kernel stats (outputs under gpurun_out/r01).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r01}
mkdir -p $O
cd $R
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -2 $O/bench.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --cpu-baseline 0 --val 0 > $O/prof.log 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
