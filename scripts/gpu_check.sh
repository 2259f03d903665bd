#!/bin/bash
# GPU-box check used each round: smoke, pytest -m gpu, bench, rocprofv3 kernel stats (outputs under gpurun_out/$TAG).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r01}
mkdir -p $O
cd $R
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -2 $O/bench.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${PROBES:-}" ]; then
  timeout -k 10 200 python scripts/hbm_probe.py > $O/hbm_probe.log 2>&1 || exit $?
  timeout -k 10 200 python scripts/gemm_ksweep.py > $O/ksweep.log 2>&1 || exit $?
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --cpu-baseline 0 --val 0 > $O/prof.log 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
