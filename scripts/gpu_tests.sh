#!/bin/bash
# smoke + pytest -m gpu on the GPU box (outputs under gpurun_out/$TAG); stops at the first failing step.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r02}
mkdir -p $O
cd $R
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q ${PYTEST_ARGS:-} --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 $O/pytest_gpu.log
exit $rc
