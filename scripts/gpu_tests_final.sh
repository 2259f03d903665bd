#!/bin/bash
# Round end: smoke + the whole GPU test suite (one process), as the driver runs them at round end.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-tests}; mkdir -p $O; cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
