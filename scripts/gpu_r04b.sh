#!/bin/bash
# Round-4 first GPU check of the re-entry commit: smoke, the W2/PH/step-oracle tests, then the val-Dice diagnostics.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04b}; mkdir -p $O; cd $R
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_topo_w2.py tests/test_gpu_ph.py tests/test_gpu_step_oracle.py tests/test_gpu_graph_step.py > $O/pytest_a.log 2>&1 || { tail -30 $O/pytest_a.log; exit 1; }
tail -1 $O/pytest_a.log
grep -E "DiceCE" $O/pytest_a.log || true
bash scripts/gpu_r04a.sh
