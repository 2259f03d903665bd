#!/bin/bash
# Round 4: fused DiceCE backward + post-processing row pass: parity tests, the step tests, same-process step A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04j}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fused_pp.py tests/test_gpu_losses.py tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
STEP_VARIANTS=default,pp_unfused timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab.log 2>&1 || { tail -10 $O/step_ab.log; exit 1; }
tail -4 $O/step_ab.log
