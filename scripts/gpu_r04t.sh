#!/bin/bash
# Round 4: the keys gradient of the mask head and the final attention as one product (strided d up1pre): parity tests,
# step A/B, kernel stats.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04t}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_upmask.py tests/test_gpu_model.py tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py tests/test_gpu_step_oracle.py > $O/pytest_t.log 2>&1 || { tail -30 $O/pytest_t.log; exit 1; }
tail -1 $O/pytest_t.log
STEP_VARIANTS=default,dkeys_sep timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab_dkeys.log 2>&1 || { tail -20 $O/step_ab_dkeys.log; exit 1; }
tail -1 $O/step_ab_dkeys.log
