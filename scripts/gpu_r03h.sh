#!/bin/bash
# Global attention: 4-wave two-workgroups-per-CU variant vs the 8-wave kernel (timing + bit identity); step A/B of
# the forked topological forward; the step / W2 / loss tests.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03h}; mkdir -p $O; cd $R
ATTN_VARIANTS=1,2 timeout -k 10 300 python -u scripts/attn_ab.py > $O/attn_ab.log 2>&1 || exit $?
grep side $O/attn_ab.log
timeout -k 10 300 python -u scripts/step_ab3.py > $O/step_ab3.log 2>&1 || exit $?
tail -1 $O/step_ab3.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_topo_w2.py tests/test_gpu_losses.py tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py tests/test_gpu_training_loop.py tests/test_gpu_layers.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; exit $rc
