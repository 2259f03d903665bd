#!/bin/bash
# One-shot windowed attention (parity, A/B vs the tile-ring kernel, step A/B) + postproc_fwd staging fix (parity).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03s}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_losses.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ATTN_SIDES=14 ATTN_WVARIANTS=0,-1 timeout -k 10 200 python -u scripts/attn_ab.py > $O/attn_win_ab.log 2>&1 || { tail -20 $O/attn_win_ab.log; exit 1; }
cat $O/attn_win_ab.log | grep side
STEP_VARIANTS=default,win_ring timeout -k 10 250 python -u scripts/step_ab3.py > $O/step_ab_win.log 2>&1 || { tail -20 $O/step_ab_win.log; exit 1; }
tail -1 $O/step_ab_win.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_graph_step.py tests/test_gpu_vitl.py > $O/pytest2.log 2>&1 || { tail -30 $O/pytest2.log; exit 1; }
tail -1 $O/pytest2.log
