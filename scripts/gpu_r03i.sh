#!/bin/bash
# Image-side dW timing (split counts, torch.mm bar); graph-step / attention tests after the 4-wave global-attention
# default and the fork_topo=False default; the default bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03i}; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/dw_ab.py > $O/dw_ab.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_graph_step.py tests/test_gpu_layers.py tests/test_gpu_pipeline.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/dw_ab.log
cut -c1-400 $O/bench.json
