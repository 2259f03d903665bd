#!/bin/bash
# octsam_wgrad parity + timing against the split-K GEMM; decoder / graph-step / attention tests; the default bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03j}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k wgrad > $O/pytest_wgrad.log 2>&1 || { tail -30 $O/pytest_wgrad.log; exit 1; }
tail -1 $O/pytest_wgrad.log
timeout -k 10 300 python -u scripts/dw_ab.py > $O/dw_ab.log 2>&1 || { tail -20 $O/dw_ab.log; exit 1; }
cat $O/dw_ab.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_graph_step.py tests/test_gpu_layers.py tests/test_gpu_pipeline.py tests/test_gpu_gemm.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
