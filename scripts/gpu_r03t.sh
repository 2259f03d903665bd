#!/bin/bash
# GEMM phase stamps (main loop / epilogue per tile, epilogue alignment across CUs) on the encoder shapes; GEMM tests.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03t}; mkdir -p $O; cd $R
timeout -k 10 200 python -u scripts/gemm_stamps.py > $O/gemm_stamps.log 2>&1 || { tail -20 $O/gemm_stamps.log; exit 1; }
cat $O/gemm_stamps.log | grep name
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
