#!/bin/bash
# GEMM A/B (two-workgroup 256x128 kernel vs 8-phase 256x256, both with the uniform-wave epilogue fix), step A/B
# (device vs host W2, copy-in), GEMM / step-oracle / training-loop tests, bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03e}; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/gemm_ab.py > $O/gemm_ab.log 2>&1 || exit $?
grep name $O/gemm_ab.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_model.py tests/test_gpu_step_oracle.py tests/test_gpu_training_loop.py tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/step_ab3.py > $O/step_ab3.log 2>&1 || exit $?
tail -1 $O/step_ab3.log
timeout -k 10 600 python bench.py --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || exit $?
tail -2 $O/bench.err
