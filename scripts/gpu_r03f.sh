#!/bin/bash
# Same-box two-build A/B of gemm.hip (round-2 source vs the uniform-wave epilogue fix), step A/B (device W2 forked
# beside the DiceCE backward vs host W2), the step / W2 / loop tests, bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03f}; mkdir -p $O; cd $R
for rnd in 1 2; do
  for lib in default dilabhelmholtzoct_amd/csrc/build/ab/liboctsam_old.so; do
    if [ $lib = default ]; then unset OCTSAM_LIB; else export OCTSAM_LIB=$R/$lib; fi
    timeout -k 10 200 python scripts/gemm_lib_ab.py >> $O/gemm_lib_ab.log 2>&1 || exit $?
  done
done
unset OCTSAM_LIB
grep lib $O/gemm_lib_ab.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_topo_w2.py tests/test_gpu_losses.py tests/test_gpu_training_loop.py tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py tests/test_gpu_dp.py tests/test_gpu_rccl.py tests/test_gpu_gemm.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/step_ab3.py > $O/step_ab3.log 2>&1 || exit $?
tail -1 $O/step_ab3.log
timeout -k 10 600 python bench.py --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || exit $?
tail -2 $O/bench.err
