#!/bin/bash
# Full GPU suite (new: device W2, RCCL world 1, configs[3]/[4] step vs oracle, val-Dice on the 128/32 protocol from
# the oracle start point) and the default bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03d}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread tests/test_gpu_val_dice.py > $O/pytest_valdice.log 2>&1
rc=$?; tail -3 $O/pytest_valdice.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/ --deselect tests/test_gpu_val_dice.py::test_val_dice_parity > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
tail -2 $O/bench.err
