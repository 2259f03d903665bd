#!/bin/bash
# Round 5: the multi-seed val-Dice test (oracle-made warm start), then the default bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05c}; mkdir -p $O; cd $R
OCTSAM_VALDICE_HIP_OUT=$O/valdice_hip.json timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_val_dice.py > $O/pytest_valdice.log 2>&1 || { grep -E "^pair|mean over|FAIL|Error|assert" $O/pytest_valdice.log | tail -30; exit 1; }
grep -E "^pair|mean over|passed|failed" $O/pytest_valdice.log
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
