#!/bin/bash
# The val-Dice test file (chunked, 157 pairs) and the default bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-vdbench}; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_val_dice.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_valdice.log 2>&1 || { tail -30 $O/pytest_valdice.log; exit 1; }
tail -2 $O/pytest_valdice.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
