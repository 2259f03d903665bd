#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04l}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused_pp.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
cd $R
STEP_VARIANTS=default,pp_unfused timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab.log 2>&1 || { tail -10 $O/step_ab.log; exit 1; }
tail -1 $O/step_ab.log
