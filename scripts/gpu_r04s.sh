#!/bin/bash
# Round 4: LayerNorm forward / backward with two row groups in flight per wave: parity tests, kernel times, step A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04s}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_model.py tests/test_gpu_graph_step.py tests/test_gpu_vith.py > $O/pytest_s.log 2>&1 || { tail -30 $O/pytest_s.log; exit 1; }
tail -1 $O/pytest_s.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
grep -E "ln_fwd|ln_bwd" $O/kernel_stats_sequential.csv | cut -c1-50,150-
