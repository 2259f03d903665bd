#!/bin/bash
# Round 5: fork_topo on by default: the step tests (graph, pipeline, oracle, DP) and a bench run.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05q}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py \
  tests/test_gpu_step_oracle.py tests/test_gpu_dp.py tests/test_gpu_fused_pp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python bench.py --cpu-baseline 0 --val 0 --val-protocol 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
