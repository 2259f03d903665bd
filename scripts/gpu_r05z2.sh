#!/bin/bash
# Round 5: QKV on hipBLASLt by default: GEMM tests, step tests, vit-l with / without the QKV kind.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05z2}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $O/tests_gemm.log 2>&1; tail -12 $O/tests_gemm.log | grep -E "passed|failed|FAILED"
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py \
  tests/test_gpu_model.py tests/test_gpu_step_oracle.py tests/test_gpu_dp.py tests/test_gpu_layers.py > $O/tests_step.log 2>&1 || { tail -30 $O/tests_step.log; exit 1; }
tail -1 $O/tests_step.log
F="--model facebook/sam-vit-large --prompt points --batch 4 --cpu-baseline 0 --val 0 --val-protocol 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 --top-off 0 --roof-steps 0"
for rnd in 1 2; do
  for fp in 1 131073; do
    timeout -k 10 400 python bench.py $F --gemm-fast-path $fp > $O/l_${fp}_$rnd.json 2> $O/l_${fp}_$rnd.err || { tail -5 $O/l_${fp}_$rnd.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/l_${fp}_$rnd.json').read().strip().splitlines()[-1]); print('vit-l fast_path=$fp round $rnd', d['value'], d['ms_per_step'], d.get('sequential_ms_per_step'))"
  done
done
