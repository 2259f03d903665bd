#!/bin/bash
# Round 5: hipBLASLt for the encoder's in-place-residual GEMMs: GEMM + step tests, step A/B, bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05v}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $O/tests_gemm.log 2>&1 || { tail -30 $O/tests_gemm.log; exit 1; }
tail -1 $O/tests_gemm.log
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py \
  tests/test_gpu_model.py tests/test_gpu_step_oracle.py tests/test_gpu_dp.py > $O/tests_step.log 2>&1 || { tail -30 $O/tests_step.log; exit 1; }
tail -1 $O/tests_step.log
STEP_VARIANTS=default,blaslt_off timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab.log 2>&1 || { tail -5 $O/step_ab.log; exit 1; }
tail -1 $O/step_ab.log
STEP_PIPELINE=0 STEP_VARIANTS=default,blaslt_off timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab_seq.log 2>&1 || { tail -5 $O/step_ab_seq.log; exit 1; }
tail -1 $O/step_ab_seq.log
timeout -k 10 600 python bench.py --cpu-baseline 0 --val 0 --val-protocol 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 --top-off 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('sequential_ms_per_step')); r=d['roofline']; print(r['frac'], r['launches'], r['avg_launch_us'], r.get('library_gemm'))"
