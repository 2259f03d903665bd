#!/bin/bash
# Round 4: lean GEMM epilogue kind 27 (e16 C + broadcast fp32 residual): parity tests, kernel time in the step.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04q}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_model.py tests/test_gpu_graph_step.py > $O/pytest_q.log 2>&1 || { tail -30 $O/pytest_q.log; exit 1; }
tail -1 $O/pytest_q.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
grep -E "gemm8_kernel<0, 0, (0|27)>" $O/kernel_stats_sequential.csv | cut -c1-60,150-
grep -E '"value"' $O/profseq.log | cut -c1-200 || true
