#!/bin/bash
# Round 4: persistence with radix sorts on dense value ranks + precomputed persistence ranking, W2 gradient rows
# from LDS-staged contributions: bit-exactness tests, phase timing, W2/PH kernel times in the step.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04h}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ph.py tests/test_gpu_topo_w2.py > $O/pytest_ph.log 2>&1 || { tail -30 $O/pytest_ph.log; exit 1; }
tail -1 $O/pytest_ph.log
timeout -k 10 60 ./scripts/micro/ph_timing_probe > $O/ph_timing.log 2>&1 || { tail -5 $O/ph_timing.log; exit 1; }
cat $O/ph_timing.log
if [ -x ./scripts/micro/uf_resolve_probe ]; then timeout -k 10 60 ./scripts/micro/uf_resolve_probe > $O/uf_resolve_probe.log 2>&1 || exit 1; cat $O/uf_resolve_probe.log; fi
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_losses.py tests/test_gpu_graph_step.py tests/test_gpu_pipeline.py > $O/pytest_b.log 2>&1 || { tail -30 $O/pytest_b.log; exit 1; }
tail -1 $O/pytest_b.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
grep -E "w2_|cubical|dicece" $O/kernel_stats_sequential.csv | cut -c1-60,200-
