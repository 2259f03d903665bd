#!/bin/bash
# Round-3 snapshot on the GPU box (outputs under gpurun_out/$TAG): smoke, pytest -m gpu, bench (default flags),
# rocprofv3 kernel-trace/stats of the bench (pipelined) and of the sequential step, and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs on gfx950) over a short eager bench: the dominant GEMM family's HBM bytes
# per launch (traffic_gemm8.json, read by bench.py) and the per-kernel traffic table.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r03final}
mkdir -p $O
cd $R
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --cpu-baseline 0 --val 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/prof $O/kernel_stats_pipelined.csv --delete-trace || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
SHORT="--eager --steps 2 --warmup 1 --cpu-baseline 0 --val 0 --roof-steps 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc/fetch -o run -- python3 $R/bench.py $SHORT > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc/write -o run -- python3 $R/bench.py $SHORT > $O/pmc_write.log 2>&1 || exit 1
python3 $R/scripts/pmc_traffic.py $O/pmc gemm8_kernel $O/traffic_gemm8.json || exit 1
python3 $R/scripts/pmc_kernels.py $O/pmc $O/traffic_kernels.json > $O/traffic_kernels.txt || exit 1
rm -rf $O/pmc
echo done
