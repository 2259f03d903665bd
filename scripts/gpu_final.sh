#!/bin/bash
# Round-end snapshot on the GPU box (outputs under gpurun_out/$TAG; smoke + pytest -m gpu run separately by
# scripts/gpu_tests_final.sh): the two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs on gfx950) over a short eager
# bench -> the GEMM family's HBM bytes per launch (traffic_gemm_family.json: gemm8 + gemm8p + gemm4w, the launch set of
# roofline.compulsory_bytes_per_launch; copied into profiles/ on the box so the bench below reads it) and the
# per-kernel traffic table; then the bench (default flags) and rocprofv3 kernel-trace/stats of the bench (pipelined)
# and of the sequential step.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SHORT="--eager --steps 2 --warmup 1 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --roof-steps 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc/fetch -o run -- python3 $R/bench.py $SHORT > $O/pmc_fetch.log 2>&1 || exit 1
echo "pmc fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc/write -o run -- python3 $R/bench.py $SHORT > $O/pmc_write.log 2>&1 || exit 1
echo "pmc write ok"
python3 $R/scripts/pmc_traffic.py $O/pmc gemm8w_kernel,gemm8_kernel,gemm8p_kernel,gemm4w_kernel $O/traffic_gemm_family.json || exit 1
cp $O/traffic_gemm_family.json $R/profiles/traffic_gemm_family.json
python3 $R/scripts/pmc_kernels.py $O/pmc $O/traffic_kernels.json > $O/traffic_kernels.txt || exit 1
rm -rf $O/pmc
cd $R
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/prof $O/kernel_stats_pipelined.csv --delete-trace || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
echo done
