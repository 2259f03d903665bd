#!/bin/bash
# HBM traffic of the dominant GEMM family (octsam_gemm path 2: gemm8, gemm8p, gemm4w) per launch for one bench workload: two PMC passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950) over a short eager bench, then scripts/pmc_traffic.py.
# Env: TAG (output dir under gpurun_out/), EXTRA (bench flags selecting the workload), OUT (json name).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-traffic}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SHORT="--eager --steps 2 --warmup 1 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --loop-images 0 --roof-steps 0 --data-path 0 --e2e-steps 0 --topo-all 0 ${EXTRA:-}"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc/fetch -o run -- python3 $R/bench.py $SHORT > $O/pmc_fetch.log 2>&1 || exit $?
echo "pmc fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc/write -o run -- python3 $R/bench.py $SHORT > $O/pmc_write.log 2>&1 || exit $?
echo "pmc write ok"
python3 $R/scripts/pmc_traffic.py $O/pmc gemm8_kernel,gemm8p_kernel,gemm4w_kernel $O/${OUT:-traffic_gemm_family.json}
