#!/bin/bash
# Per-kernel HBM traffic of the whole training step (two PMC passes over a short eager bench: FETCH_SIZE, WRITE_SIZE)
# -> scripts/pmc_kernels.py table; GEMM yardstick: default / no-epilogue / no-main-loop builds and torch.matmul
# (hipBLASLt) on the encoder shapes.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03r}; mkdir -p $O
cd $R
GEMM_SHAPES=qkv_glob,proj,fc1,fc2 GEMM_VARIANTS=default,noepi,noloop,blaslt timeout -k 10 200 python -u scripts/gemm_variants.py > $O/gemm_yard.log 2>&1 || { tail -20 $O/gemm_yard.log; exit 1; }
cat $O/gemm_yard.log
cd /tmp && export TMPDIR=/tmp
SHORT="--eager --steps 2 --warmup 1 --cpu-baseline 0 --val 0 --roof-steps 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc/fetch -o run -- python3 $R/bench.py $SHORT > $O/pmc_fetch.log 2>&1 || exit $?
echo "pmc fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc/write -o run -- python3 $R/bench.py $SHORT > $O/pmc_write.log 2>&1 || exit $?
echo "pmc write ok"
python3 $R/scripts/pmc_kernels.py $O/pmc $O/traffic_kernels.json > $O/traffic_kernels.txt || exit 1
head -30 $O/traffic_kernels.txt
rm -rf $O/pmc
