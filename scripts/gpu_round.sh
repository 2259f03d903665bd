#!/bin/bash
# Round snapshot on the GPU box (outputs under gpurun_out/$TAG): smoke, pytest -m gpu, bench (default flags),
# rocprofv3 kernel-trace/stats of the bench, and two PMC passes (FETCH_SIZE, WRITE_SIZE; they cannot share a
# pass on gfx950) over a short eager bench for the dominant kernel's HBM traffic per launch.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-round}
mkdir -p $O
cd $R
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json | cut -c1-400
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --cpu-baseline 0 --val 0 > $O/prof.log 2>&1; rc=$?
echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
SHORT="--eager --steps 2 --warmup 1 --cpu-baseline 0 --val 0 --roof-steps 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc/fetch -o run -- python3 $R/bench.py $SHORT > $O/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc/write -o run -- python3 $R/bench.py $SHORT > $O/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 $R/scripts/pmc_traffic.py $O/pmc gemm8_kernel $O/traffic_gemm8.json
