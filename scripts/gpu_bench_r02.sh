#!/bin/bash
# Round-2 measurement: headline bench (configs[2]), configs[4] slice (vit-h, both, fp16), rocprofv3 stats.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-bench}; mkdir -p $O; cd $R
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.err
timeout -k 10 400 python bench.py --model facebook/sam-vit-huge --prompt both --dtype fp16 --cpu-baseline 0 --val 0 --data-path 0 --e2e-steps 0 --topo-all 0 --steps 5 --warmup 2 > $O/bench_vith.json 2> $O/bench_vith.err || exit $?
tail -1 $O/bench_vith.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --cpu-baseline 0 --val 0 --data-path 0 --e2e-steps 0 --topo-all 0 > $O/prof.log 2>&1 || exit $?
echo prof ok
