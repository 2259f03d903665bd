#!/bin/bash
# Round 5: kernel trace of the pipelined step (default bench flags, short) -> timeline occupancy (scripts/timeline.py).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05j}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 --roof-steps 0 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 $R/scripts/timeline.py $O/kt 60 > $O/timeline.txt && cat $O/timeline.txt
python3 $R/scripts/timeline.py $O/kt 160 > $O/timeline160.txt && head -8 $O/timeline160.txt
rm -rf $O/kt
