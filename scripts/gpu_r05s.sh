#!/bin/bash
# Round 5: where the step's small launches come from: kernel trace of a sequential graph-mode bench, neighbours of
# copyBuffer / axpby / splitk_reduce / elementwise launches.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05s}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --pipeline 0 --steps 4 --warmup 2 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 --roof-steps 0 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
for pat in copyBuffer axpby splitk_reduce elementwise cast16x8 fillBuffer; do
  echo "== $pat"; python3 $R/scripts/trace_neighbors.py $O/trace $pat 17 || exit 1
done > $O/neighbors.txt
cat $O/neighbors.txt | cut -c1-230
rm -rf $O/trace
