#!/bin/bash
# Round 5: bench (headline loop only) with fork_topo on / off, alternating processes on one box.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05r}; mkdir -p $O; cd $R
F="--cpu-baseline 0 --val 0 --val-protocol 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 --top-off 0 --roof-steps 0 --steps 20"
for rnd in 1 2 3; do
  for fk in 1 0; do
    timeout -k 10 300 python bench.py $F --fork-topo $fk > $O/b_${fk}_$rnd.json 2> $O/b_${fk}_$rnd.err || { tail -5 $O/b_${fk}_$rnd.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/b_${fk}_$rnd.json').read().strip().splitlines()[-1]); print('fork_topo=$fk round $rnd', d['value'], d['ms_per_step'], d.get('sequential_ms_per_step'))"
  done
done
