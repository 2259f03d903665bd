#!/bin/bash
# Round 5: vit-h fp16 (configs[4] slice) with and without the token-side hipBLASLt kind, alternating processes on one box.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05cc}; mkdir -p $O; cd $R
F="--model facebook/sam-vit-huge --prompt both --dtype fp16 --cpu-baseline 0 --val 0 --val-protocol 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 --top-off 0 --roof-steps 0"
for rnd in 1 2; do
  for fp in 1 262145; do
    timeout -k 10 400 python bench.py $F --gemm-fast-path $fp > $O/b_${fp}_$rnd.json 2> $O/b_${fp}_$rnd.err || { tail -5 $O/b_${fp}_$rnd.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${fp}_$rnd.json').read().strip().splitlines()[-1]); print('fast_path=$fp round $rnd', d['value'], d['ms_per_step'], d.get('sequential_ms_per_step'))"
  done
done
