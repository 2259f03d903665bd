#!/bin/bash
# Round 4: the bench's new legs (val-Dice protocol beside the committed oracle values, configs[1] top-off), then
# the sequential rocprofv3 kernel stats at HEAD.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04g}; mkdir -p $O; cd $R
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/bench_legs.json 2> $O/bench_legs.err || { tail -20 $O/bench_legs.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_legs.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step']); print(json.dumps(d['val_dice_protocol'])); print(json.dumps(d['top_off']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
head -40 $O/kernel_stats_sequential.csv | cut -c1-160
