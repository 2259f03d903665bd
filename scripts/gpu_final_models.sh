#!/bin/bash
# Round end: the per-GPU slices of BASELINE configs[4] (vit-h, both prompts, fp16 encoder) and configs[3] (vit-l,
# points, B = 4) through bench.py (headline loop only).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-final_models}; mkdir -p $O; cd $R
F="--cpu-baseline 0 --val 0 --val-protocol 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 --top-off 0"
timeout -k 10 500 python bench.py --model facebook/sam-vit-huge --prompt both --dtype fp16 $F > $O/bench_vith.json 2> $O/bench_vith.err || { tail -5 $O/bench_vith.err; exit 1; }
cut -c1-200 $O/bench_vith.json
timeout -k 10 500 python bench.py --model facebook/sam-vit-large --prompt points --batch 4 $F > $O/bench_vitl.json 2> $O/bench_vitl.err || { tail -5 $O/bench_vitl.err; exit 1; }
cut -c1-200 $O/bench_vitl.json
