#!/bin/bash
# Round 4: post-processing adjoint column pass with 4 rows per workgroup (bit-identical): tests incl. the val-Dice
# protocol (its warm-state fingerprint must equal the golden's), kernel time.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04v}; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_losses.py tests/test_gpu_fused_pp.py tests/test_gpu_graph_step.py tests/test_gpu_val_dice.py > $O/pytest_v.log 2>&1 || { grep -E "^after|fingerprint|FAIL|Error" $O/pytest_v.log | tail -20; exit 1; }
grep -E "^after|fingerprint" $O/pytest_v.log; tail -1 $O/pytest_v.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
grep -E "pp_bwd_cols|dicece_pp_rows" $O/kernel_stats_sequential.csv | cut -c1-50,100-
