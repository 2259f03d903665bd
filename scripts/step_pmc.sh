#!/bin/bash
# Issue profile of every kernel of the eager step (SQ counter passes over a short eager bench, one pass per run as
# gfx950 requires), summarised per kernel by scripts/pmc_issue.py; outputs under gpurun_out/$TAG.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-step_pmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SHORT="--eager --steps 2 --warmup 1 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --roof-steps 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/pmc/p1 -o run -- python3 $R/bench.py $SHORT > $O/p1.log 2>&1 || exit 1
echo "pass 1 ok"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/pmc/p2 -o run -- python3 $R/bench.py $SHORT > $O/p2.log 2>&1 || exit 1
echo "pass 2 ok"
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc/p3 -o run -- python3 $R/bench.py $SHORT > $O/p3.log 2>&1 || exit 1
echo "pass 3 ok"
python3 $R/scripts/pmc_issue.py $O/pmc $O/issue.json 20 > $O/issue.txt || exit 1
rm -rf $O/pmc
head -40 $O/issue.txt | cut -c1-400
