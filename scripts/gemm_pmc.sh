#!/bin/bash
# PMC passes over one GEMM shape; outputs under gpurun_out/$TAG
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-gpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS=${ARGS:-"32768 3072 768"}
P="python3 $R/scripts/gemm_prof.py $ARGS"
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- $P > $O/kt.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/p1 -o p1 -- $P 5 > $O/p1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- $P 5 > $O/p2.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o p3 -- $P 5 > $O/p3.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p4 -o p4 -- $P 5 > $O/p4.log 2>&1 || exit $?
echo ok
