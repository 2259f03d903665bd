#!/bin/bash
# PMC passes over the windowed attention kernel (vit-b, B=8 shapes); outputs under gpurun_out/$TAG
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-pmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS=${ARGS:-"14 200 12 64"}
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/scripts/attn_prof.py $ARGS > $O/kt.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/p1 -o p1 -- python3 $R/scripts/attn_prof.py $ARGS 5 > $O/p1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- python3 $R/scripts/attn_prof.py $ARGS 5 > $O/p2.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o p3 -- python3 $R/scripts/attn_prof.py $ARGS 5 > $O/p3.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INST_CYCLES_VMEM GRBM_COUNT GRBM_GUI_ACTIVE --output-format csv -d $O/p4 -o p4 -- python3 $R/scripts/attn_prof.py $ARGS 5 > $O/p4.log 2>&1 || exit $?
echo ok
