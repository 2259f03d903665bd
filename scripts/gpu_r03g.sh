#!/bin/bash
# PMC passes: global and windowed ViT attention (vit-b, B = 8), the decoder's largest k-major dW GEMM.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03g}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, command...
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n/kt -o kt -- "$@" > $O/$n.kt.log 2>&1 || return $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/$n/p1 -o p1 -- "$@" > $O/$n.p1.log 2>&1 || return $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/$n/p2 -o p2 -- "$@" > $O/$n.p2.log 2>&1 || return $?
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$n/p3 -o p3 -- "$@" > $O/$n.p3.log 2>&1 || return $?
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum --output-format csv -d $O/$n/p4 -o p4 -- "$@" > $O/$n.p4.log 2>&1 || return $?
  python3 $R/scripts/pmc_summary.py $O/$n > $O/$n.summary.txt
}
run attn_global python3 $R/scripts/attn_prof.py 64 8 12 64 5 || exit $?
run attn_window python3 $R/scripts/attn_prof.py 14 200 12 64 5 || exit $?
run dw python3 $R/scripts/dw_prof.py 5 || exit $?
cat $O/*.summary.txt
