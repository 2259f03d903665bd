#!/bin/bash
# Diagnostic probes on the GPU box (outputs under gpurun_out/$TAG): attention launch times, GEMM variants
# (default / no epilogue / no main loop / hipBLASLt) on the encoder shapes, and the windowed attention PMC passes.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-probe}
mkdir -p $O
cd $R
timeout -k 10 120 python scripts/attn_time.py > $O/attn_time.log 2>&1; rc=$?
echo "attn_time rc=$rc"; cat $O/attn_time.log
[ $rc -eq 0 ] || exit $rc
GEMM_SHAPES=${GEMM_SHAPES:-qkv_glob,fc1,fc2,proj} GEMM_VARIANTS=${GEMM_VARIANTS:-default,noepi,noloop,blaslt} \
  timeout -k 10 240 python scripts/gemm_variants.py > $O/gemm_variants.log 2>&1; rc=$?
echo "gemm_variants rc=$rc"; cat $O/gemm_variants.log
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-probe}/wpmc bash scripts/attn_pmc.sh; rc=$?
echo "attn_pmc rc=$rc"
exit $rc
