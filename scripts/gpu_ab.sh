#!/bin/bash
# One A/B iteration on the GPU box (outputs under gpurun_out/$TAG): the named GPU tests, attention launch
# times, GEMM variant times on $GEMM_SHAPES, then the default bench line (no CPU baseline / val).
# usage: TAG=x bash scripts/gpu_ab.sh tests/test_a.py ...
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-ab}
mkdir -p $O
cd $R
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/t.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 120 python scripts/attn_time.py > $O/attn_time.log 2>&1; rc=$?
echo "attn_time rc=$rc"; grep '^{' $O/attn_time.log
[ $rc -eq 0 ] || exit $rc
GEMM_SHAPES=${GEMM_SHAPES:-qkv_glob,fc1,fc2,proj} GEMM_VARIANTS=${GEMM_VARIANTS:-default,noepi} \
  timeout -k 10 240 python scripts/gemm_variants.py > $O/gemm_variants.log 2>&1; rc=$?
echo "gemm_variants rc=$rc"; grep '^{' $O/gemm_variants.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-baseline 0 --val 0 > $O/b.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $O/b.log | cut -c1-300
exit $rc
