#!/bin/bash
# hipBLASLt's kernel choice on the encoder GEMM shapes (Tensile names encode macro tile / wave tiling / MFMA).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03u}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/blt -o run -- python3 $R/scripts/blaslt_probe.py > $O/blt.log 2>&1 || { tail -5 $O/blt.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/blt $O/blaslt_kernels.csv --delete-trace || exit 1
cut -c1-400 $O/blaslt_kernels.csv
