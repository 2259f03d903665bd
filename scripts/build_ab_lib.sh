#!/bin/bash
# Build dilabhelmholtzoct_amd/csrc/build/ab/liboctsam_old.so: the current objects with FILE (a csrc/*.hip) taken
# from git HEAD instead — the "before" arm of a same-box two-build A/B (OCTSAM_LIB). Run after `make`.
# usage: bash scripts/build_ab_lib.sh upmask.hip
set -eu
F=$1
cd "$(dirname "$0")/../dilabhelmholtzoct_amd/csrc"
mkdir -p build/ab build/include
git show HEAD:dilabhelmholtzoct_amd/csrc/$F > build/ab/old_$F
cp common.h build/ab/ && cp ../../include/octsam.h build/include/
sed -i 's#"../../include/octsam.h"#"../include/octsam.h"#' build/ab/old_$F
EXTRA=""
[ $F = vit_attention.hip ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form=1 -fno-honor-nans -mno-amdgpu-ieee"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $EXTRA -c build/ab/old_$F -o build/ab/old.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab/liboctsam_old.so build/ab/old.o $(ls build/*.o | grep -v "build/${F}.o")
ls -la build/ab/liboctsam_old.so
