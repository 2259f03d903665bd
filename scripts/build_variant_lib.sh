#!/bin/bash
# Build ab_libs/NAME.so: the current objects with FILE (a csrc/*.hip) recompiled with extra FLAGS -- the other arm of a
# same-box two-build A/B (OCTSAM_LIB selects it). Run after `make`.
# usage: bash scripts/build_variant_lib.sh decoder_attn.hip "-DDEC_TR_ASM=0" liboctsam_dec_builtin
set -eu
F=$1; FLAGS=$2; NAME=$3
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R/dilabhelmholtzoct_amd/csrc
mkdir -p build/ab $R/ab_libs
EXTRA=""
[ $F = vit_attention.hip ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form=1 -fno-honor-nans -mno-amdgpu-ieee"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $EXTRA $FLAGS -c $F -o build/ab/variant.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/ab_libs/$NAME.so build/ab/variant.o $(ls build/*.o | grep -v "build/${F}.o")
ls -la $R/ab_libs/$NAME.so
