#!/bin/bash
# Build an A/B variant of the engine library: voiceactivityprojection_amd/_lib/<name>.so with one
# kernel source recompiled under extra defines (load it with VAP_LIB_AB=<name>.so).
# Usage: tools/build_variant.sh <name> <source.hip> "<-DFOO=1 ...>"   (run after `make`)
set -e
NAME=$1; SRC=$2; DEFS=$3
cd "$(dirname "$0")/../voiceactivityprojection_amd/csrc"
EXTRA=""
case $SRC in k_attn.hip) EXTRA="-mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans -mno-amdgpu-ieee";; k_conv01.hip) EXTRA="-mllvm -amdgpu-mfma-vgpr-form";; esac
mkdir -p build/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $EXTRA $DEFS -c $SRC -o build/var/$NAME.o
OBJS=$(ls build/*.o | grep -v "build/${SRC%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build/var/$NAME.o -o ../_lib/$NAME.so
echo "built _lib/$NAME.so"
