#!/bin/bash
# Build an A/B variant of libnusi.so (timing experiments only):
#   scripts/build_variant.sh <name> [flags...]           current tree + extra compile flags
#   REV=<git rev> scripts/build_variant.sh <name> [...]  sources of a committed revision
# -> build/variants/libnusi_<name>.so ; select it with NUSIPROP_LIB=... scripts/dev_scan_timing.py
set -e
V=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=/tmp/nusi_var_$V
rm -rf $D; mkdir -p $D
SRC=${SRCDIR:-$ROOT}
if [ -n "$REV" ]; then
  SRC=$D/src; mkdir -p $SRC
  git -C $ROOT archive $REV include nusiprop_amd/csrc | tar -x -C $SRC
fi
C=$SRC/nusiprop_amd/csrc
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I$SRC/include -Wno-unused-value $*"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-spill-vgpr-to-agpr=0 -c -o $D/k.o $C/nusi_kernels.hip &
/opt/rocm/bin/hipcc $F -mllvm -pragma-unroll-threshold=1000000 -c -o $D/c.o $C/nusi_cascade.hip &
/opt/rocm/bin/hipcc $F -c -o $D/a.o $C/nusi_capi.cpp &
wait
mkdir -p $ROOT/build/variants
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $ROOT/build/variants/libnusi_$V.so $D/k.o $D/c.o $D/a.o
echo built build/variants/libnusi_$V.so
