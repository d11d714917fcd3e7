#!/bin/bash
# Build an A/B variant of libnusi.so with extra compile flags:
#   scripts/build_variant.sh <name> [flags...]  ->  nusiprop_amd/libnusi_<name>.so
# (timing experiments only; select it with NUSIPROP_LIB=... scripts/dev_scan_timing.py)
set -e
V=$1; shift
D=/tmp/nusi_var_$V
mkdir -p $D
C=nusiprop_amd/csrc
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Iinclude -Wno-unused-value $*"
/opt/rocm/bin/hipcc $F -c -o $D/k.o $C/nusi_kernels.hip &
/opt/rocm/bin/hipcc $F -mllvm -pragma-unroll-threshold=1000000 -c -o $D/c.o $C/nusi_cascade.hip &
/opt/rocm/bin/hipcc $F -c -o $D/a.o $C/nusi_capi.cpp &
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o nusiprop_amd/libnusi_$V.so $D/k.o $D/c.o $D/a.o
echo built nusiprop_amd/libnusi_$V.so
