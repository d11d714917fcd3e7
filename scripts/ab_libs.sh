#!/bin/bash
# A/B of library variants on bench workloads: bash scripts/ab_libs.sh <tag> "<workloads>" <variant>...
# (variant "base" = nusiprop_amd/libnusi.so, else build/variants/libnusi_<v>.so from scripts/build_variant.sh)
OUT=gpurun_out/$1; shift
WL=$1; shift
mkdir -p $OUT
for v in "$@"; do
  L=$PWD/build/variants/libnusi_$v.so
  [ "$v" = base ] && L=$PWD/nusiprop_amd/libnusi.so
  for w in $WL; do
    NUSIPROP_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --no-parity --workload $w > $OUT/${w}_$v.json 2> $OUT/${w}_$v.err || exit 1
  done
done
