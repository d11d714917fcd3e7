#!/bin/bash
# A/B timing of library variants nusiprop_amd/libnusi_<v>.so on the C4 scan (1024 points).
OUT=gpurun_out/${1:-ab}; shift
mkdir -p $OUT
for v in "$@"; do
  NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_$v.so timeout -k 10 300 python scripts/dev_scan_timing.py 1024 300 > $OUT/$v.log 2>&1 || { echo "variant $v failed rc=$?" >> $OUT/$v.log; exit 1; }
done
