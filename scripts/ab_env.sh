#!/bin/bash
# A/B timing of environment settings on the C4 scan: bash scripts/ab_env.sh <tag> "<VAR=val ...>" ...
OUT=gpurun_out/$1; shift
mkdir -p $OUT
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python scripts/dev_scan_timing.py 1024 300 > $OUT/env$i.log 2>&1 || { echo "env $e failed" >> $OUT/env$i.log; exit 1; }
  echo "$e" >> $OUT/env$i.log
done
