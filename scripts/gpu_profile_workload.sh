#!/bin/bash
# rocprofv3 kernel stats + PMC traffic passes (FETCH_SIZE calibrated, WRITE_SIZE) for one bench workload,
# then its bench line carrying the measured traffic: bash scripts/gpu_profile_workload.sh <tag> <workload> [steps]
TAG=${1:-wl}; WL=${2:-c3}; ST=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BARGS="--workload $WL --steps $ST --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $BARGS > $OUT/kt.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o fetch --output-format csv -- python3 bench.py $BARGS > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o write --output-format csv -- python3 bench.py $BARGS > $OUT/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_calib -o calib --output-format csv -- ./scripts/calib/pmc_calib > $OUT/pmc_calib.log 2>&1 && \
python scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_calib --lib nusiprop_amd/libnusi.so > $OUT/pmc_traffic_summary.json && \
timeout -k 10 600 python bench.py $BARGS --traffic-json $OUT/pmc_traffic_summary.json > $OUT/bench.json 2> $OUT/bench.err
