#!/bin/bash
# One GPU session: smoke, rocprofv3 kernel stats, PMC traffic passes (+ FETCH_SIZE
# calibration), then the bench line carrying the measured traffic.  Each GPU step
# has its own time limit; steps are chained with && so that a failure or timeout
# ends the session.  Outputs go to gpurun_out/<tag>/.
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BARGS="--steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $BARGS > $OUT/kt.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o fetch --output-format csv -- python3 bench.py $BARGS > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o write --output-format csv -- python3 bench.py $BARGS > $OUT/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_calib -o calib --output-format csv -- ./scripts/calib/pmc_calib > $OUT/pmc_calib.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace -d $OUT/pmc_valu -o valu --output-format csv -- python3 bench.py $BARGS > $OUT/pmc_valu.log 2>&1 && \
python scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_calib $OUT/pmc_valu --lib nusiprop_amd/libnusi.so > $OUT/pmc_traffic_summary.json && \
timeout -k 10 600 python bench.py --traffic-json $OUT/pmc_traffic_summary.json > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "session rc=$rc" > $OUT/rc.txt
exit $rc
