#!/bin/bash
# One GPU session: smoke, default bench, rocprofv3 kernel stats, PMC traffic passes.
# Each GPU step has its own time limit; steps are chained with && so that a
# failure or timeout ends the session.  Outputs go to gpurun_out/<tag>/.
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/kt.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
rc=$?
echo "session rc=$rc" > $OUT/rc.txt
find $OUT -name "*.csv" | head -50 >> $OUT/rc.txt
exit $rc
