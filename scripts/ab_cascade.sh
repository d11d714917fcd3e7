#!/bin/bash
# A/B of the cascade kernels on C4 and C5 (bench lines, no CPU baseline); GPU tests first.
TAG=${1:-r2b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 $B --workload c4 > $OUT/c4_ws.json 2> $OUT/c4_ws.err && \
NUSI_CASCADE_WS=0 timeout -k 10 300 $B --workload c4 > $OUT/c4_mfma.json 2> $OUT/c4_mfma.err && \
timeout -k 10 300 $B --workload c5 > $OUT/c5_mrhs.json 2> $OUT/c5_mrhs.err && \
NUSI_MRHS=0 timeout -k 10 300 $B --workload c5 > $OUT/c5_ws1.json 2> $OUT/c5_ws1.err && \
NUSI_MRHS=0 NUSI_CASCADE_WS=0 timeout -k 10 300 $B --workload c5 > $OUT/c5_mfma.json 2> $OUT/c5_mfma.err
rc=$?
echo "rc=$rc" > $OUT/rc.txt
exit $rc
