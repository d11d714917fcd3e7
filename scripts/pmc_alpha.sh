#!/bin/bash
# SQ counters for the table/cascade kernels (separate passes; --pmc with --kernel-trace only).
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d $OUT/p1 -o p1 --output-format csv -- python3 scripts/dev_scan_timing.py 256 300 > $OUT/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH --kernel-trace -d $OUT/p2 -o p2 --output-format csv -- python3 scripts/dev_scan_timing.py 256 300 > $OUT/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_IFETCH --kernel-trace -d $OUT/p3 -o p3 --output-format csv -- python3 scripts/dev_scan_timing.py 256 300 > $OUT/p3.log 2>&1
echo "rc=$?" > $OUT/rc.txt
