#!/bin/bash
# SQ counters of the table/cascade kernels (separate passes; --pmc with --kernel-trace only):
#   bash scripts/pmc_alpha.sh <tag> ["<runner command>"]   (default runner: the C4 scan, scripts/dev_scan_timing.py)
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
R="${2:-python3 scripts/dev_scan_timing.py 1024 300}"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/p1 -o p1 -- $R > $OUT/p1.log 2>&1 && \
$P --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH -d $OUT/p2 -o p2 -- $R > $OUT/p2.log 2>&1 && \
$P --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_IFETCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR -d $OUT/p3 -o p3 -- $R > $OUT/p3.log 2>&1 && \
$P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d $OUT/p4 -o p4 -- $R > $OUT/p4.log 2>&1
echo "rc=$?" > $OUT/rc.txt
