#!/bin/bash
# rocprofv3 kernel stats + PMC passes for the bench workloads at the current tree, one workload after the other:
#   bash scripts/gpu_profile_all.sh <tag> ["c4 c5 c3"]
# A workload name with the suffix _shared (c4_shared) profiles bench.py --shared-order (NUSI_OPT_REFERENCE_ORDER = 0);
# the others run the library default, the reference order.  The summary records that order (--order), and bench.py
# uses profiles/pmc_traffic_<workload>[_shared].json only for the mode it times.
# Per workload: kernel trace + stats, FETCH_SIZE, WRITE_SIZE, fp64 VALU counts, MFMA busy (each pass its own run),
# the FETCH_SIZE calibration kernel, the summary (scripts/pmc_summary.py, with the library's sha256), and the
# bench line that carries it.  Every GPU step has its own time limit; the steps are chained with &&.
TAG=${1:-prof}
WLS=${2:-c4 c5 c3}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
# the matrix-core counters this box offers (an unknown name fails the pass)
MF=""
for c in SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES; do
  grep -qw "$c" $OUT/avail.txt && MF="$MF $c"
done
echo "mfma counters:$MF" > $OUT/mfma_counters.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_calib -o calib --output-format csv -- ./scripts/calib/pmc_calib > $OUT/pmc_calib.log 2>&1 || exit 1
for WL in $WLS; do
  W=${WL%_shared}
  if [ "$W" != "$WL" ]; then ORD=shared; OPT=--shared-order; else ORD=reference; OPT=; fi
  case $W in c3) ST=2;; c5) ST=3;; *) ST=5;; esac
  O=$OUT/$WL
  mkdir -p $O
  B="--workload $W $OPT --steps $ST --warmup 1 --no-cpu-baseline --no-secondary --no-parity"
  P="timeout -s KILL 420 rocprofv3 --kernel-trace --output-format csv"
  timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py $B > $O/kt.log 2>&1 && \
  $P --pmc FETCH_SIZE -d $O/pmc_fetch -o fetch -- python3 bench.py $B > $O/pmc_fetch.log 2>&1 && \
  $P --pmc WRITE_SIZE -d $O/pmc_write -o write -- python3 bench.py $B > $O/pmc_write.log 2>&1 && \
  $P --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -d $O/pmc_valu -o valu -- python3 bench.py $B > $O/pmc_valu.log 2>&1 && \
  { [ -z "$MF" ] || $P --pmc $MF -d $O/pmc_mfma -o mfma -- python3 bench.py $B > $O/pmc_mfma.log 2>&1; } && \
  python scripts/pmc_summary.py $O/pmc_fetch $O/pmc_write $OUT/pmc_calib $O/pmc_valu --mfma $O/pmc_mfma --lib nusiprop_amd/libnusi.so --order $ORD --steps $((ST + 1)) > $O/pmc_traffic_summary.json && \
  timeout -k 10 420 python bench.py $B --steps $((ST * 4)) --traffic-json $O/pmc_traffic_summary.json > $O/bench.json 2> $O/bench.err || exit 1
done
echo ok > $OUT/rc.txt
