#!/bin/bash
# One GPU session on the box (the only session driver; round-specific scripts are not kept):
#   gpurun -- bash scripts/gpu_session.sh <tag> <step> [<step> ...]
# Steps run in order, each under its own time limit, and the session stops at the first failing step
# (a GPU fault, abort, time limit or failed test ends it; nothing is retried).  Output: gpurun_out/<tag>/.
#   tests[=<k-expr>]        python -m pytest tests -m gpu [-k <k-expr>]            -> pytest.log
#   smoke                   __graft_entry__.smoke()                                 -> smoke.log
#   profile=<wl>[,<wl>..]   rocprofv3 kernel stats + PMC passes (scripts/gpu_profile_all.sh) -> prof/<wl>/;
#                           the summaries are copied to profiles/pmc_traffic_<wl>.json
#   bench[=<a>,<b>,..]      python bench.py <a> <b> ..  (commas = spaces)           -> bench_<i>.json / .err
#   prof=<a>,<b>,..         rocprofv3 --kernel-trace --stats of bench.py <a> <b> .. -> kt_<i>/
#   py=<script>,<a>,..      python <script> <a> ..                                   -> py_<i>.out / .err
#   vbench=<v>,<a>,..       bench.py <a> .. on the A/B library build/variants/libnusi_<v>.so (scripts/build_variant.sh)
#   vpy=<v>,<script>,<a>,.. python <script> <a> .. on that library                   -> vpy_<i>.out / .err
#   vprof=<v>,<a>,..        prof= of bench.py <a> .. on that library                  -> vkt_<i>_<v>/
#   vpmc=<v>,<workload>     SQ instruction / busy counters of bench.py on library v (base = libnusi.so) -> vpmc_<i>_<v>/
set -o pipefail
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for STEP in "$@"; do
  i=$((i + 1))
  NAME=${STEP%%=*}
  ARG=""
  [ "$NAME" != "$STEP" ] && ARG=${STEP#*=}
  ARGS=${ARG//,/ }
  echo "[$(date +%T)] step $i: $STEP" >> $OUT/session.log
  case $NAME in
    tests)
      K=()
      [ -n "$ARG" ] && K=(-k "$ARG")
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
        > $OUT/pytest.log 2>&1 || { echo "tests failed" >> $OUT/session.log; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1 ;;
    profile)
      bash scripts/gpu_profile_all.sh $TAG/prof "$ARGS" || exit 1
      for w in $ARGS; do cp $OUT/prof/$w/pmc_traffic_summary.json profiles/pmc_traffic_$w.json || exit 1; done ;;
    bench)
      timeout -k 10 900 python bench.py $ARGS > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 1 ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_$i -o kt --output-format csv -- python3 bench.py $ARGS \
        > $OUT/kt_$i.log 2>&1 || exit 1 ;;
    py)
      timeout -k 10 600 python $ARGS > $OUT/py_$i.out 2> $OUT/py_$i.err || exit 1 ;;
    vbench)
      V=${ARGS%% *}; A=${ARGS#* }; [ "$A" = "$ARGS" ] && A=""
      NUSIPROP_LIB=$PWD/build/variants/libnusi_$V.so timeout -k 10 600 python bench.py $A > $OUT/vbench_${i}_$V.json \
        2> $OUT/vbench_${i}_$V.err || exit 1 ;;
    vprof)
      V=${ARGS%% *}; A=${ARGS#* }; [ "$A" = "$ARGS" ] && A=""
      NUSIPROP_LIB=$PWD/build/variants/libnusi_$V.so timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/vkt_${i}_$V \
        -o kt --output-format csv -- python3 bench.py $A > $OUT/vkt_${i}_$V.log 2>&1 || exit 1 ;;
    vpmc)   # vpmc=<v>,<workload>: SQ instruction counters of the A/B library's kernels (v = base: libnusi.so)
      V=${ARGS%% *}; W=${ARGS#* }
      L=$PWD/build/variants/libnusi_$V.so; [ "$V" = base ] && L=$PWD/nusiprop_amd/libnusi.so
      NUSIPROP_LIB=$L timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/vpmc_${i}_$V \
        --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
        -o pmc -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-parity \
        > $OUT/vpmc_${i}_$V.log 2>&1 || exit 1 ;;
    vpy)
      V=${ARGS%% *}; A=${ARGS#* }
      NUSIPROP_LIB=$PWD/build/variants/libnusi_$V.so timeout -k 10 600 python $A > $OUT/vpy_${i}_$V.out \
        2> $OUT/vpy_${i}_$V.err || exit 1 ;;
    *)
      echo "unknown step $STEP" >> $OUT/session.log; exit 2 ;;
  esac
done
echo "[$(date +%T)] done" >> $OUT/session.log
