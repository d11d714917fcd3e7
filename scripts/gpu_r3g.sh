# round 3: stage-latency floor microbenchmark, then cascade A/B of library variants on C4/C5/C3
set -o pipefail
T=${1:-r3g}
mkdir -p gpurun_out/$T
timeout -k 10 120 ./scripts/dev/stage_floor > gpurun_out/$T/stage_floor.log 2>&1 && \
bash scripts/ab_libs.sh $T/ab "c3 c4 c5" base r492
