# round 3: Gamma and alphaTilde as two kernels (gsplit) against the one-kernel tree (base)
set -o pipefail
T=${1:-r3s}
mkdir -p gpurun_out/$T
bash scripts/ab_libs.sh $T/ab "c4 c5 c3" base gsplit
