# round 3: k_cascade_wsp with the non-resonant flag a compile-time constant (timing variant nr) against the tree
set -o pipefail
T=${1:-r3w}
mkdir -p gpurun_out/$T
bash scripts/ab_libs.sh $T/ab "c3" base nr
