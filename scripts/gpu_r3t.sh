# round 3: scheduler-option variants of the whole library against the tree (base)
set -o pipefail
T=${1:-r3t}
mkdir -p gpurun_out/$T
bash scripts/ab_libs.sh $T/ab "c4 c5 c3" base ilp memcl trk
