# round 3: GPU tests + smoke + C4/C5/C3 lines at the tree, then the A/B of library variants on C4/C5
set -o pipefail
T=${1:-r3f}
bash scripts/gpu_check.sh $T && bash scripts/ab_libs.sh $T/ab "c4 c5" base p2top
