# round 3: alpha variants A/B (wave-owned rows at 4 / 3 waves per SIMD, the by-value leaves fix alone at 4 / 3)
set -o pipefail
T=${1:-r3q}
mkdir -p gpurun_out/$T
bash scripts/ab_libs.sh $T/ab "c4 c5" base w3 bpre bprew3 r3o
