# round 3: k_alpha_batch two points per barrier pair (512-thread workgroups): GPU tests, then A/B against HEAD
set -o pipefail
T=${1:-r3u}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && \
bash scripts/ab_libs.sh $T/ab "c4 c5 c3" base head
