# round 3, the alpha point loop on wave-owned rows: GPU tests, then A/B against the r3o library (libnusi_r3o.so)
set -o pipefail
T=${1:-r3p}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && \
bash scripts/ab_libs.sh $T/ab "c4 c5 c3" base r3o
