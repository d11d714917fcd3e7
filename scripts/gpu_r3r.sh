# round 3: GPU tests at the adopted alpha leaves fix, then it (base) against Gamma / alphaTilde occupancy variants
set -o pipefail
T=${1:-r3r}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && \
bash scripts/ab_libs.sh $T/ab "c4 c5 c3" base ga2 ga1
