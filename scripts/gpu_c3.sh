# C3 check: phi-phi parity tests, then the C3 bench line (N_E=1200, phi-phi on, reference table geometry)
set -o pipefail
TAG=${1:-c3}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_phiphi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 && \
timeout -k 10 500 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.err
