# quick GPU iteration: selected -m gpu tests (pytest -k expression $2), then C4 and C3 bench lines
set -o pipefail
TAG=${1:-q}
K=${2:-cascade}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/$TAG/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench_c4.json 2> gpurun_out/$TAG/bench_c4.err && \
timeout -k 10 500 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.err
