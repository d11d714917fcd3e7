set -o pipefail
TAG=${1:-r1n}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 && \
bash scripts/gpu_bench_profile.sh $TAG && \
timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/$TAG/bench_c5.json 2> gpurun_out/$TAG/bench_c5.err
