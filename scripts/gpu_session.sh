set -o pipefail
mkdir -p gpurun_out/r1g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1g/pytest.log 2>&1 && \
bash scripts/gpu_bench_profile.sh r1g
