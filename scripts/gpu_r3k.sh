# round 3: gamma-batch cascade tests + C5 lines with the gamma batch vs pairs
set -o pipefail
T=${1:-r3k}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gamma_batch.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline --rhs 16 > gpurun_out/$T/bench_c5_gb.json 2> gpurun_out/$T/bench_c5_gb.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline --rhs 2 > gpurun_out/$T/bench_c5_r2.json 2> gpurun_out/$T/bench_c5_r2.err
