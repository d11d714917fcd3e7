# the per-config bench lines: C2 (single propagation), C1 (test.cpp, with its CPU lines), C5 (8192-point block)
set -o pipefail
TAG=${1:-lines}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.err && \
timeout -k 10 400 python bench.py --workload c1 --steps 20 --warmup 3 --cpu-seconds 20 > gpurun_out/$TAG/bench_c1.json 2> gpurun_out/$TAG/bench_c1.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench_c5.json 2> gpurun_out/$TAG/bench_c5.err
