# round 3: shift-reuse tests + the c4s and c4 lines
set -o pipefail
T=${1:-r3i}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_shift_reuse.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c4s --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$T/bench_c4s.json 2> gpurun_out/$T/bench_c4s.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$T/bench_c4.json 2> gpurun_out/$T/bench_c4.err && \
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c4 > gpurun_out/$T/trace_c4.log 2>&1 && \
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c5 > gpurun_out/$T/trace_c5.log 2>&1
