# cascade iteration on the GPU: cascade-related -m gpu tests, stage stamps (trace build), A/B lines, C3 bench
set -o pipefail
T=${1:-r3c}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "cascade or c5 or c1 or tables_bitexact or drop_in or full_size or batch or gamma" > gpurun_out/$T/pytest.log 2>&1 && \
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c4 > gpurun_out/$T/trace_c4.log 2>&1 && \
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c5 > gpurun_out/$T/trace_c5.log 2>&1 && \
timeout -k 10 300 python scripts/dev_ab_opts.py c4 "default:;wf:CASCADE=WAVEFRONT" 5 > gpurun_out/$T/ab_c4.log 2>&1 && \
timeout -k 10 300 python scripts/dev_ab_opts.py c5 "default:;rhs1:CASCADE_RHS=1" 5 > gpurun_out/$T/ab_c5.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$T/bench_c3.json 2> gpurun_out/$T/bench_c3.err
