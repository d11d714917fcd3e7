# round 3: latency roles on a push-free SIMD -- cascade tests, A/B vs ns0 on C4/C5/C3, trace of the placement
set -o pipefail
T=${1:-r3m}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gamma_batch.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cascade or c5 or gamma" > gpurun_out/$T/pytest.log 2>&1 && \
bash scripts/ab_libs.sh $T/ab "c4 c5 c3" base ns0 && \
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c4 > gpurun_out/$T/trace_c4.log 2>&1
