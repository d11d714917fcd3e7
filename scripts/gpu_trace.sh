# stage stamps and wave placement of k_cascade_ws (diagnostic build libnusi_trace.so: bash scripts/build_variant.sh trace -DNUSI_WS_TRACE)
set -o pipefail
mkdir -p gpurun_out/r3d
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c4 > gpurun_out/r3d/trace_c4.log 2>&1 && \
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c5 > gpurun_out/r3d/trace_c5.log 2>&1
