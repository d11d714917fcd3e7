set -o pipefail
mkdir -p gpurun_out/r3b
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c4 > gpurun_out/r3b/trace_c4.log 2>&1 && \
NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_trace.so timeout -k 10 120 python scripts/dev_ws_trace.py c5 > gpurun_out/r3b/trace_c5.log 2>&1 && \
bash scripts/pmc_alpha.sh r3b/pmc_wave "python3 scripts/dev_ab_opts.py c4 wave:ALPHA_KERNEL=0 3" && \
bash scripts/pmc_alpha.sh r3b/pmc_batch "python3 scripts/dev_ab_opts.py c4 batch:ALPHA_KERNEL=3 3"
