# round 3: identity-permutation fast path in the solve -- cascade tests, A/B vs the previous tree (hd), then the
# default bench invocation (C4 + secondary C5 / C3 lines + CPU baseline)
set -o pipefail
T=${1:-r3n}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gamma_batch.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cascade or c5 or gamma or tables_bitexact" > gpurun_out/$T/pytest.log 2>&1 && \
bash scripts/ab_libs.sh $T/ab "c4 c5 c3" base hd && \
timeout -k 10 600 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err
