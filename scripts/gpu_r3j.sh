# round 3: record prefetch in k_cascade_ws -- cascade tests, then A/B against the previous tree (h0) on C4/C5
set -o pipefail
T=${1:-r3j}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cascade or c5 or c1 or tables_bitexact or full_size or gamma or scan_subset" > gpurun_out/$T/pytest.log 2>&1 && \
bash scripts/ab_libs.sh $T/ab "c4 c5" base h0
