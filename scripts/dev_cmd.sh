bash scripts/ab_libs.sh r2x "c4 c5" base sedge ga2 ga3 bw3 && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2x/pytest.log 2>&1
