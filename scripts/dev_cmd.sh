bash scripts/ab_libs.sh r2w "c4 c3" head noesc && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2w/pytest.log 2>&1
