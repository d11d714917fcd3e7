bash scripts/ab_libs.sh r2q "c4 c5 c3" nostg stg qc5 && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2q/pytest.log 2>&1
