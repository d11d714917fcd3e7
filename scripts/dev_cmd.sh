mkdir -p gpurun_out/r2final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2final/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2final/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/r2final/bench.json 2> gpurun_out/r2final/bench.err
