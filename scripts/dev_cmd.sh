mkdir -p gpurun_out/r2z
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2z/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/r2z/bench_default.json 2> gpurun_out/r2z/bench_default.err
