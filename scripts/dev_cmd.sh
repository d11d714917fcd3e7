mkdir -p gpurun_out/r2u
timeout -k 10 400 python -u -m pytest tests/test_phiphi.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "phiphi or kernels_names or c3" > gpurun_out/r2u/pytest.log 2>&1 && \
NUSI_SPLINE_WINDOWS=0 timeout -k 10 400 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2u/c3_nowin.json 2>gpurun_out/r2u/c3_nowin.err && \
timeout -k 10 400 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2u/c3_win.json 2>gpurun_out/r2u/c3_win.err
