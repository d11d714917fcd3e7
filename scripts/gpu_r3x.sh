# round 3 final tree (after the non-resonant step-pass instance): tests + smoke, rocprofv3 + PMC for c4 c5 c3 c4s, then the default bench invocation
set -o pipefail
T=${1:-r3x}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 && \
bash scripts/gpu_profile_all.sh $T/prof "c4 c5 c3 c4s" && \
for w in c4 c5 c3 c4s; do cp gpurun_out/$T/prof/$w/pmc_traffic_summary.json profiles/pmc_traffic_$w.json; done && \
timeout -k 10 600 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err
