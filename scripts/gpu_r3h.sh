# round 3: the cascade tests + C3 line at the tree, then the profile session (rocprofv3 + PMC, c4 c5 c3)
set -o pipefail
T=${1:-r3h}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 && \
bash scripts/gpu_profile_all.sh $T/prof "c4 c5 c3"
