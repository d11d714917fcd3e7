#!/bin/bash
# GPU check of the tree: every -m gpu test, smoke, then C4 / C5 / C3 bench lines (no CPU baseline).
# Each GPU step has its own time limit and the steps are chained with &&: the first failure ends the session.
#   bash scripts/gpu_check.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=${2:-}
KA=()
[ -n "$K" ] && KA=(-k "$K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $OUT/bench_c4.json 2> $OUT/bench_c4.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err && \
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err
rc=$?
echo "rc=$rc" > $OUT/rc.txt
exit $rc
