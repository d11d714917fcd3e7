#!/bin/bash
# On the GPU box: run scripts/gpu_session.sh inside the frozen .snap/ tree and copy its output to the top-level
# gpurun_out/ (the directory gpurun returns).  The session's own exit status is returned.  While it runs, the last
# line of its session log is echoed every 30 s (the session's steps write only into .snap/gpurun_out/, and a run
# silent for 3 minutes is taken to be hung).
SNAP=$(cd "$(dirname "$0")/.." && pwd)
TOP=$(cd "$SNAP/.." && pwd)
TAG=${1:?tag}
cd "$SNAP"
bash scripts/gpu_session.sh "$@" &
PID=$!
while kill -0 $PID 2>/dev/null; do
  sleep 30
  kill -0 $PID 2>/dev/null && echo "[$(date +%T)] running: $(tail -1 gpurun_out/$TAG/session.log 2>/dev/null)"
done
wait $PID
rc=$?
mkdir -p "$TOP/gpurun_out/$TAG"
cp -r "gpurun_out/$TAG/." "$TOP/gpurun_out/$TAG/"
cp SNAP_HEAD "$TOP/gpurun_out/$TAG/" 2>/dev/null
for w in c4 c5 c3 c4s c4_shared c5_shared c3_shared; do
  [ -f "profiles/pmc_traffic_$w.json" ] && [ "profiles/pmc_traffic_$w.json" -nt SNAP_HEAD ] && \
    cp "profiles/pmc_traffic_$w.json" "$TOP/gpurun_out/$TAG/pmc_traffic_$w.json"
done
exit $rc
