#!/bin/bash
# Socket power and clocks while the headline inference kernel runs back to back (tools/infer_trajectory.py, one long
# trajectory), sampled with rocm-smi (read-only queries) before, during and after. Output: gpurun_out/power_probe.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/power_probe.log
: > "$OUT"
echo "== idle" >> "$OUT"; timeout 20 rocm-smi --showpower --showclocks >> "$OUT" 2>&1
timeout -k 10 120 python tools/infer_trajectory.py --chunks 400 --chunk 100 --frames 4 > gpurun_out/power_traj.log 2>&1 &
PID=$!
for i in $(seq 1 40); do
  sleep 0.5
  kill -0 $PID 2>/dev/null || break
  echo "== t=$i" >> "$OUT"; timeout 10 rocm-smi --showpower --showclocks >> "$OUT" 2>&1
done
wait $PID; rc=$?
echo "trajectory rc=$rc" >> "$OUT"
exit $rc
