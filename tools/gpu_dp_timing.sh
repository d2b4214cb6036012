#!/bin/bash
# DP step timing on one GPU shared by 2 ranks (tools/dp_step_timing.py): a plain run, then each rank under its own
# rocprofv3 kernel trace (no launcher between the profiler and python) for the exchange kernels' durations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29617 tools/dp_step_timing.py --steps 300 > gpurun_out/dp_timing.log 2>&1 || { echo "plain run failed"; tail -20 gpurun_out/dp_timing.log; exit 3; }
tail -1 gpurun_out/dp_timing.log
pids=()
for r in 0 1; do
  (cd /tmp && RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29618 timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/dp_prof_$r" -o run --output-format csv -- \
    python3 "$ROOT/tools/dp_step_timing.py" --steps 100 > "$ROOT/gpurun_out/dp_prof_$r.log" 2>&1) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "profiled rc=$rc"
exit $rc
