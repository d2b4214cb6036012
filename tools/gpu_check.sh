#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace. Stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then echo "pytest crashed/timed out (rc=$rc): stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log | tail; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --train-frames 5 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log"; exit 5; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_wide" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_wide.py" --queries 8388608 > "$GRAFT_REPO_ROOT/gpurun_out/prof_wide.log" 2>&1 || { echo "rocprof wide failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_wide.log"; exit 5; }
cd "$GRAFT_REPO_ROOT"
PMC_HBM_ONLY=1 bash tools/gpu_pmc.sh pmc_bench python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --train-frames 1 --no-cpu || exit 6
python tools/pmc_to_json.py gpurun_out/pmc_bench infer_kernel gpurun_out/pmc_infer.json > /dev/null || exit 7
echo "all done"
