#!/bin/bash
# Round-end GPU session (one box): full GPU tests, smoke, bench, rocprofv3 kernel-trace stats of the bench and of the
# width-128 bench, PMC passes (tools/gpu_pmc.sh) on the bench. Stops at the first failure. Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest failed (rc=$rc): stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --train-frames 5 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log"; exit 5; }
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_pmc.sh pmc_bench python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --train-frames 2 --no-cpu || exit 6
python tools/pmc_to_json.py gpurun_out/pmc_bench infer_kernel gpurun_out/pmc_infer.json > /dev/null || exit 7
python tools/pmc_summary.py gpurun_out/pmc_bench > gpurun_out/pmc_bench_summary.txt || exit 8
echo "all done"
