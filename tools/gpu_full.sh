#!/bin/bash
# Full GPU check: every -m gpu test, smoke(), then the default bench (one box, one call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_$tag.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu_$tag.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 5; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 6; }
tail -1 gpurun_out/bench_$tag.log
