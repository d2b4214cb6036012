#!/bin/bash
# round 4: the tagged-word exchange -- DP GPU tests (world-1 fused, 2-rank split, knob 0), the 2-rank DP timing with
# kernel traces, one default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1 || { echo "dp tests failed"; tail -40 gpurun_out/pytest_dp.log; exit 2; }
tail -2 gpurun_out/pytest_dp.log
bash tools/gpu_dp_timing.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_f.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_f.log; exit 4; }
tail -1 gpurun_out/bench_f.log
