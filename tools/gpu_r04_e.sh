#!/bin/bash
# round 4: padded RadianceQuery layout + the fused peer exchange -- their GPU tests first, then the full suite +
# smoke, the 2-rank DP timing (fused vs separate launches vs gloo) with kernel traces, and one default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_padded.py tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 gpurun_out/pytest_new.log; exit 2; }
tail -2 gpurun_out/pytest_new.log
bash tools/gpu_round.sh tests || exit $?
bash tools/gpu_dp_timing.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_e.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_e.log; exit 4; }
tail -1 gpurun_out/bench_e.log
