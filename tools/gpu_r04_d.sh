#!/bin/bash
# round 4: the peer exchange fused into the reduction -- its GPU tests first, then the full suite + smoke, the 2-rank
# DP timing (fused vs separate launches vs gloo) with kernel traces, and one default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1 || { echo "dp tests failed"; tail -30 gpurun_out/pytest_dp.log; exit 2; }
tail -2 gpurun_out/pytest_dp.log
bash tools/gpu_round.sh tests || exit $?
bash tools/gpu_dp_timing.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_d.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_d.log; exit 4; }
tail -1 gpurun_out/bench_d.log
