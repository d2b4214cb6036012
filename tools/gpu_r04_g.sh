#!/bin/bash
# round 4: own partials in registers (fused exchange) -- DP GPU tests, the N > 1 bench rehearsal (2 ranks on one GPU:
# the split exchange inside bench.py's dp_exchange leg), one default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_stream.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1 || { echo "dp tests failed"; tail -40 gpurun_out/pytest_dp.log; exit 2; }
tail -2 gpurun_out/pytest_dp.log
bash tools/rehearse_dp2.sh || { echo "rehearsal failed"; exit 3; }
timeout -k 10 600 python bench.py > gpurun_out/bench_g.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_g.log; exit 4; }
tail -1 gpurun_out/bench_g.log
