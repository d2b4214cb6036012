#!/bin/bash
# round-4 mid-round check: the full GPU suite + smoke on this tree, the Hash feature-pass ablations, one default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_round.sh tests || exit $?
bash tools/gpu_r04_hash_abl.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_mid.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_mid.log; exit 4; }
tail -1 gpurun_out/bench_mid.log
