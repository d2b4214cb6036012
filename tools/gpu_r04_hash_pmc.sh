#!/bin/bash
# PMC passes over the Hash inference + training bench (tools/bench_hash.py), summary of the feature-pass and MLP kernels,
# and a kernel-trace summary of the same command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_pmc.sh pmc_hash python3 "$ROOT/tools/bench_hash.py" --iters 5 || exit 6
python tools/pmc_summary.py gpurun_out/pmc_hash hash > gpurun_out/pmc_hash_summary.txt || exit 7
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_hash" -o run --output-format csv -- python3 "$ROOT/tools/bench_hash.py" --iters 30 > "$ROOT/gpurun_out/prof_hash.log" 2>&1) || exit 8
tail -1 gpurun_out/prof_hash.log
