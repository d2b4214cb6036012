#!/bin/bash
# Quick GPU iteration: parity tests + in-process A/B of the inference variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab_infer.py "$@" > gpurun_out/ab_infer.json 2> gpurun_out/ab_infer.err || { tail gpurun_out/ab_infer.err; exit 4; }
cat gpurun_out/ab_infer.json
