#!/bin/bash
# Hash feature-pass step: GPU Hash tests (bitwise vs the gather kernel), then in-process A/Bs: packed arithmetic vs the
# round-3 form (debug library, hash_feat_abl 8) at the default P, and P at the new arithmetic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hash.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_hash.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_hash.log
[ $rc -eq 0 ] || exit $rc
NRC_LIB_PATH=neural-radiance-caching_amd/libnrc_amd_debug.so timeout -k 10 200 python tools/ab_hash_p.py --knob hash_feat_abl --ps=-1,16,8 --rounds 7 > gpurun_out/ab_hash_abl8.json 2> gpurun_out/ab_hash_abl8.err || exit 4
cat gpurun_out/ab_hash_abl8.json
timeout -k 10 200 python tools/ab_hash_p.py --ps 32,16 --rounds 5 > gpurun_out/ab_hash_p2.json 2> gpurun_out/ab_hash_p2.err || exit 5
cat gpurun_out/ab_hash_p2.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -k "peer" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_peer3.log 2>&1 || { echo "peer tests failed"; tail -20 gpurun_out/pytest_peer3.log; exit 9; }
tail -1 gpurun_out/pytest_peer3.log
