#!/bin/bash
# round-4 GPU step: tcnn-numerics tests, peer-exchange tests, then the 2-tile energy A/B (stops at a test failure)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tcnn_numerics.py "tests/test_gpu_dp.py::test_peer_exchange_argument_checks" "tests/test_gpu_dp.py::test_two_ranks_on_one_gpu_peer_exchange" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_r04b.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_r04b.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
NRC_LIB_PATH=neural-radiance-caching_amd/libnrc_amd_debug.so timeout -k 10 400 python tools/energy_ab.py --variants 47,52,56,57,58,59 --rounds 3 > gpurun_out/energy_ab_2tile_b.json 2> gpurun_out/energy_ab_2tile_b.err
echo "energy rc=$?"
exit $rc
