#!/bin/bash
# round 4: where the 3-waves-per-SIMD shape (variant 62) stops paying: A/B 47 vs 62 at 2^19, 3 * 2^18, 2^20, 3 * 2^19
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export NRC_LIB_PATH=$(pwd)/neural-radiance-caching_amd/libnrc_amd_debug.so
for n in 524288 786432 1048576 1572864; do
  timeout -k 10 300 python tools/ab_infer.py --n $n --variants 47,62 --weights bench --rounds 9 --iters 30 > gpurun_out/ab_tail_$n.json 2> gpurun_out/ab_tail_$n.err || { echo "A/B $n failed"; tail -20 gpurun_out/ab_tail_$n.err; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_tail_$n.json'));print($n,{k:round(v['median_us'],2) for k,v in d['variants'].items()})"
done
# the product's small-launch shape (kInferSmallN): parity, determinism and padded tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_padded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_small.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_small.log; exit 3; }
tail -2 gpurun_out/pytest_small.log
