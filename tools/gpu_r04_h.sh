#!/bin/bash
# round 4: fewer waves per CU for the C4 shard's tail (debug variants 61/62 vs 47), in-process A/B at 2^19 and 2^21
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export NRC_LIB_PATH=$(pwd)/neural-radiance-caching_amd/libnrc_amd_debug.so
timeout -k 10 300 python tools/ab_infer.py --n 524288 --variants 47,61,62 --weights bench --rounds 9 --iters 40 > gpurun_out/ab_tail_2pow19.json 2> gpurun_out/ab_tail_2pow19.err || { echo "A/B 2^19 failed"; tail -20 gpurun_out/ab_tail_2pow19.err; exit 2; }
tail -c 1500 gpurun_out/ab_tail_2pow19.json
timeout -k 10 300 python tools/ab_infer.py --n 2097152 --variants 47,61,62 --weights bench --rounds 7 --iters 20 > gpurun_out/ab_tail_2pow21.json 2> gpurun_out/ab_tail_2pow21.err || { echo "A/B 2^21 failed"; tail -20 gpurun_out/ab_tail_2pow21.err; exit 3; }
tail -c 1500 gpurun_out/ab_tail_2pow21.json
