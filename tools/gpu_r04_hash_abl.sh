#!/bin/bash
# Hash feature-pass ablations (debug library, timing only): where the pass's time goes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NRC_LIB_PATH=neural-radiance-caching_amd/libnrc_amd_debug.so timeout -k 10 300 python tools/ab_hash_p.py --knob hash_feat_abl --ps=-1,1,2,4,32,33,36 --rounds 5 > gpurun_out/ab_hash_ablations.json 2> gpurun_out/ab_hash_ablations.err || exit 4
cat gpurun_out/ab_hash_ablations.json
