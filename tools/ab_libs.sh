#!/bin/bash
# Cross-build A/B (same box, alternating processes): tools/ab_libs.sh <variant> <lib1> <lib2> ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$1; shift
for rep in 1 2 3; do
  for L in "$@"; do
    r=$(NRC_LIB_PATH=$L timeout -k 10 120 python tools/ab_infer.py --variants $V --rounds 5 --iters 20 | python3 -c "import json,sys; d=json.load(sys.stdin); print('%.1f'%list(d['variants'].values())[0]['median_us'])") || exit 1
    echo "$L $r us"
  done
done
