#!/bin/bash
# Cross-build A/B of the training step (alternating processes): tools/ab_train_libs.sh <lib1> <lib2> ...
# Prints the step timings of tools/ab_train.py and the phase medians of tools/train_stamps.py per build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
  for L in "$@"; do
    r=$(NRC_LIB_PATH=$L timeout -k 10 120 python tools/ab_train.py 2>/dev/null | grep '^{') || exit 1
    echo "$L $r"
  done
done
for L in "$@"; do
  r=$(NRC_LIB_PATH=$L timeout -k 10 120 python tools/train_stamps.py 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'end_max': d['end_max'], **d['phase_median']}))") || exit 1
  echo "$L stamps $r"
done
