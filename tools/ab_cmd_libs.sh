#!/bin/bash
# Alternating-process A/B of any timing command across builds: tools/ab_cmd_libs.sh "<cmd>" <lib1> <lib2> ...
# (each run: NRC_LIB_PATH=<lib> <cmd>; prints the last stdout line of every run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CMD=$1; shift
for rep in 1 2 3; do
  for L in "$@"; do
    r=$(NRC_LIB_PATH=$L timeout -k 10 180 bash -c "$CMD" 2>/dev/null | tr -d '\n' ) || exit 1
    echo "$L $r"
  done
done
