#!/bin/bash
# Round-end GPU session, in two calls (each under gpurun's 20-minute limit). Stops at the first failure; outputs
# under gpurun_out/.
#   tools/gpu_round.sh tests  : full GPU tests, smoke
#   tools/gpu_round.sh bench  : PMC passes of the bench (tools/gpu_pmc.sh; HBM bytes -> profiles/pmc_infer_<round>.json
#                               on the box, so the bench line below carries the traffic of this box), the bench,
#                               rocprofv3 kernel-trace stats of the bench and of a train-only run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=$(python3 -c "import re;print(re.search(r'^ROUND = \"(r\d+)\"', open('bench.py').read(), re.M).group(1))")
case "${1:-tests}" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo "pytest failed (rc=$rc): stopping"; exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 3; }
  tail -2 gpurun_out/smoke.log
  ;;
bench)
  bash tools/gpu_pmc.sh pmc_bench python3 "$ROOT/bench.py" --steps 10 --warmup 2 --train-frames 2 --no-cpu --sustained 0 --frame-iters 2 --no-wide --no-hash --no-c4 || exit 6
  python tools/pmc_to_json.py gpurun_out/pmc_bench infer_kernel gpurun_out/pmc_infer.json > /dev/null || exit 7
  python tools/pmc_summary.py gpurun_out/pmc_bench > gpurun_out/pmc_bench_summary.txt || exit 8
  cp gpurun_out/pmc_infer.json "profiles/pmc_infer_$ROUND.json"
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
  tail -1 gpurun_out/bench.log
  # --no-c4: the infer kernel's rocprof summary then holds the 2^21-query launches only (the C4 shards'
  # 2^19-query launches had been averaged in); the profiled run prints its own bench line (prof_bench.log)
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --train-frames 5 --no-cpu --no-c4 --sustained 200 > "$ROOT/gpurun_out/prof_bench.log" 2>&1 || { echo "rocprof failed"; tail -20 "$ROOT/gpurun_out/prof_bench.log"; exit 5; }
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train" -o run --output-format csv -- python3 "$ROOT/tools/time_train.py" --rounds 3 --iters 40 > "$ROOT/gpurun_out/prof_train.log" 2>&1 || { echo "train rocprof failed"; tail -20 "$ROOT/gpurun_out/prof_train.log"; exit 9; }
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train128" -o run --output-format csv -- python3 "$ROOT/tools/time_train.py" --width 128 --rounds 3 --iters 40 > "$ROOT/gpurun_out/prof_train128.log" 2>&1 || { echo "train128 rocprof failed"; exit 10; }
  ;;
esac
echo "all done"
