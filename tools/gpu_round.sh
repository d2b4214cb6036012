#!/bin/bash
# GPU sessions on a gpurun box, one subcommand per call (each under gpurun's 20-minute limit). Every GPU step runs
# under its own timeout; a failing step ends the call with its own exit code (no retries). Outputs under gpurun_out/.
#
#   tools/gpu_round.sh tests [pytest args...]   GPU tests (default: the whole -m gpu suite), then smoke()
#   tools/gpu_round.sh pytest <paths...>         just the given GPU tests (no smoke)
#   tools/gpu_round.sh bench                     PMC passes of the bench (HBM bytes -> profiles/pmc_infer_<round>.json on
#                                                the box), the default bench line, rocprofv3 kernel-trace stats of the bench
#                                                and of train-only runs (width 64 and 128)
#   tools/gpu_round.sh bench-line [args...]      one bench.py line (default flags unless given)
#   tools/gpu_round.sh ab-infer <n> <variants> [rounds] [iters]   in-process A/B of inference variants (debug library)
#   tools/gpu_round.sh energy <variants> [rounds]                 J/query A/B of inference variants (debug library)
#   tools/gpu_round.sh power [power_paths.py args...]             power / clock / nJ per query of the product paths
#   tools/gpu_round.sh hash-abl <knob values> [knob]              Hash feature-pass A/B over a knob (tools/ab_hash_p.py)
#   tools/gpu_round.sh hash-train-ab [values] [knob] [tag] [k=v...] fused Hash training step A/B (tools/ab_hash_train.py)
#   tools/gpu_round.sh bench-hash [k=v...]                        tools/bench_hash.py with knobs (Hash inference + train step)
#   tools/gpu_round.sh pmc-train                                  PMC passes of the 64-wide training step
#   tools/gpu_round.sh pmc-hash                                   PMC + kernel trace of tools/bench_hash.py
#   tools/gpu_round.sh dp-timing                                  2-rank DP timing (tools/gpu_dp_timing.sh)
#   tools/gpu_round.sh rehearse-dp2                               2 ranks on one GPU through bench.py (tools/rehearse_dp2.sh)
# Subcommands can be chained in one gpurun call with &&.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
ROUND=$(python3 -c "import re;print(re.search(r'^ROUND = \"(r\d+)\"', open('bench.py').read(), re.M).group(1))")
DEBUG_LIB="$ROOT/neural-radiance-caching_amd/libnrc_amd_debug.so"
cmd="${1:-tests}"
[ $# -gt 0 ] && shift

run_pytest() {  # <log name> <timeout s> <pytest args...>
  local log=$1 to=$2; shift 2
  timeout -k 10 "$to" python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "pytest rc=$rc"; tail -3 "gpurun_out/$log"
  return $rc
}

case "$cmd" in
tests)
  if [ $# -gt 0 ]; then run_pytest pytest_gpu.log 1000 "$@" || exit $?
  else run_pytest pytest_gpu.log 1000 tests -m gpu || exit $?; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 3; }
  tail -2 gpurun_out/smoke.log
  ;;
pytest)
  run_pytest pytest_sel.log 900 "$@" || exit $?
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
bench-line)
  timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_line.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_line.log; exit 4; }
  tail -1 gpurun_out/bench_line.log
  ;;
ab-infer)
  n=$1 variants=$2 rounds=${3:-9} iters=${4:-30}
  NRC_LIB_PATH="$DEBUG_LIB" timeout -k 10 300 python tools/ab_infer.py --n "$n" --variants "$variants" --weights bench --rounds "$rounds" --iters "$iters" > "gpurun_out/ab_infer_$n.json" 2> "gpurun_out/ab_infer_$n.err" || { echo "A/B $n failed"; tail -20 "gpurun_out/ab_infer_$n.err"; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_infer_$n.json'));print($n,{k:round(v['median_us'],2) for k,v in d['variants'].items()})"
  ;;
energy)
  variants=$1 rounds=${2:-3}
  NRC_LIB_PATH="$DEBUG_LIB" timeout -k 10 400 python tools/energy_ab.py --variants "$variants" --rounds "$rounds" > gpurun_out/energy_ab.json 2> gpurun_out/energy_ab.err || { echo "energy A/B failed"; tail -20 gpurun_out/energy_ab.err; exit 2; }
  tail -c 2000 gpurun_out/energy_ab.json
  ;;
power)
  timeout -k 10 300 python tools/power_paths.py "$@" > gpurun_out/power_paths.json 2> gpurun_out/power_paths.err || { echo "power_paths failed"; tail -20 gpurun_out/power_paths.err; exit 3; }
  python -c "
import json; d=json.load(open('gpurun_out/power_paths.json'))
print('idle', d['idle'])
for p, r in d['paths'].items(): print(p, {k: r.get(k) for k in ('us_median','power_w','gfx_mhz','nj_per_query')})
"
  ;;
hash-abl)
  values=$1 knob=${2:-hash_feat_abl}
  NRC_LIB_PATH="$DEBUG_LIB" timeout -k 10 300 python tools/ab_hash_p.py --knob "$knob" --ps="$values" --rounds 5 > gpurun_out/ab_hash.json 2> gpurun_out/ab_hash.err || { echo "hash A/B failed"; tail -20 gpurun_out/ab_hash.err; exit 4; }
  cat gpurun_out/ab_hash.json
  ;;
hash-train-ab)
  values=${1:-16,0,2,4,6,8} knob=${2:-scatter_part} tag=${3:-0}; shift $(( $# < 3 ? $# : 3 ))
  held=(); for kv in "$@"; do held+=(--set "$kv"); done
  timeout -k 10 300 python tools/ab_hash_train.py --knob "$knob" --values="$values" "${held[@]}" > "gpurun_out/ab_hash_train_$tag.json" 2> "gpurun_out/ab_hash_train_$tag.err" || { echo "hash train A/B failed"; tail -20 "gpurun_out/ab_hash_train_$tag.err"; exit 4; }
  cat "gpurun_out/ab_hash_train_$tag.json"
  ;;
bench-hash)  # tools/bench_hash.py (Hash inference + training step) with optional knobs: bench-hash [name=value ...]
  kn=(); for kv in "$@"; do kn+=(--knob "$kv"); done
  timeout -k 10 120 python tools/bench_hash.py --iters 30 "${kn[@]}" > gpurun_out/bench_hash.json || { echo "bench_hash failed"; exit 5; }
  grep -E "train_step|infer_us" gpurun_out/bench_hash.json
  ;;
pmc-train)  # PMC passes of the 64-wide training step (tools/time_train.py)
  bash tools/gpu_pmc.sh pmc_t16 python3 "$ROOT/tools/time_train.py" --rounds 1 --iters 10 || exit 6
  python tools/pmc_summary.py gpurun_out/pmc_t16 train > gpurun_out/pmc_t16.txt || exit 7
  cat gpurun_out/pmc_t16.txt
  ;;
pmc-hash)
  bash tools/gpu_pmc.sh pmc_hash python3 "$ROOT/tools/bench_hash.py" --iters 5 || exit 6
  python tools/pmc_summary.py gpurun_out/pmc_hash hash > gpurun_out/pmc_hash_summary.txt || exit 7
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_hash" -o run --output-format csv -- python3 "$ROOT/tools/bench_hash.py" --iters 30 > "$ROOT/gpurun_out/prof_hash.log" 2>&1) || exit 8
  tail -1 gpurun_out/prof_hash.log
  ;;
dp-timing)
  bash tools/gpu_dp_timing.sh || exit $?
  ;;
rehearse-dp2)
  bash tools/rehearse_dp2.sh || { echo "rehearsal failed"; exit 3; }
  ;;
*)
  echo "unknown subcommand $cmd"; exit 64
  ;;
esac
echo "all done"
