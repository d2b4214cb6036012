set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_cmd_libs.sh "python tools/bench_hash.py | python tools/jfield.py infer_us train_step_us" build/ab/lib_gate.so build/ab/lib_hpair.so
