set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
grep -h "grad rel vs mixed" gpurun_out/pytest_gpu.log | head -3
[ $rc -eq 0 ] || exit $rc
bash tools/ab_train_libs.sh build/ab/lib_redoff.so build/ab/lib_slab16h.so 2>&1 | grep -v stamps
