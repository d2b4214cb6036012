set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "train or fused or hyper or determin or set_config" > gpurun_out/t16_tests.log 2>&1; rc=$?
tail -4 gpurun_out/t16_tests.log
if [ $rc -gt 1 ]; then echo "tests crashed rc=$rc"; exit $rc; fi
timeout -k 10 200 python tools/ab_train.py > gpurun_out/ab_train.json 2>gpurun_out/ab_train.err && cat gpurun_out/ab_train.json
timeout -k 10 120 python tools/train_stamps.py > gpurun_out/stamps16.json 2>gpurun_out/stamps16.err && cat gpurun_out/stamps16.json || tail gpurun_out/stamps16.err
