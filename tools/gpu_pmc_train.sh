set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_pmc.sh pmc_t16 python3 "$GRAFT_REPO_ROOT/tools/time_train.py" --rounds 1 --iters 10 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_t16 train > gpurun_out/pmc_t16.txt && cat gpurun_out/pmc_t16.txt
