bash tools/gpu_round.sh pytest tests/test_gpu_hash.py tests/test_gpu_hash_exchange.py tests/test_gpu_padded.py -v || exit 1
for k in 32 16 8; do timeout -k 10 120 python tools/bench_hash.py --iters 30 --knob hash_feat_p=$k > gpurun_out/bh_p$k.json || exit 5; grep -E "train_step" gpurun_out/bh_p$k.json; done
timeout -k 10 120 python tools/bench_hash.py --iters 30 > gpurun_out/bh_def.json || exit 6
timeout -k 10 120 python tools/bench_hash.py --iters 30 --knob train_kernel=32 > gpurun_out/bh_32.json || exit 7
grep -E "train_step|infer_us" gpurun_out/bh_def.json gpurun_out/bh_32.json
bash tools/gpu_round.sh hash-abl -1,128 || exit 8
