set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/cvt_clamp_probe > gpurun_out/cvt_clamp.json || exit 3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "encode_fast or every_infer_variant or set_hyper or set_config" > gpurun_out/pt_r02a.log 2>&1 || { tail -30 gpurun_out/pt_r02a.log; exit 4; }
tail -3 gpurun_out/pt_r02a.log
timeout -k 10 300 python tools/ab_infer.py --variants 23,30,31,32 --rounds 7 --iters 20 > gpurun_out/ab_r02a.json 2>&1 || exit 5
timeout -k 10 300 python tools/ab_infer.py --n 16777216 --variants 23,30,31,32 --rounds 5 --iters 5 > gpurun_out/ab_r02a_24.json 2>&1 || exit 6
cat gpurun_out/cvt_clamp.json gpurun_out/ab_r02a.json gpurun_out/ab_r02a_24.json
