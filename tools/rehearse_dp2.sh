#!/bin/bash
# Rehearsal of the N = 2 bench path (torch.distributed.run, DataParallelTrainer, all_reduce) with two ranks sharing
# one GPU over gloo: checks the multi-rank code path on a 1-GPU box. Not a measurement (the ranks share the GPU).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --train-frames 2 --frame-iters 0 --no-cpu --dist-backend gloo > gpurun_out/mr2.log 2>&1; rc=$?
tail -3 gpurun_out/mr2.log; exit $rc
