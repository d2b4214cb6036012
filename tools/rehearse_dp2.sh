#!/bin/bash
# Rehearsals of the N > 1 bench path on a 1-GPU box (not measurements):
#  (1) two ranks sharing the GPU over gloo (torch.distributed.run, the Python all-reduce: RCCL cannot put two ranks
#      on one device), C4 sharding of the queries and of every minibatch;
#  (2) N = 1 with --rehearse-comm: training through a world-1 RCCL communicator inside the library (nrc_train_dp).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --train-frames 2 --frame-iters 0 --no-cpu --no-wide --no-hash --dist-backend gloo > gpurun_out/mr2.log 2>&1; rc=$?
tail -1 gpurun_out/mr2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --train-frames 2 --frame-iters 0 --no-cpu --no-wide --no-hash --rehearse-comm > gpurun_out/mr1_comm.log 2>&1; rc=$?
tail -1 gpurun_out/mr1_comm.log; exit $rc
