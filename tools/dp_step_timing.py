"""Per-step time of data-parallel training on one GPU shared by the ranks: the library's one-shot
peer exchange (nrc_peer_exchange_* + nrc_train_dp; fused into the reduction, and as separate launches) against the Python all-reduce over gloo (DataParallelTrainer), for
the reference's per-step minibatch split over the ranks (b_local = 16,384 / world) and weak-scaled (b_local = 16,384).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \\
        tools/dp_step_timing.py [--steps 200]

Both ranks share one card here, so a step's time includes the other rank's kernels; the exchange kernels' own durations
come from a rocprofv3 kernel trace of the same command. Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    nrc = nrc_loader.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream()
    B = nrc.BATCH_SIZE
    q_np, t_np = nrc.synthetic.cornell_batch(B, seed=5)
    q, t = torch.from_numpy(q_np).to(dev), torch.from_numpy(t_np).to(dev)
    res = {}
    for split in (True, False):
        b_local = B // world if split else B
        global_b = B if split else B * world
        s0 = rank * b_local if split else 0
        qs, ts = q[s0:s0 + b_local], t[s0:s0 + b_local]
        for mode in ("peer", "peer_push", "gloo"):
            # peer: the exchange fused into the reduction (production); peer_push: reduce / push / apply launches
            nrc._lib.set_knob("peer_path", 0 if mode == "peer_push" else -1)
            net = nrc.Network()
            net.init(stream=stream)
            grad = torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev)
            trainer = nrc.dp.DataParallelTrainer(net, grad)
            trainer.broadcast_state(net, dev)
            if mode.startswith("peer"):
                nrc.dp.open_peer_exchange(net)
                step = lambda: net.train_dp(qs, ts, b_local, global_b)  # noqa: E731
            else:
                step = lambda: trainer.step(qs, ts, b_local, global_b)  # noqa: E731
            for _ in range(args.warmup):
                step()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps * 1e6
            worst = torch.tensor([dt])
            dist.all_reduce(worst, op=dist.ReduceOp.MAX)
            p = net.get_state(nrc.StateSlot.PARAMS)
            ps = [torch.zeros(p.size) for _ in range(world)]
            dist.all_gather(ps, torch.from_numpy(p))
            same = all(torch.equal(ps[0], x) for x in ps[1:])
            res[f"{mode}_{'split' if split else 'weak'}"] = {"b_local": b_local, "global_b": global_b,
                                                            "us_per_step": float(worst.item()), "replicas_equal": same}
            if mode.startswith("peer"):
                dist.barrier()
                net.peer_exchange_close()
            net.destroy()
    if rank == 0:
        print(json.dumps({"world": world, "one_gpu_shared": True, "steps": args.steps, "results": res}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
