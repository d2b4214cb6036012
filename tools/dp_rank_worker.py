"""One rank of tests/test_gpu_dp.py::test_two_ranks_on_one_gpu_gloo: torch.distributed over gloo, the real HIP
nrc_train_grad / nrc_train_apply through nrc_amd.dp.DataParallelTrainer, every rank on cuda:0.

    RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tools/dp_rank_worker.py <out_dir> [global_batch]
        [encoding] [steps] [exchange]

global_batch (default 16,384) is split over the ranks; 4,096 gives configs[3]'s per-rank slice of 2,048 samples.
encoding Hash: the exact grid exchange (DataParallelTrainer with an int64 grid_fixed buffer).
exchange "peer": the library's one-shot peer exchange (nrc_peer_exchange_*, handles all-gathered over gloo) through
nrc_train_dp instead of the Python all-reduce, fused into the reduction (the production path); "peer_push": the same
exchange as separate reduce / push / apply launches (knob peer_path = 0). Both ranks share cuda:0, so "peer" runs
the split form of the fused exchange (nrc_peer_exchange_open detects the shared device).
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main() -> None:
    import torch
    import torch.distributed as dist

    out = Path(sys.argv[1])
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    encoding = sys.argv[3] if len(sys.argv) > 3 else "Frequency"
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    peer = len(sys.argv) > 5 and sys.argv[5] in ("peer", "peer_push")
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    nrc = nrc_loader.load()
    if len(sys.argv) > 5 and sys.argv[5] == "peer_push":
        nrc._lib.set_knob("peer_path", 0)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), encoding=getattr(nrc.InputEncoding, encoding))
    if (out / "params.npy").exists():
        net.set_state(nrc.StateSlot.PARAMS, np.load(out / "params.npy"))
    grad = torch.zeros(net.grad_floats, dtype=torch.float32, device=dev)
    if encoding == "Hash":
        fixed = torch.zeros(nrc.HASH_GRID_PARAMS, dtype=torch.int64, device=dev)
        trainer = nrc.dp.DataParallelTrainer(net, grad, grid_fixed=fixed, mlp_params=nrc.HASH_MLP_PARAMS)
    else:
        trainer = nrc.dp.DataParallelTrainer(net, grad)
    trainer.broadcast_state(net, dev)
    if peer:
        nrc.dp.open_peer_exchange(net)
    losses = []
    for it in range(steps):
        q, t = nrc.synthetic.cornell_batch(B, seed=80 + it)
        s, c = nrc.dp.shard_range(B, rank, world)
        qd = torch.from_numpy(np.ascontiguousarray(q[s:s + c])).to(dev)
        td = torch.from_numpy(np.ascontiguousarray(t[s:s + c])).to(dev)
        losses.append(net.train_dp(qd, td, c, B, loss=True) if peer else trainer.step(qd, td, c, B, loss=True))
    torch.cuda.synchronize()
    if peer:
        dist.barrier()  # no rank unmaps or frees a buffer a peer may still write
        net.peer_exchange_close()
    np.save(out / f"params_{rank}.npy", net.get_state(nrc.StateSlot.PARAMS))
    np.save(out / f"infer_{rank}.npy", net.get_state(nrc.StateSlot.INFER))
    np.save(out / f"loss_{rank}.npy", np.array(losses))
    net.destroy()
    dist.destroy_process_group()
    print(f"rank {rank} ok")


if __name__ == "__main__":
    main()
