"""Data-parallel sharding of the NRC hot path over one process per GPU (torch.distributed).

New capability: the reference runs one independent, unsynchronised network
per device (/root/reference/nrc/src/Device.cpp:420, nrc/inc/Device.h:621) and has no collectives.

* Inference: queries are independent units; each rank takes a contiguous shard of the frame's
  queries. No collective on the data path.
* Training: one exchange step per minibatch. Each rank computes the loss-scaled gradient of its local
  samples normalised by the GLOBAL batch (3 * global_b), the ranks sum it (one all-reduce of
  NRC_GRAD_FLOATS f32 = 88 KiB, or NRC_HASH_GRAD_FLOATS = 3.9 MiB with the grid-table gradient for
  InputEncoding::Hash: RCCL over xGMI with the "nccl" backend; gloo on CPU), and every rank applies the
  identical Adam + EMA step (Hash: plus the sparse grid Adam over the entries with a non-zero summed
  gradient), so replicas stay bit-identical.

``backend`` is any object with ``train_grad(inputs, targets, b, global_b, grad)`` and
``train_apply(grad, loss)`` — ``network.Network`` on the GPU, an oracle-backed stand-in in the
CPU tests. With a ``grid_fixed`` buffer (InputEncoding::Hash: int64 [HASH_GRID_PARAMS]) the trainer uses the exact
grid exchange instead (``train_grad_fixed`` / ``train_apply_fixed``, nrc_c.h): the f32 all-reduce covers only the MLP
gradient and the loss, the grid sums travel as int64 and are rounded to f16 once, after the sum over ranks.
"""
from __future__ import annotations


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [start, start + count) of n units for rank (sizes differ by at most 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, rem = divmod(int(n), int(world))
    start = rank * base + min(rank, rem)
    count = base + (1 if rank < rem else 0)
    return start, count


def open_peer_exchange(net, group=None) -> None:
    """Set up the library's one-shot peer gradient exchange (nrc_peer_exchange_*) on every rank of the group: each rank
    allocates its receive buffer, the 64-byte IPC handles are all-gathered over torch.distributed (any backend), and
    every rank maps its peers' buffers. Afterwards ``net.train_dp`` exchanges gradients GPU to GPU without RCCL."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    mine = torch.frombuffer(bytearray(net.peer_exchange_handle(world)), dtype=torch.uint8)
    if dist.get_backend(group) == "nccl":
        mine = mine.cuda()
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    net.peer_exchange_open(rank, world, b"".join(bytes(p.cpu().numpy().tobytes()) for p in parts))
    dist.barrier(group=group)


class DataParallelTrainer:
    def __init__(self, backend, grad_buffer, group=None, grid_fixed=None, mlp_params: int | None = None):
        import torch.distributed as dist

        self.backend = backend
        self.grad = grad_buffer  # torch tensor of backend.grad_floats f32 on the backend's device
        self.group = group
        self.grid_fixed = grid_fixed  # Hash exact exchange: int64 [HASH_GRID_PARAMS] on the backend's device
        # with grid_fixed: the MLP part of grad (loss at grad[-4]); required, since grad[:None] would be the whole
        # buffer (the loss summed twice and the unwritten grid part reduced)
        if grid_fixed is not None and (mlp_params is None or not 0 < int(mlp_params) <= len(grad_buffer) - 4):
            raise ValueError("DataParallelTrainer: grid_fixed needs mlp_params (HASH_MLP_PARAMS), the MLP part of grad")
        self.mlp_params = None if mlp_params is None else int(mlp_params)
        self._dist = dist

    def broadcast_state(self, net, device) -> None:
        """Make every replica continue from rank 0's complete optimizer state: the five state slots (weights, the
        inference/EMA weights, the raw EMA, Adam m and v) and the Adam step counter, which sets the bias
        corrections of the next step. InputEncoding::Hash also keeps a step counter per grid entry that the C-ABI
        does not export, so for a Hash network this is only allowed before the first step (all counters 0)."""
        import torch

        from .network import InputEncoding, StateSlot

        step = torch.tensor([int(net.step)], dtype=torch.int64, device=device)
        self._dist.broadcast(step, src=0, group=self.group)
        if getattr(net, "encoding", None) == InputEncoding.Hash and int(step.item()) != 0:
            raise RuntimeError("broadcast_state: a Hash network can only be synchronised before its first step")
        for slot in StateSlot:
            t = torch.from_numpy(net.get_state(slot)).to(device)
            self._dist.broadcast(t, src=0, group=self.group)
            net.set_state(slot, t.cpu().numpy())
        net.step = int(step.item())

    def step(self, inputs, targets, b_local: int, global_b: int, loss: bool = False):
        if self.grid_fixed is not None:
            self.backend.train_grad_fixed(inputs, targets, b_local, global_b, self.grad, self.grid_fixed)
            sum_ = self._dist.ReduceOp.SUM
            self._dist.all_reduce(self.grad[:self.mlp_params], op=sum_, group=self.group)
            self._dist.all_reduce(self.grad[-4:], op=sum_, group=self.group)
            self._dist.all_reduce(self.grid_fixed, op=sum_, group=self.group)
            return self.backend.train_apply_fixed(self.grad, self.grid_fixed, loss)
        self.backend.train_grad(inputs, targets, b_local, global_b, self.grad)
        self._dist.all_reduce(self.grad, op=self._dist.ReduceOp.SUM, group=self.group)
        return self.backend.train_apply(self.grad, loss)
