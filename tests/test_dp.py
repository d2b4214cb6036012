"""Data-parallel sharding on CPU: torch.distributed gloo, world size 2 (the N > 1 path of bench.py,
with the gfx950 backend replaced by an oracle-backed stand-in that has the same train_grad /
train_apply contract as nrc_amd.Network).

Checks: contiguous query shards cover the frame exactly once; a DP step over 2 ranks equals one
single-process step on the concatenated batch; replicas stay bit-identical (Frequency and Hash).
"""
import os
import socket

import numpy as np
import pytest

import nrc_loader


def test_shard_range_covers_exactly_once(nrc):
    for n in [0, 1, 7, 1 << 21, (1 << 22) + 3]:
        for world in [1, 2, 3, 8]:
            seen = 0
            prev_end = 0
            for r in range(world):
                s, c = nrc.dp.shard_range(n, r, world)
                assert s == prev_end and c >= 0
                prev_end = s + c
                seen += c
            assert seen == n and prev_end == n
    with pytest.raises(ValueError):
        nrc.dp.shard_range(10, 2, 2)


class OracleBackend:
    """Stand-in for nrc_amd.Network on CPU (test only): same train_grad / train_apply contract."""

    def __init__(self, params, hash_grid=False):
        self.orc = nrc_loader.load_oracle()
        self.hash_grid = hash_grid
        self.st = (self.orc.HashAdamEmaState if hash_grid else self.orc.AdamEmaState)(params)
        self.grad_floats = params.size + 4

    def train_grad(self, q, t, b, global_b, grad):
        import torch

        fn = self.orc.hash_grad if self.hash_grid else self.orc.grad
        g, loss = fn(self.st.params, q[:b], t[:b], n_total=3.0 * global_b, mode=self.orc.FP32, threads=2)
        grad.zero_()
        grad[: g.size] = torch.from_numpy(g)
        grad[g.size] = loss

    def train_apply(self, grad, loss=False):
        self.st.apply(grad[: self.st.params.size].numpy().astype(np.float32))
        return float(grad[self.st.params.size]) if loss else None


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init_params(orc, hash_grid):
    if hash_grid:
        p = orc.hash_init_params(1337)
        p[orc.HASH_MLP_PARAMS:] = np.random.default_rng(2).uniform(-0.5, 0.5, orc.HASH_GRID_PARAMS).astype(np.float32)
        return p
    return orc.init_params(1337) * np.float32(1.5)


def _worker(rank, world, port, B, steps, out_dir, hash_grid=False):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nrc = nrc_loader.load()
    orc = nrc_loader.load_oracle()
    params = _init_params(orc, hash_grid)
    backend = OracleBackend(params, hash_grid)
    grad = torch.zeros(backend.grad_floats, dtype=torch.float32)
    trainer = nrc.dp.DataParallelTrainer(backend, grad)
    losses = []
    for it in range(steps):
        q, t = nrc.synthetic.cornell_batch(B, seed=40 + it)
        s, c = nrc.dp.shard_range(B, rank, world)
        losses.append(trainer.step(q[s:s + c], t[s:s + c], c, B, loss=True))
    np.save(os.path.join(out_dir, f"params_{rank}.npy"), backend.st.params)
    np.save(os.path.join(out_dir, f"infer_{rank}.npy"), backend.st.infer)
    np.save(os.path.join(out_dir, f"loss_{rank}.npy"), np.array(losses))
    dist.destroy_process_group()


def test_dp_step_equals_single_process_step(tmp_path):
    import torch.multiprocessing as mp

    world, B, steps = 2, 384, 3
    mp.spawn(_worker, args=(world, _free_port(), B, steps, str(tmp_path)), nprocs=world, join=True)
    orc = nrc_loader.load_oracle()
    nrc = nrc_loader.load()
    st = orc.AdamEmaState(orc.init_params(1337) * np.float32(1.5))
    ref_losses = []
    for it in range(steps):
        q, t = nrc.synthetic.cornell_batch(B, seed=40 + it)
        g, loss = orc.grad(st.params, q, t, mode=orc.FP32, threads=2)
        st.apply(g)
        ref_losses.append(loss)
    p0, p1 = np.load(tmp_path / "params_0.npy"), np.load(tmp_path / "params_1.npy")
    np.testing.assert_array_equal(p0, p1)  # replicas identical
    np.testing.assert_array_equal(np.load(tmp_path / "infer_0.npy"), np.load(tmp_path / "infer_1.npy"))
    assert np.linalg.norm(p0 - st.params) <= 1e-5 * np.linalg.norm(st.params)
    np.testing.assert_allclose(np.load(tmp_path / "loss_0.npy"), ref_losses, rtol=1e-5)


def test_dp_step_equals_single_process_step_hash(tmp_path):
    """InputEncoding::Hash: the exchanged buffer carries the grid-table gradient too (NRC_HASH_GRAD_FLOATS); the
    sparse grid Adam steps the entries whose summed gradient is non-zero, as the single-process step does."""
    import torch.multiprocessing as mp

    world, B, steps = 2, 256, 2
    mp.spawn(_worker, args=(world, _free_port(), B, steps, str(tmp_path), True), nprocs=world, join=True)
    orc = nrc_loader.load_oracle()
    nrc = nrc_loader.load()
    assert nrc.HASH_GRAD_FLOATS == orc.HASH_NUM_PARAMS + 4
    st = orc.HashAdamEmaState(_init_params(orc, True))
    ref_losses = []
    for it in range(steps):
        q, t = nrc.synthetic.cornell_batch(B, seed=40 + it)
        g, loss = orc.hash_grad(st.params, q, t, mode=orc.FP32, threads=2)
        st.apply(g)
        ref_losses.append(loss)
    p0, p1 = np.load(tmp_path / "params_0.npy"), np.load(tmp_path / "params_1.npy")
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(np.load(tmp_path / "infer_0.npy"), np.load(tmp_path / "infer_1.npy"))
    M = orc.HASH_MLP_PARAMS
    assert np.linalg.norm(p0[:M] - st.params[:M]) <= 1e-4 * np.linalg.norm(st.params[:M])
    moved, moved_ref = p0[M:] != _init_params(orc, True)[M:], st.params[M:] != _init_params(orc, True)[M:]
    assert moved_ref.sum() > 1000 and np.mean(moved == moved_ref) >= 0.9999
    np.testing.assert_allclose(np.load(tmp_path / "loss_0.npy"), ref_losses, rtol=1e-5)
