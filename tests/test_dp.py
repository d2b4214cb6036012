"""Data-parallel sharding on CPU: torch.distributed gloo, world sizes 2 and 4 (the N > 1 path of bench.py,
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

    # Hash exact exchange (nrc_train_grad_fixed / nrc_train_apply_fixed contract): the grid part travels as int64
    # fixed-point sums (value x 2^24; the stand-in quantises the oracle's f32 gradient), the f32 grid part of grad is
    # not written
    def train_grad_fixed(self, q, t, b, global_b, grad, grid_fixed):
        import torch

        M = self.orc.HASH_MLP_PARAMS
        g, loss = self.orc.hash_grad(self.st.params, q[:b], t[:b], n_total=3.0 * global_b, mode=self.orc.FP32,
                                     threads=2)
        grad[:M] = torch.from_numpy(g[:M])
        grad[g.size] = loss
        grid_fixed[:] = torch.from_numpy(np.rint(g[M:].astype(np.float64) * 2.0 ** 24).astype(np.int64))

    def train_apply_fixed(self, grad, grid_fixed, loss=False):
        M = self.orc.HASH_MLP_PARAMS
        g = np.concatenate([grad[:M].numpy(), (grid_fixed.numpy() / 2.0 ** 24).astype(np.float32)])
        self.st.apply(g.astype(np.float32))
        return float(grad[self.st.params.size]) if loss else None

    # state access with nrc_amd.Network's names (StateSlot order: PARAMS, INFER, EMA, ADAM_M, ADAM_V)
    _SLOTS = ("params", "infer", "ema", "m", "v")

    def get_state(self, slot):
        return getattr(self.st, self._SLOTS[int(slot)]).copy()

    def set_state(self, slot, values):
        setattr(self.st, self._SLOTS[int(slot)], np.array(values, dtype=np.float32))

    @property
    def step(self):
        return self.st.step

    @step.setter
    def step(self, v):
        self.st.step = int(v)


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


def _worker(rank, world, port, B, steps, out_dir, hash_grid=False, fixed=False):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nrc = nrc_loader.load()
    orc = nrc_loader.load_oracle()
    params = _init_params(orc, hash_grid)
    backend = OracleBackend(params, hash_grid)
    grad = torch.full((backend.grad_floats,), 9.0, dtype=torch.float32)  # the grid part must play no role (fixed)
    if fixed:
        grid_fixed = torch.zeros(orc.HASH_GRID_PARAMS, dtype=torch.int64)
        trainer = nrc.dp.DataParallelTrainer(backend, grad, grid_fixed=grid_fixed, mlp_params=orc.HASH_MLP_PARAMS)
    else:
        grad.zero_()
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


@pytest.mark.parametrize("world", [2, 4])
def test_dp_step_equals_single_process_step(tmp_path, world):
    import torch.multiprocessing as mp

    B, steps = 384, 3
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
    p0 = np.load(tmp_path / "params_0.npy")
    for r in range(1, world):  # replicas identical
        np.testing.assert_array_equal(p0, np.load(tmp_path / f"params_{r}.npy"))
        np.testing.assert_array_equal(np.load(tmp_path / "infer_0.npy"), np.load(tmp_path / f"infer_{r}.npy"))
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


def _bcast_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nrc = nrc_loader.load()
    orc = nrc_loader.load_oracle()
    backend = OracleBackend(orc.init_params(1337))
    trainer = nrc.dp.DataParallelTrainer(backend, torch.zeros(backend.grad_floats))
    # the replicas diverge first: different local steps (different moments, EMA and step counters)
    for it in range(rank + 1):
        q, t = nrc.synthetic.cornell_batch(128, seed=70 + 10 * rank + it)
        backend.train_grad(q, t, 128, 128, trainer.grad)
        backend.train_apply(trainer.grad)
    trainer.broadcast_state(backend, "cpu")
    # one more synchronised DP step from the broadcast state
    q, t = nrc.synthetic.cornell_batch(256, seed=99)
    s, c = nrc.dp.shard_range(256, rank, world)
    trainer.step(q[s:s + c], t[s:s + c], c, 256)
    for slot in range(5):
        np.save(os.path.join(out_dir, f"slot{slot}_{rank}.npy"), backend.get_state(slot))
    np.save(os.path.join(out_dir, f"step_{rank}.npy"), np.array([backend.step]))
    dist.destroy_process_group()


def test_broadcast_state_syncs_every_slot_and_the_step(tmp_path):
    """after broadcast_state every replica holds rank 0's weights, EMA, Adam moments and step counter,
    so the next data-parallel step keeps them bit-identical even when they had diverged before."""
    import torch.multiprocessing as mp

    mp.spawn(_bcast_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for slot in range(5):
        np.testing.assert_array_equal(np.load(tmp_path / f"slot{slot}_0.npy"), np.load(tmp_path / f"slot{slot}_1.npy"))
    assert int(np.load(tmp_path / "step_0.npy")[0]) == int(np.load(tmp_path / "step_1.npy")[0]) == 2


def test_dp_trainer_fixed_grid_exchange(tmp_path):
    """DataParallelTrainer with an int64 grid_fixed buffer (the Hash exact exchange): the f32 all-reduce covers the
    MLP gradient and the loss slots only, the grid sums are summed as int64 — the replicas equal a single process
    that sums the two shards' fixed-point grid gradients as integers."""
    import torch.multiprocessing as mp

    world, B, steps = 2, 256, 2
    mp.spawn(_worker, args=(world, _free_port(), B, steps, str(tmp_path), True, True), nprocs=world, join=True)
    orc = nrc_loader.load_oracle()
    nrc = nrc_loader.load()
    M = orc.HASH_MLP_PARAMS
    st = orc.HashAdamEmaState(_init_params(orc, True))
    ref_losses = []
    for it in range(steps):
        q, t = nrc.synthetic.cornell_batch(B, seed=40 + it)
        g_mlp, fixed, loss = np.zeros(M, np.float32), np.zeros(orc.HASH_GRID_PARAMS, np.int64), 0.0
        for r in range(world):
            s, c = nrc.dp.shard_range(B, r, world)
            g, lr = orc.hash_grad(st.params, q[s:s + c], t[s:s + c], n_total=3.0 * B, mode=orc.FP32, threads=2)
            g_mlp += g[:M]
            fixed += np.rint(g[M:].astype(np.float64) * 2.0 ** 24).astype(np.int64)
            loss += lr
        st.apply(np.concatenate([g_mlp, (fixed / 2.0 ** 24).astype(np.float32)]))
        ref_losses.append(loss)
    p0, p1 = np.load(tmp_path / "params_0.npy"), np.load(tmp_path / "params_1.npy")
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(p0[M:], st.params[M:])
    assert np.linalg.norm(p0[:M] - st.params[:M]) <= 1e-5 * np.linalg.norm(st.params[:M])
    np.testing.assert_allclose(np.load(tmp_path / "loss_0.npy"), ref_losses, rtol=1e-5)


def test_dp_trainer_fixed_grid_requires_mlp_params():
    """with grid_fixed but no mlp_params, grad[:None] was the whole buffer (the loss all-reduced twice, the
    unwritten grid part reduced); the trainer now refuses that configuration."""
    import torch

    nrc = nrc_loader.load()
    grad = torch.zeros(nrc.HASH_GRAD_FLOATS)
    fixed = torch.zeros(nrc.HASH_GRID_PARAMS, dtype=torch.int64)
    for bad in (None, 0, nrc.HASH_GRAD_FLOATS):
        with pytest.raises(ValueError):
            nrc.dp.DataParallelTrainer(object(), grad, grid_fixed=fixed, mlp_params=bad)
    t = nrc.dp.DataParallelTrainer(object(), grad, grid_fixed=fixed, mlp_params=nrc.HASH_MLP_PARAMS)
    assert t.mlp_params == nrc.HASH_MLP_PARAMS
