"""Data parallelism on the GPU path.

* In-library RCCL (nrc_set_comm + nrc_train_dp): with a world-1 communicator the step is bitwise the fused
  nrc_train step (the all-reduce of one rank is the identity); the frame driver's shard entry with a world-1
  communicator reproduces nrc_process_frame bitwise.
* Two ranks on one GPU over gloo (torch.distributed) with the real HIP nrc_train_grad / nrc_train_apply: the
  replicas stay bit-identical, and after the steps they match the single-process nrc_train on the concatenated
  16,384-sample minibatches to the gradient's summation-order tolerance. (RCCL itself cannot put two ranks on one
  device; the multi-GPU RCCL path is the driver's 8-GPU bench, rehearsed here with the same code over gloo.)
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def torch():
    import torch as _t

    return _t


def to_dev(torch, dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("encoding", ["Frequency", "Hash"])
def test_world1_rccl_step_is_bitwise_nrc_train(nrc, torch, dev, golden, encoding):
    """Hash: nrc_train_dp runs the exact grid exchange (int64 sums in the exchange encoding, one RCCL group with the
    f32 MLP gradient), which at world 1 must reproduce the fused step's grid update bit for bit."""
    comm = nrc.Communicator(nrc.Communicator.unique_id(), 1, 0)
    nets = []
    for _ in range(2):
        n = nrc.Network()
        n.init(stream=torch.cuda.current_stream(), encoding=getattr(nrc.InputEncoding, encoding))
        if encoding == "Frequency":
            n.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
        nets.append(n)
    nets[1].set_comm(comm)
    assert nets[1].comm_rank() == (0, 1)
    losses = [[], []]
    for it in range(3):
        q_np, t_np = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=60 + it)
        q, t = to_dev(torch, dev, q_np), to_dev(torch, dev, t_np)
        losses[0].append(nets[0].train(q, t, loss=True))
        losses[1].append(nets[1].train_dp(q, t, nrc.BATCH_SIZE, nrc.BATCH_SIZE, loss=True))
    assert losses[0] == losses[1]
    for slot in nrc.StateSlot:
        np.testing.assert_array_equal(nets[0].get_state(slot), nets[1].get_state(slot))
    assert nets[0].step == nets[1].step == 3
    with pytest.raises(nrc.NrcError):
        nets[0].train_dp(q, t, nrc.BATCH_SIZE, nrc.BATCH_SIZE)  # no communicator attached
    for n in nets:
        n.destroy()
    comm.destroy()


def test_world1_rccl_frame_shard_is_bitwise_process_frame(nrc, torch, dev):
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(160, 96, (8, 8), seed=3)
    cap = F.NUM_TRAINING_RECORDS_PER_FRAME
    nrec = min(f.num_training_records, cap)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    pad = lambda a, w: np.concatenate([a[:nrec], np.zeros((cap - nrec, w), np.float32)])  # noqa: E731
    rec = np.zeros(cap, F.TRAINING_RECORD_DTYPE)
    rec[:nrec] = f.train_records[:nrec]
    S, T = f.screen_size, f.num_tiles

    def buffers():
        return F.FrameBuffers(t(f.queries_inference), torch.zeros((S + T, 3), device=dev), t(f.last_render_throughput),
                              torch.zeros((S, 4), device=dev), F.records_to_device(f.end_vertices, dev),
                              F.records_to_device(rec, dev), [t(pad(f.train_queries, 15)), torch.zeros((cap, 15), device=dev)],
                              [t(pad(f.train_targets, 3)), torch.zeros((cap, 3), device=dev)])

    comm = nrc.Communicator(nrc.Communicator.unique_id(), 1, 0)
    outs = []
    for use_dp in (False, True):
        net = nrc.Network()
        net.init(stream=torch.cuda.current_stream())
        fb = buffers()
        if use_dp:
            net.set_comm(comm)
        losses = []
        for it in range(2):
            fp = F.FrameParams(S, T, f.num_training_records, F.RenderMode.Full, it, it, 1)
            losses.append(F.process_frame_shard(net, fb, fp, 0, S) if use_dp else F.process_frame(net, fb, fp))
        torch.cuda.synchronize()
        outs.append((losses, fb.output_rgba.cpu().numpy(), net.get_state(nrc.StateSlot.PARAMS)))
        net.destroy()
    comm.destroy()
    assert outs[0][0] == outs[1][0]
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    np.testing.assert_array_equal(outs[0][2], outs[1][2])


def test_frame_pixel_shards_cover_the_frame(nrc, torch, dev):
    """nrc_process_frame_shard without a communicator: two replicas rendering [0, S/2) and [S/2, S) write exactly
    their halves of the frame buffer, and together equal the whole-frame nrc_process_frame; every replica infers all
    train-suffix ends, so their training (full minibatches here) is identical."""
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(160, 96, (8, 8), seed=6)
    cap = F.NUM_TRAINING_RECORDS_PER_FRAME
    nrec = min(f.num_training_records, cap)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    pad = lambda a, w: np.concatenate([a[:nrec], np.zeros((cap - nrec, w), np.float32)])  # noqa: E731
    rec = np.zeros(cap, F.TRAINING_RECORD_DTYPE)
    rec[:nrec] = f.train_records[:nrec]
    S, T = f.screen_size, f.num_tiles
    res = []
    for rng in [(0, S), (0, S // 2 + 7), (S // 2 + 7, S)]:
        net = nrc.Network()
        net.init(stream=torch.cuda.current_stream())
        fb = F.FrameBuffers(t(f.queries_inference), torch.zeros((S + T, 3), device=dev), t(f.last_render_throughput),
                            torch.full((S, 4), -1.0, device=dev), F.records_to_device(f.end_vertices, dev),
                            F.records_to_device(rec, dev), [t(pad(f.train_queries, 15)), torch.zeros((cap, 15), device=dev)],
                            [t(pad(f.train_targets, 3)), torch.zeros((cap, 3), device=dev)])
        fp = F.FrameParams(S, T, f.num_training_records, F.RenderMode.Full, 0, 0, 1)
        loss = F.process_frame(net, fb, fp) if rng == (0, S) else F.process_frame_shard(net, fb, fp, *rng)
        torch.cuda.synchronize()
        res.append((rng, loss, fb.output_rgba.cpu().numpy(), net.get_state(nrc.StateSlot.PARAMS)))
        net.destroy()
    full = res[0][2]
    for rng, loss, out, params in res[1:]:
        a, b = rng
        np.testing.assert_array_equal(out[a:b], full[a:b])
        assert (np.delete(out, np.arange(a, b), axis=0) == -1.0).all()
        assert loss == res[0][1]
        np.testing.assert_array_equal(params, res[0][3])


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("B", [16384, 4096])
def test_two_ranks_on_one_gpu_gloo(tmp_path, nrc, torch, dev, golden, B):
    """tools/dp_rank_worker.py x 2 (gloo, both on cuda:0): bit-identical replicas, equal to the single-process step
    on the full minibatches within the summation-order tolerance. B = 4,096: each rank trains configs[3]'s per-rank
    slice of 2,048 samples (the small-block shape of the decoupled-chain kernel)."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    np.save(tmp_path / "params.npy", golden["params_b"])
    procs = [subprocess.Popen([sys.executable, str(ROOT / "tools" / "dp_rank_worker.py"), str(tmp_path), str(B)],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    logs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), logs
    steps = 3
    ref = nrc.Network()
    ref.init(stream=torch.cuda.current_stream())
    ref.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
    ref_losses = []
    for it in range(steps):
        q_np, t_np = nrc.synthetic.cornell_batch(B, seed=80 + it)
        ref_losses.append(ref.train_batch(to_dev(torch, dev, q_np), to_dev(torch, dev, t_np), B, loss=True))
    for slot in ("params", "infer"):
        a, b = np.load(tmp_path / f"{slot}_0.npy"), np.load(tmp_path / f"{slot}_1.npy")
        np.testing.assert_array_equal(a, b)
    p = np.load(tmp_path / "params_0.npy")
    r = ref.get_state(nrc.StateSlot.PARAMS)
    assert np.linalg.norm(p - r) <= 1e-4 * np.linalg.norm(r)
    np.testing.assert_allclose(np.load(tmp_path / "loss_0.npy"), ref_losses, rtol=1e-5)
    ref.destroy()


def test_two_ranks_on_one_gpu_gloo_hash_exact(tmp_path, nrc, torch, dev):
    """Hash over gloo with the exact grid exchange (int64 all-reduce of the exchange-encoded fixed-point sums): the
    replicas are bit-identical and their grid update is bitwise the single-process step over the whole minibatch (the
    MLP part: summation-order tolerance). One step: afterwards the MLP weights differ by f32 rounding, and so would
    the next step's grid gradient."""
    B = 16384
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(ROOT / "tools" / "dp_rank_worker.py"), str(tmp_path), str(B), "Hash",
                               "1"], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    logs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), logs
    ref = nrc.Network()
    ref.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash)
    p0 = ref.get_state(nrc.StateSlot.PARAMS)
    q_np, t_np = nrc.synthetic.cornell_batch(B, seed=80)
    ref_loss = ref.train_batch(to_dev(torch, dev, q_np), to_dev(torch, dev, t_np), B, loss=True)
    for slot in ("params", "infer"):
        np.testing.assert_array_equal(np.load(tmp_path / f"{slot}_0.npy"), np.load(tmp_path / f"{slot}_1.npy"))
    M = nrc.HASH_MLP_PARAMS
    p, r = np.load(tmp_path / "params_0.npy"), ref.get_state(nrc.StateSlot.PARAMS)
    assert (r[M:] != p0[M:]).sum() > 10_000
    np.testing.assert_array_equal(p[M:], r[M:])
    assert np.linalg.norm(p[:M] - r[:M]) <= 3e-3 * np.linalg.norm(r[:M])
    np.testing.assert_allclose(np.load(tmp_path / "loss_0.npy"), [ref_loss], rtol=1e-5)
    ref.destroy()


@pytest.mark.parametrize("B,path", [(16384, "peer"), (4096, "peer"), (4096, "peer_push")])
def test_two_ranks_on_one_gpu_peer_exchange(tmp_path, nrc, torch, dev, golden, B, path):
    """The one-shot peer exchange (nrc_peer_exchange_*): two processes on cuda:0, IPC handles
    all-gathered over gloo, nrc_train_dp pushing each rank's gradient into the other's receive buffer and summing in
    rank order -- "peer": the production choice, which for ranks sharing a device is the split form of the exchange
    fused into the reduction (reduce + push, then wait + sum + Adam; the fused single launch is exercised by the world-1
    test below), "peer_push": round 4's first version (reduce / push / apply launches).
    Replicas bit-identical, and bitwise the single-process step that sums the two shards' gradients
    (g0 + g1, one f32 addition -- also what a 2-rank RCCL all-reduce computes) and applies them with nrc_train_apply."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    np.save(tmp_path / "params.npy", golden["params_b"])
    steps = 3
    procs = [subprocess.Popen([sys.executable, str(ROOT / "tools" / "dp_rank_worker.py"), str(tmp_path), str(B),
                               "Frequency", str(steps), path], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    logs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), logs
    ref = nrc.Network()
    ref.init(stream=torch.cuda.current_stream())
    ref.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
    g = [torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev) for _ in range(2)]
    ref_losses = []
    for it in range(steps):
        q_np, t_np = nrc.synthetic.cornell_batch(B, seed=80 + it)
        for r in range(2):
            s, c = nrc.dp.shard_range(B, r, 2)
            ref.train_grad(to_dev(torch, dev, q_np[s:s + c]), to_dev(torch, dev, t_np[s:s + c]), c, B, g[r])
        ref_losses.append(ref.train_apply(g[0] + g[1], loss=True))
    for slot in ("params", "infer"):
        a, b = np.load(tmp_path / f"{slot}_0.npy"), np.load(tmp_path / f"{slot}_1.npy")
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(a, ref.get_state(getattr(nrc.StateSlot, slot.upper())))
    np.testing.assert_array_equal(np.load(tmp_path / "loss_0.npy"), np.array(ref_losses, np.float32))
    ref.destroy()


@pytest.mark.parametrize("B", [16384, 2048, 0])
def test_peer_exchange_world_1_is_the_fused_step(nrc, torch, dev, golden, B):
    """A world-1 peer exchange (what bench.py's per-rank leg runs): nrc_train_dp through the fused reduce + exchange
    launch keeps its own partials in registers -- at world 1 it stores nothing and skips the wait loop, so this covers
    the reduce + sum + Adam half only (the stores and the wait at world >= 2: the sequenced test below) -- and must be
    bitwise the state and loss of nrc_train's reduce + Adam (the same slab sums, a sum over one rank is the value).
    B = 0: a rank without samples takes part with a zero gradient (loss 0; Adam's l2 term still steps the weights)."""
    a, b = nrc.Network(), nrc.Network()
    for n in (a, b):
        n.init(stream=torch.cuda.current_stream())
        n.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
    h = a.peer_exchange_handle(1)
    a.peer_exchange_open(0, 1, h)
    zero_g = torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev)
    for it in range(3):
        q_np, t_np = nrc.synthetic.cornell_batch(max(B, 1), seed=90 + it)
        q, t = to_dev(torch, dev, q_np), to_dev(torch, dev, t_np)
        la = a.train_dp(q, t, B, max(B, 1), loss=True)
        lb = b.train_batch(q, t, B, loss=True) if B else b.train_apply(zero_g, loss=True)
        assert la == lb
    for slot in ("PARAMS", "INFER", "EMA", "ADAM_M", "ADAM_V"):
        np.testing.assert_array_equal(a.get_state(getattr(nrc.StateSlot, slot)), b.get_state(getattr(nrc.StateSlot, slot)))
    a.peer_exchange_close()
    a.destroy()
    b.destroy()


def test_peer_exchange_argument_checks(nrc, torch, dev):
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    with pytest.raises(nrc.NrcError):
        net.peer_exchange_handle(0)  # world >= 1
    with pytest.raises(nrc.NrcError):
        net.peer_exchange_open(0, 2, bytes(128))  # no buffer allocated yet
    h = net.peer_exchange_handle(2)
    assert len(h) == 64
    with pytest.raises(nrc.NrcError):
        net.peer_exchange_open(0, 3, bytes(192))  # world differs from the allocation
    net.peer_exchange_close()
    net.destroy()
    hnet = nrc.Network()
    hnet.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash)
    with pytest.raises(nrc.NrcError) as e:
        hnet.peer_exchange_handle(2)
    assert e.value.status == 5
    hnet.destroy()


SLOTS = ("PARAMS", "INFER", "EMA", "ADAM_M", "ADAM_V")


@pytest.fixture()
def knobs(nrc):
    yield nrc._lib.set_knob
    for k in ("peer_path", "px_polls"):
        nrc._lib.set_knob(k, -1)


@pytest.mark.parametrize("world,B", [(2, 16384), (4, 16384), (8, 16384), (8, 4096)])
def test_sequenced_fused_peer_exchange(nrc, torch, dev, golden, knobs, world, B):
    """the fused exchange at world >= 2 -- its stores into every peer's buffer and its wait loop
    (reduce_exchange_kernel<..., WAIT=true>, what every rank runs with one rank per GPU) -- executed in one process
    without co-residency: world handles on one GPU joined by nrc_peer_exchange_open_local (plain device pointers, no
    IPC); per step ranks 1..N-1 run the split form's gradient pass + push alone (knob peer_path 3), then rank 0 runs
    the fused kernel (peer_path 1; every word it awaits is already in its buffer), then ranks 1..N-1 run the split form's
    wait + sum + Adam alone (peer_path 4; rank 0's words have arrived). Every handle's five state slots and loss must be
    bitwise those of one handle applying the rank-order sum g0 + g1 + ... of the shards' gradients (nrc_train_grad)
    with nrc_train_apply. Three steps: both buffer parities; at world 8 the sequence number starts at 0xFFFFFFFE, so the
    steps carry tags 0xFFFFFFFF, 2, 3 (the wrap keeps the parity alternating). On step 2 rank 1 first makes a rejected
    call (global_b < b_local), which must not advance its sequence. A slip ends a wait with
    NRC_ERR_INTERNAL after px_polls polls instead of hanging."""
    knobs("px_polls", 1 << 14)
    nets = []
    for _ in range(world):
        n = nrc.Network()
        n.init(stream=torch.cuda.current_stream())
        n.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
        nets.append(n)
    nrc.Network.peer_exchange_open_local(nets)
    if world == 8:
        for n in nets:
            n.set_peer_seq(0xFFFFFFFE)
    ref = nrc.Network()
    ref.init(stream=torch.cuda.current_stream())
    ref.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
    g = [torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev) for _ in range(world)]
    try:
        for it in range(3):
            q_np, t_np = nrc.synthetic.cornell_batch(B, seed=300 + it)
            q, t = to_dev(torch, dev, q_np), to_dev(torch, dev, t_np)
            sh = [nrc.dp.shard_range(B, r, world) for r in range(world)]
            knobs("peer_path", 3)
            if it == 1:
                s1, c1 = sh[1]
                with pytest.raises(nrc.NrcError) as e:
                    nets[1].train_dp(q[s1:s1 + c1], t[s1:s1 + c1], c1, c1 - 1)
                assert e.value.status == 1
            for r in range(1, world):
                s, c = sh[r]
                nets[r].train_dp(q[s:s + c], t[s:s + c], c, B)
            knobs("peer_path", 1)
            s, c = sh[0]
            losses = [nets[0].train_dp(q[s:s + c], t[s:s + c], c, B, loss=True)]
            knobs("peer_path", 4)
            for r in range(1, world):
                losses.append(nets[r].train_dp(None, None, 0, B, loss=True))
            for r in range(world):
                s, c = sh[r]
                ref.train_grad(q[s:s + c], t[s:s + c], c, B, g[r])
            gs = g[0]
            for r in range(1, world):
                gs = gs + g[r]
            ref_loss = ref.train_apply(gs, loss=True)
            assert losses == [ref_loss] * world, (it, losses, ref_loss)
        for slot in SLOTS:
            want = ref.get_state(getattr(nrc.StateSlot, slot))
            for r in range(world):
                np.testing.assert_array_equal(nets[r].get_state(getattr(nrc.StateSlot, slot)), want, err_msg=f"{slot} rank {r}")
        assert all(n.step == 3 for n in nets)
    finally:
        for n in nets:
            n.peer_exchange_close()
        for n in nets:
            n.destroy()
        ref.destroy()


def test_fused_peer_exchange_missing_peer_times_out(nrc, torch, dev, golden, knobs):
    """VERDICT r04 item 1, negative case: rank 0 of a world-2 exchange runs the fused kernel while rank 1 never pushes.
    With the wait bounded to 2^13 polls (knob px_polls) the step must end with NRC_ERR_INTERNAL (the sticky protocol
    error) within seconds, not hang; the handle stays poisoned until nrc_init, and the peer is unaffected."""
    import time

    knobs("px_polls", 1 << 13)
    knobs("peer_path", 1)
    a, b = nrc.Network(), nrc.Network()
    for n in (a, b):
        n.init(stream=torch.cuda.current_stream())
        n.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
    nrc.Network.peer_exchange_open_local([a, b])
    q_np, t_np = nrc.synthetic.cornell_batch(4096, seed=5)
    q, t = to_dev(torch, dev, q_np), to_dev(torch, dev, t_np)
    try:
        t0 = time.perf_counter()
        with pytest.raises(nrc.NrcError) as e:
            a.train_dp(q[:2048], t[:2048], 2048, 4096, loss=True)
        dt = time.perf_counter() - t0
        assert e.value.status == 7 and "peer" in str(e.value), str(e.value)
        assert dt < 5.0, dt
        with pytest.raises(nrc.NrcError) as e:
            a.train_dp(q[:2048], t[:2048], 2048, 4096)
        assert e.value.status == 7
        knobs("peer_path", -1)
        b_state = b.get_state(nrc.StateSlot.PARAMS)
        np.testing.assert_array_equal(b_state, golden["params_b"])
    finally:
        for n in (a, b):
            n.peer_exchange_close()
        for n in (a, b):
            n.destroy()


def test_peer_exchange_local_argument_checks(nrc, torch, dev, knobs):
    nets = [nrc.Network() for _ in range(2)]
    for n in nets:
        n.init(stream=torch.cuda.current_stream())
    h = nrc.Network()
    h.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash)
    try:
        with pytest.raises(nrc.NrcError) as e:
            nrc.Network.peer_exchange_open_local([nets[0], h])
        assert e.value.status == 5
        with pytest.raises(nrc.NrcError):
            nrc.Network.peer_exchange_open_local([nets[0], nets[0]])
        with pytest.raises(nrc.NrcError):
            nets[0].set_peer_seq(5)  # no exchange open
        nrc.Network.peer_exchange_open_local(nets)
        with pytest.raises(nrc.NrcError):
            nets[0].set_peer_seq(0)
        knobs("peer_path", 4)
        with pytest.raises(nrc.NrcError) as e:  # nothing pushed yet
            nets[1].train_dp(None, None, 0, 16)
        assert e.value.status == 1
        for k, v in (("peer_path", 5), ("px_polls", 0), ("px_polls", (1 << 21) + 1)):
            with pytest.raises(nrc.NrcError):
                knobs(k, v)
    finally:
        for n in nets:
            n.peer_exchange_close()
        for n in nets + [h]:
            n.destroy()


def test_peer_exchange_local_group_closes_together(nrc, torch, dev, golden, knobs):
    """the handles of an in-process exchange hold raw pointers to each other's receive buffers, so closing,
    destroying or re-opening any member closes the exchange of every member (after their streams drain) instead of
    freeing one buffer under the others. Then one host thread drives two ranks round-robin with nrc_train_dp_async
    (each rank on its own stream, as two handles on one device need): no blocking loss inside the round, losses read
    after it, replicas bitwise the rank-order sum applied by one handle."""
    knobs("px_polls", 1 << 14)  # a handle left open by mistake ends its wait with an error instead of ~10 s
    nets = []
    for _ in range(4):
        n = nrc.Network()
        n.init(stream=torch.cuda.Stream())
        n.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
        nets.append(n)
    a, b, c, d = nets
    q_np, t_np = nrc.synthetic.cornell_batch(4096, seed=17)
    q, t = to_dev(torch, dev, q_np), to_dev(torch, dev, t_np)

    def closed(n):
        with pytest.raises(nrc.NrcError) as e:
            n.train_dp(q[:16], t[:16], 16, 32)
        return e.value.status == 1

    ref = nrc.Network()
    ref.init(stream=torch.cuda.current_stream())
    ref.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
    try:
        nrc.Network.peer_exchange_open_local([a, b, c])
        b.peer_exchange_close()
        assert closed(a) and closed(b) and closed(c)
        nrc.Network.peer_exchange_open_local([a, b, c])
        c.destroy()
        assert closed(a) and closed(b)
        nrc.Network.peer_exchange_open_local([a, b])
        nrc.Network.peer_exchange_open_local([b, d])  # takes b: a's group is closed, not left pointing at b's buffer
        assert closed(a)
        nrc.Network.peer_exchange_open_local([a, b])  # d's group closed in turn
        assert closed(d)
        losses = [torch.full((1,), float("nan"), device=dev) for _ in range(2)]
        g = [torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev) for _ in range(2)]
        for it in range(3):
            for r, n in enumerate((a, b)):  # one thread, round-robin, nothing blocks
                s, k = nrc.dp.shard_range(4096, r, 2)
                n.train_dp_async(q[s:s + k], t[s:s + k], k, 4096, losses[r])
            for r in range(2):
                s, k = nrc.dp.shard_range(4096, r, 2)
                ref.train_grad(q[s:s + k], t[s:s + k], k, 4096, g[r])
            ref_loss = ref.train_apply(g[0] + g[1], loss=True)
            torch.cuda.synchronize()
            assert [float(x.item()) for x in losses] == [ref_loss, ref_loss], it
        for slot in SLOTS:
            want = ref.get_state(getattr(nrc.StateSlot, slot))
            for n in (a, b):
                np.testing.assert_array_equal(n.get_state(getattr(nrc.StateSlot, slot)), want, err_msg=slot)
    finally:
        for n in (a, b, d):
            n.peer_exchange_close()
        for n in (a, b, d, ref):
            n.destroy()
