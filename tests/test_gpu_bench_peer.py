"""bench.py's N > 1 training path (round 6): open_peer_training opens the library's peer exchange on every rank and runs
one frame through it, falling back to the RCCL communicator when any rank fails. Exercised at world 1 on one GPU (a
world-1 gloo process group for the agreement, a world-1 RCCL communicator as the fallback): the success path leaves
the exchange open and nrc_train_dp on it bitwise equal to the RCCL step; a failing warm frame leaves it closed and the
RCCL path working."""
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist

    mine = not dist.is_initialized()
    if mine:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    yield dist
    if mine:
        dist.destroy_process_group()


def test_open_peer_training_success_and_fallback(nrc, dev, golden, pg):
    import torch

    sys.path.insert(0, str(ROOT))
    import bench

    B = nrc.BATCH_SIZE
    qb, tb = nrc.synthetic.cornell_batch(B, seed=91)
    q, t = torch.from_numpy(qb).to(dev), torch.from_numpy(tb).to(dev)
    nets = []
    for _ in range(2):
        n = nrc.Network()
        n.init(stream=torch.cuda.current_stream())
        n.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
        n.set_state(nrc.StateSlot.INFER, golden["params_b"])
        n.set_comm(nrc.Communicator(nrc.Communicator.unique_id(), 1, 0))
        nets.append(n)
    try:
        a, r = nets
        assert bench.open_peer_training(nrc, a, dev, lambda: a.train_dp(q, t, B, B))
        r.train_dp(q, t, B, B)  # the RCCL path, same step
        a.train_dp(q, t, B, B)  # through the exchange (still open)
        r.train_dp(q, t, B, B)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.get_state(nrc.StateSlot.PARAMS), r.get_state(nrc.StateSlot.PARAMS))
        a.peer_exchange_close()

        def boom():
            raise RuntimeError("injected")

        assert not bench.open_peer_training(nrc, r, dev, boom)
        assert "injected" in r._peer_training_error
        r.train_dp(q, t, B, B)  # the exchange is closed again: the RCCL communicator serves the step
        torch.cuda.synchronize()
    finally:
        for n in nets:
            n.set_comm(None)
            n.destroy()
