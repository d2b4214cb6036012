"""Round 6: the width-64 Frequency training step in one launch (launch_train16_fused, nrc_train16.hip) against the
two-launch step (train16_split_kernel + reduce_adam_kernel in mode kReduceFused), the default: the fused step is an
opt-in A/B (knob train_fused = 1 at nrc_init), slower on MI355X, kept tested. Same float operations in the same order, so every state slot, the loss and the f16 weight images must be
bitwise equal -- after several steps (the reducers' counters are reset by the last reducer of each launch, so a stale
count would show as a wrong step), on ragged batches (the last block's padding samples), on padded records, when the
steps are replayed from a HIP graph (no host-side generation baked into the capture), and interleaved with inference
(the inference image the reducers pack is the one `infer` reads). The data-parallel entry points (nrc_train_grad / apply)
keep the two launches and must agree with the fused step as before."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SLOTS = ("PARAMS", "INFER", "EMA", "ADAM_M", "ADAM_V")


@pytest.fixture(scope="module")
def torch():
    import torch as _t

    return _t


def _t(torch, a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _make(nrc, torch, golden, fused: bool, padded=False, stream=None):
    nrc._lib.set_knob("train_fused", 1 if fused else -1)
    try:
        cfg = nrc.default_config(nrc.InputEncoding.Frequency)
        if padded:
            cfg.query_layout = nrc.QUERY_PADDED
        n = nrc.Network()
        n.init(stream=stream or torch.cuda.current_stream(), encoding=nrc.InputEncoding.Frequency, config=cfg)
    finally:
        nrc._lib.set_knob("train_fused", -1)
    if not padded:
        for slot in ("PARAMS", "INFER"):
            n.set_state(getattr(nrc.StateSlot, slot), golden["params_b"])
    return n


def _same_state(nrc, a, b):
    for slot in SLOTS:
        np.testing.assert_array_equal(a.get_state(getattr(nrc.StateSlot, slot)),
                                      b.get_state(getattr(nrc.StateSlot, slot)), err_msg=slot)
    assert a.step == b.step


@pytest.mark.parametrize("b", [16384, 16000, 12345, 129])
def test_fused_step_bitwise_two_launch_step(nrc, torch, dev, golden, b):
    F, T = _make(nrc, torch, golden, True), _make(nrc, torch, golden, False)
    try:
        q = nrc.synthetic.cornell_queries(50_000, seed=61)
        for it in range(5):
            qb, tb = nrc.synthetic.cornell_batch(b, seed=610 + it)
            qd, td = _t(torch, qb, dev), _t(torch, tb, dev)
            lf = F.train_batch(qd, td, b, loss=True)
            lt = T.train_batch(qd, td, b, loss=True)
            assert lf == lt, (it, lf, lt)
            if it == 2:  # inference between steps reads the image the reducers packed
                outs = []
                for n in (F, T):
                    o = torch.empty((len(q), 3), device=dev)
                    n.infer(_t(torch, q, dev), o, len(q))
                    outs.append(o.cpu().numpy())
                np.testing.assert_array_equal(outs[0], outs[1])
        _same_state(nrc, F, T)
    finally:
        F.destroy()
        T.destroy()


def test_fused_step_padded_records(nrc, torch, dev, golden):
    from test_gpu_padded import padded
    F, T = _make(nrc, torch, golden, True, True), _make(nrc, torch, golden, False, True)
    try:
        for it in range(3):
            q15, tb = nrc.synthetic.cornell_batch(16384, seed=620 + it)
            qd, td = _t(torch, padded(q15, 0.25 * it), dev), _t(torch, tb, dev)
            assert F.train_batch(qd, td, 16384, loss=True) == T.train_batch(qd, td, 16384, loss=True)
        _same_state(nrc, F, T)
    finally:
        F.destroy()
        T.destroy()


def test_fused_step_graph_replay(nrc, torch, dev, golden):
    """12 steps captured in a HIP graph and replayed 3 times against 3 x 12 eager two-launch steps. A captured call
    bakes its optimizer step number into the graph, so the eager handle rewinds its step counter before each 12."""
    cs = torch.cuda.Stream()
    F = _make(nrc, torch, golden, True, stream=cs)
    T = _make(nrc, torch, golden, False)
    B = nrc.BATCH_SIZE
    try:
        qb, tb = nrc.synthetic.cornell_batch(4 * B, seed=630)
        qd, td = _t(torch, qb, dev), _t(torch, tb, dev)
        for n in (F, T):  # one eager step first: the slabs are allocated outside the capture
            n.train(qd, td)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cs):
            for i in range(12):
                F.train(qd[(i % 4) * B:], td[(i % 4) * B:])
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        for _ in range(3):
            T.step = 1
            for i in range(12):
                T.train(qd[(i % 4) * B:], td[(i % 4) * B:])
        torch.cuda.synchronize()
        assert F.step == T.step == 13
        _same_state(nrc, F, T)
        del g
    finally:
        F.destroy()
        T.destroy()


def test_fused_step_and_data_parallel_entries_agree(nrc, torch, dev, golden):
    """nrc_train (one launch) == nrc_train_grad + nrc_train_apply (the kReduceOnly / kApplyOnly launches), bitwise."""
    F, G = _make(nrc, torch, golden, True), _make(nrc, torch, golden, True)
    try:
        grad = torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev)
        for it in range(3):
            qb, tb = nrc.synthetic.cornell_batch(16384, seed=640 + it)
            qd, td = _t(torch, qb, dev), _t(torch, tb, dev)
            lf = F.train_batch(qd, td, 16384, loss=True)
            G.train_grad(qd, td, 16384, 16384, grad)
            lg = G.train_apply(grad, loss=True)
            assert lf == lg
        _same_state(nrc, F, G)
    finally:
        F.destroy()
        G.destroy()
