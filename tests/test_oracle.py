"""CPU tests of the oracle (oracle/nrc_oracle.c) against an independent float64 numpy restatement,
torch autograd, finite differences and the committed golden vectors. No GPU.

Parity with tiny-cuda-nn itself is UNPINNED (tcnn absent, no reference fixtures): see DESIGN.md.
"""
import numpy as np
import pytest

import nrc_loader

onp = None


def _onp():
    global onp
    if onp is None:
        nrc_loader.load_oracle()
        import oracle_np

        onp = oracle_np
    return onp


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def test_f16_round_matches_numpy(orc):
    rng = np.random.default_rng(0)
    vals = np.concatenate([
        rng.normal(0, 1, 2000), rng.normal(0, 1e-5, 500), rng.normal(0, 1e4, 500),
        [0.0, -0.0, 65504.0, 65519.99, 65520.0, 1e-8, 2.0**-24, 2.0**-25, 3 * 2.0**-26, 6.1e-5, np.inf, -np.inf],
    ]).astype(np.float32)
    ours = np.array([orc.f16_round(float(v)) for v in vals], dtype=np.float32)
    ref = vals.astype(np.float16).astype(np.float32)
    np.testing.assert_array_equal(ours, ref)


def test_encode_matches_numpy(nrc, orc):
    q = nrc.synthetic.cornell_queries(3000, seed=11)
    np.testing.assert_allclose(orc.encode(q), _onp().encode(q), rtol=0, atol=2e-6)


def test_oneblob_properties(orc):
    # bins of every OneBlob dimension sum to 1 for any input, including the raw angles the reference
    # feeds (theta in [0, pi], phi in (-pi, pi]) that lie outside [0, 1]
    xs = np.linspace(-4.0, 4.0, 4001, dtype=np.float32)
    q = np.zeros((xs.size, 15), np.float32)
    q[:, 3:9] = xs[:, None]
    e = orc.encode(q)
    blob = e[:, 36:60].reshape(-1, 6, 4)
    np.testing.assert_allclose(blob.sum(-1), 1.0, atol=3e-6)
    assert (blob >= -1e-6).all()
    # far outside [0, 1] (x < -1.25 or x >= 2) the period-1 wrap of the formula dumps all mass into the last bin
    far = (xs < -1.26) | (xs > 2.0)
    np.testing.assert_allclose(blob[far, :, 3], 1.0, atol=1e-6)
    # inside the unit interval a blob is a smooth bump with its peak in the bin containing x
    x = 0.6
    e1 = orc.encode(np.array([[0, 0, 0, x, x, x, x, x, x, 0, 0, 0, 0, 0, 0]], np.float32))[0, 36:40]
    assert np.argmax(e1) == 2


def test_triangle_wave_spec(orc):
    q = np.zeros((5, 15), np.float32)
    q[:, 0] = [0.0, 0.25, 0.5, 0.75, 0.125]
    e = orc.encode(q)
    np.testing.assert_allclose(e[:, 0], [1.0, 0.5, 0.0, 0.5, 0.75], atol=1e-7)  # |2 frac(x) - 1|
    np.testing.assert_allclose(e[:, 1], [1.0, 0.0, 1.0, 0.0, 0.5], atol=1e-7)  # octave 1
    assert (e[:, 66:80] == 1.0).all()


def test_forward_fp32_matches_numpy(nrc, orc):
    q = nrc.synthetic.cornell_queries(2000, seed=12)
    p = orc.init_params(1337) * np.float32(1.5)
    y, _ = _onp().forward(p, q)
    assert rel(orc.forward(p, q, orc.FP32), y[:, :3]) < 1e-6


@pytest.mark.parametrize("threads", [1, 3])
def test_grad_fp32_matches_numpy(nrc, orc, threads):
    q, t = nrc.synthetic.cornell_batch(512, seed=13)
    p = orc.init_params(1337) * np.float32(1.5)
    g, loss = orc.grad(p, q, t, mode=orc.FP32, threads=threads)
    loss_np, g_np = _onp().loss_and_grad(p, q, t)
    assert abs(loss - loss_np) <= 1e-6 * abs(loss_np)
    assert rel(g, g_np) < 1e-6


def test_grad_matches_torch_autograd(nrc, orc):
    torch = pytest.importorskip("torch")
    q, t = nrc.synthetic.cornell_batch(256, seed=14)
    p = orc.init_params(1337) * np.float32(1.5)
    enc = torch.from_numpy(_onp().encode(q))
    Ws, off = [], 0
    for o, i in _onp().LAYER_SHAPES:
        Ws.append(torch.tensor(p[off:off + o * i].astype(np.float64).reshape(o, i), requires_grad=True))
        off += o * i
    a = enc
    for l in range(5):
        a = torch.relu(a @ Ws[l].T)
    y = torch.relu(a @ Ws[5].T)[:, :3]
    tt = torch.from_numpy(t.astype(np.float64))
    lum = (0.299 * y[:, 0] + 0.587 * y[:, 1] + 0.114 * y[:, 2]).detach()  # denominator not differentiated
    L = ((y - tt) ** 2 / (lum * lum + 0.01)[:, None]).sum() / (3 * q.shape[0])
    L.backward()
    g_t = np.concatenate([w.grad.numpy().reshape(-1) for w in Ws]) * 128.0
    g, loss = orc.grad(p, q, t, mode=orc.FP32)
    assert abs(loss - L.item()) <= 1e-6 * L.item()
    assert rel(g, g_t) < 1e-6


def test_grad_finite_differences(nrc):
    q, t = nrc.synthetic.cornell_batch(64, seed=15)
    p = (nrc_loader.load_oracle().init_params(1337) * np.float32(1.5)).astype(np.float64)
    loss0, g = _onp().loss_and_grad(p, q, t, loss_scale=1.0)
    rng = np.random.default_rng(0)
    idx = rng.choice(np.flatnonzero(np.abs(g) > 1e-3 * np.abs(g).max()), 12, replace=False)
    for i in idx:
        eps = 1e-6
        pp, pm = p.copy(), p.copy()
        pp[i] += eps
        pm[i] -= eps
        # the reference's loss treats the luminance denominator as a constant: freeze it
        fd = (_frozen_loss(pp, p, q, t) - _frozen_loss(pm, p, q, t)) / (2 * eps)
        assert abs(fd - g[i]) <= 1e-4 * abs(g[i]) + 1e-9, (i, fd, g[i])


def _frozen_loss(p, p_den, q, t):
    y, _ = _onp().forward(p, q)
    yd, _ = _onp().forward(p_den, q)
    lum = 0.299 * yd[:, 0] + 0.587 * yd[:, 1] + 0.114 * yd[:, 2]
    return float(np.sum((y[:, :3] - t) ** 2 / (lum * lum + 0.01)[:, None]) / (3 * q.shape[0]))


def test_mixed_and_tcnn_modes_close_to_fp32(nrc, orc):
    q = nrc.synthetic.cornell_queries(2048, seed=16)
    p = orc.init_params(1337) * np.float32(1.6)
    y32 = orc.forward(p, q, orc.FP32)
    assert rel(orc.forward(p, q, orc.MIXED), y32) < 5e-3
    assert rel(orc.forward(p, q, orc.TCNN), y32) < 1e-2


def test_adam_ema_matches_numpy(orc):
    rng = np.random.default_rng(5)
    p = rng.normal(0, 0.1, orc.NUM_PARAMS).astype(np.float32)
    st = orc.AdamEmaState(p)
    w, m, v, ema = p.astype(np.float64), 0.0, 0.0, 0.0
    for step in range(1, 4):
        g = rng.normal(0, 1.0, orc.NUM_PARAMS).astype(np.float32)
        st.apply(g)
        gg = g / 128.0 + 1e-6 * w
        m = 0.9 * m + 0.1 * gg
        v = 0.999 * v + 0.001 * gg * gg
        lr_t = 1e-3 * np.sqrt(1 - 0.999 ** step) / (1 - 0.9 ** step)
        w = w - lr_t / (np.sqrt(v) + 1e-8) * m
        ema = 0.99 * ema + 0.01 * w
        np.testing.assert_allclose(st.params, w, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(st.infer, ema / (1 - 0.99 ** step), rtol=1e-5, atol=1e-7)
    # first debiased EMA equals the first updated weights
    st2 = orc.AdamEmaState(p)
    st2.apply(rng.normal(0, 1, orc.NUM_PARAMS).astype(np.float32))
    np.testing.assert_allclose(st2.infer, st2.params, rtol=1e-6, atol=1e-9)


def test_golden_vectors_reproduce(nrc, orc, golden):
    g = golden
    np.testing.assert_array_equal(nrc.synthetic.cornell_queries(4096, seed=1), g["queries"])
    np.testing.assert_array_equal(orc.init_params(1337), g["params"])
    np.testing.assert_array_equal(orc.encode(g["queries"][:256]), g["enc"])
    np.testing.assert_array_equal(orc.encode(g["queries_edge"]), g["enc_edge"])
    for name, mode in [("fp32", orc.FP32), ("mixed", orc.MIXED), ("tcnn", orc.TCNN)]:
        np.testing.assert_array_equal(orc.forward(g["params_b"], g["queries"], mode), g[f"y_{name}"])
        gr, loss = orc.grad(g["params_b"], g["queries"][:1024], g["targets"], mode=mode)
        assert rel(gr, g[f"grad_{name}"]) < 1e-6
        assert abs(loss - float(g[f"loss_{name}"])) <= 1e-9 * abs(loss)
    st = orc.AdamEmaState(g["params_b"])
    st.apply(g["grad_mixed"])
    np.testing.assert_array_equal(st.params, g["adam1_params"])
    np.testing.assert_array_equal(st.infer, g["adam1_infer"])


def test_synthetic_stream_shapes_and_ranges(nrc):
    q, t = nrc.synthetic.cornell_batch(10000, seed=3)
    assert q.shape == (10000, 15) and q.dtype == np.float32 and q.flags.c_contiguous
    assert q.nbytes == 10000 * 60  # packed 60-byte RadianceQuery rows
    assert np.abs(q[:, 0:3]).max() <= 0.05 + 1e-7
    assert (q[:, 3] >= 0).all() and (q[:, 3] <= np.pi + 1e-6).all()
    assert (np.abs(q[:, 4]) <= np.pi + 1e-6).all()
    assert ((q[:, 7:9] >= 0) & (q[:, 7:9] <= 1)).all()
    assert abs((q[:, 7] == 1.0).mean() - 0.9) < 0.02
    assert (t > 0).all() and t.shape == (10000, 3)
    assert nrc.synthetic.cornell_queries(0).shape == (0, 15)
