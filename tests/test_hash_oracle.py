"""CPU checks of the InputEncoding::Hash oracle (oracle/nrc_hash_oracle.c) against independent restatements:
a numpy corner/index restatement of tcnn's grid addressing and a float64 torch autograd model of the whole
Hash config (HashGrid + OneBlob + Identity -> 64x5 MLP -> RelativeL2Luminance)."""
import numpy as np
import pytest

P1, P2 = 2654435761, 805459861


def corners_np(q, level):
    """tcnn grid_index / pos_fract / trilinear weights, restated in numpy (f32 where tcnn is f32)."""
    scale = np.float32(16.0 * 2.0 ** level - 1.0)
    res = 16 << level
    x = np.asarray(q[:3], np.float32)
    pos = (np.float64(scale) * x.astype(np.float64) + 0.5).astype(np.float32)  # fmaf(scale, x, 0.5)
    fl = np.floor(pos)
    cell = fl.astype(np.int64) & 0xFFFFFFFF
    fr = (pos - fl).astype(np.float32)
    size = 4096 if level == 0 else 32768
    base = 0 if level == 0 else 4096 + (level - 1) * 32768
    ent, wts = [], []
    for c in range(8):
        bits = [(c >> d) & 1 for d in range(3)]
        w = np.float32(1.0)
        for d in range(3):
            w = np.float32(w * (fr[d] if bits[d] else np.float32(1.0) - fr[d]))
        g = [(int(cell[d]) + bits[d]) & 0xFFFFFFFF for d in range(3)]
        if level <= 1:
            i = (g[0] + g[1] * res + g[2] * res * res) & 0xFFFFFFFF
        else:
            i = (g[0] ^ ((g[1] * P1) & 0xFFFFFFFF) ^ ((g[2] * P2) & 0xFFFFFFFF)) & 0xFFFFFFFF
        ent.append(base + (i & (size - 1)))
        wts.append(w)
    return np.array(ent, np.uint32), np.array(wts, np.float32)


def test_corner_addressing_matches_numpy(nrc, orc):
    q = nrc.synthetic.cornell_queries(64, seed=4)
    q[:8, :3] = [[0, 0, 0], [1, 1, 1], [-0.05, 0.05, 0.0], [0.5, 0.25, 0.125], [0.999, 0.001, -0.001],
                 [1e-9, -1e-9, 0.3], [-1, -1, -1], [2.5, -3.5, 0.7]]
    for s in range(len(q)):
        for level in range(16):
            e, w = orc.hash_corners(q[s], level)
            e2, w2 = corners_np(q[s], level)
            np.testing.assert_array_equal(e, e2)
            np.testing.assert_array_equal(w, w2)
            assert abs(float(w.astype(np.float64).sum()) - 1.0) < 1e-6


def test_level_sizes_and_layout():
    entries = [4096] + [32768] * 15
    assert sum(entries) * 2 == 991232
    # dense levels: resolution^3 fits the table (16^3, 32^3), hashed otherwise
    assert 16 ** 3 <= 32768 and 32 ** 3 <= 32768 and 64 ** 3 > 32768


def _torch_model(params, queries, targets):
    """float64 autograd model of the Hash config; returns (loss, grad) — the oracle's FP32 mode."""
    import torch
    p = torch.tensor(params.astype(np.float64), requires_grad=True)
    q = queries
    n = q.shape[0]
    feats = []
    for level in range(16):
        E = np.zeros((n, 8), np.int64)
        W = np.zeros((n, 8), np.float64)
        for s in range(n):
            e, w = corners_np(q[s], level)
            E[s], W[s] = e, w
        for f in range(2):
            idx = torch.tensor(21504 + 2 * E + f)
            feats.append((p[idx] * torch.tensor(W)).sum(1))
    hash_f = torch.stack(feats, 1)  # level-major, feature-minor
    import nrc_loader
    orc = nrc_loader.load_oracle()
    rest = torch.tensor(orc.encode(q)[:, 36:66].astype(np.float64))
    enc = torch.cat([hash_f, rest, torch.ones((n, 2), dtype=torch.float64)], 1)
    offs = [0, 4096, 8192, 12288, 16384, 20480]
    h = enc
    for l in range(5):
        Wl = p[offs[l]:offs[l] + 4096].reshape(64, 64)
        h = torch.relu(h @ Wl.T)
    y = torch.relu(h @ p[20480:21504].reshape(16, 64).T)[:, :3]
    lum = (0.299 * y[:, 0] + 0.587 * y[:, 1] + 0.114 * y[:, 2]).detach()
    t = torch.tensor(targets.astype(np.float64))
    loss = (((y - t) ** 2) / (lum[:, None] ** 2 + 0.01)).sum() / (3 * n)
    loss.backward()
    return float(loss.detach()), p.grad.numpy(), y.detach().numpy()


def test_hash_forward_and_grad_match_torch_autograd(nrc, orc):
    rng = np.random.default_rng(0)
    params = orc.hash_init_params(7)
    params[21504:] = rng.uniform(-0.5, 0.5, 991232).astype(np.float32)  # non-trivial grid values
    params[:21504] *= np.float32(1.5)
    q, t = nrc.synthetic.cornell_batch(24, seed=5)
    q[:, :3] = rng.uniform(-0.3, 1.2, (24, 3)).astype(np.float32)
    loss_t, grad_t, y_t = _torch_model(params, q, t)
    y = orc.hash_forward(params, q, orc.FP32)
    np.testing.assert_allclose(y, y_t, rtol=2e-5, atol=1e-6)
    g, loss = orc.hash_grad(params, q, t, mode=orc.FP32, loss_scale=1.0)
    assert abs(loss - loss_t) <= 1e-5 * abs(loss_t)
    touched = np.flatnonzero(grad_t)
    assert touched.size > 24 * 16  # grid entries receive gradient
    np.testing.assert_allclose(g, grad_t, rtol=2e-4, atol=1e-7 * np.abs(grad_t).max())


def test_hash_modes_close(nrc, orc):
    params = orc.hash_init_params(3)
    params[21504:] *= np.float32(2000.0)
    q = nrc.synthetic.cornell_queries(256, seed=9)
    y32 = orc.hash_forward(params, q, orc.FP32)
    for mode in (orc.MIXED, orc.TCNN):
        y = orc.hash_forward(params, q, mode)
        assert np.linalg.norm(y - y32) / np.linalg.norm(y32) < 1e-2


def test_hash_sparse_adam(orc):
    params = orc.hash_init_params(1)
    st = orc.HashAdamEmaState(params)
    g = np.zeros(orc.HASH_NUM_PARAMS, np.float32)
    g[:21504] = 0.5
    g[21504 + 10] = 3.0
    st.apply(g)
    # untouched grid entries: weights, moments, steps unchanged; EMA still filtered
    assert st.grid_steps[10] == 1 and st.grid_steps[11] == 0
    assert st.params[21504 + 11] == params[21504 + 11] and st.m[21504 + 11] == 0.0
    assert st.params[21504 + 10] != params[21504 + 10]
    assert st.ema[21504 + 11] == params[21504 + 11] * (np.float32(1.0) - np.float32(0.99))
    # matrix params: every param steps (l2 regularised)
    g2 = np.zeros_like(g)
    st.apply(g2)
    assert np.all(st.params[:21504] != params[:21504])
    assert st.grid_steps[10] == 1  # zero gradient: no step for the grid entry


def test_f16_round_double_matches_numpy(orc):
    """The half-FMA emulation rounds the exact f64 result straight to f16 (numpy's float64 -> float16 is direct)."""
    rng = np.random.default_rng(0)
    x = rng.normal(size=20000) * np.exp(rng.uniform(-25, 11, 20000))
    # ties and near-ties of the f16 grid, which an f32 intermediate can double-round
    base = rng.uniform(-2, 2, 2000).astype(np.float16).astype(np.float64)
    x = np.concatenate([x, base + 2.0 ** -12 * np.sign(base), base + 2.0 ** -12 * np.sign(base) + 2.0 ** -40])
    L = orc.lib()
    got = np.array([L.orc_f16_round_double(float(v)) for v in x], np.float32)
    with np.errstate(over="ignore"):
        ref = x.astype(np.float16).astype(np.float32)
    np.testing.assert_array_equal(got, ref)
