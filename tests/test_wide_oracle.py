"""CPU tests of the width-128 oracle (oracle/nrc_wide_oracle.c; BASELINE configs[4]): the e4m3
rounding and row-exponent rules against independent numpy restatements, and the FP32 / MIXED / FP8 forward modes
against a float64 numpy model built from the 64-wide restatement's encoder. No GPU.

Parity is unpinned (the reference only configures 64 neurons and has no fixtures): see DESIGN.md §5, §12.
"""
import numpy as np

import nrc_loader

# every finite non-negative OCP e4m3fn value, indexed by its code (0x00 .. 0x7e)
E4M3 = np.array([(c & 7) * 2.0 ** -9 if (c >> 3) == 0 else (1 + (c & 7) / 8) * 2.0 ** ((c >> 3) - 7)
                 for c in range(0x7f)])
WIDE_SHAPES = [(128, 80), (128, 128), (128, 128), (128, 128), (128, 128), (16, 128)]


def e4m3_np(x: np.ndarray) -> np.ndarray:
    """nearest e4m3fn value, ties to the even code (|x| <= 448)"""
    x = np.asarray(x, np.float64)
    a = np.abs(x)
    i = np.clip(np.searchsorted(E4M3, a), 1, len(E4M3) - 1)
    lo, hi = E4M3[i - 1], E4M3[i]
    pick_hi = (hi - a < a - lo) | ((hi - a == a - lo) & (i % 2 == 0))
    v = np.where(pick_hi, hi, lo)
    v = np.where(a <= E4M3[0], 0.0, v)
    return np.copysign(v, x)


def test_e4m3_rounding_matches_numpy(orc):
    rng = np.random.default_rng(3)
    mids = 0.5 * (E4M3[1:] + E4M3[:-1])
    xs = np.concatenate([
        E4M3, mids, np.nextafter(mids.astype(np.float32), np.float32(0)), np.nextafter(mids.astype(np.float32),
                                                                                       np.float32(1e9)),
        rng.uniform(0, 448, 3000), np.exp2(rng.uniform(-14, 8.8, 3000)), [0.0, 1e-40, 2.0 ** -10, 3 * 2.0 ** -11],
    ]).astype(np.float32)
    xs = np.concatenate([xs, -xs])
    ours = np.array([orc.e4m3(float(v)) for v in xs])
    np.testing.assert_array_equal(ours, e4m3_np(xs.astype(np.float64)))


def test_fp8_row_exponent(orc):
    rng = np.random.default_rng(4)
    for amax in np.concatenate([np.exp2(rng.uniform(-30, 30, 500)), [448.0, 448.0 * 2 ** -3, 449.0, 1.0, 2 ** -20]]):
        amax = float(np.float32(amax))
        e = orc.fp8_row_exponent(amax)
        assert amax <= 448.0 * 2.0 ** e and amax > 448.0 * 2.0 ** (e - 1), (amax, e)
    assert orc.fp8_row_exponent(0.0) == 0


def _unpack(params):
    out, off = [], 0
    for o, i in WIDE_SHAPES:
        out.append(np.asarray(params[off:off + o * i], np.float64).reshape(o, i))
        off += o * i
    return out


def _np_forward(params, q, mode):
    import oracle_np

    W = _unpack(params)
    f16 = lambda v: v.astype(np.float32).astype(np.float16).astype(np.float64)
    a = oracle_np.encode(q)
    if mode == "fp32":
        for l in range(5):
            a = np.maximum(a @ W[l].T, 0.0).astype(np.float32).astype(np.float64)
        return np.maximum(a @ W[5].T, 0.0)[:, :3]
    a = f16(a)
    if mode == "mixed":
        for l in range(5):
            a = f16(np.maximum((a @ f16(W[l]).T).astype(np.float32), 0.0))
        return f16(np.maximum((a @ f16(W[5]).T).astype(np.float32), 0.0))[:, :3]
    # fp8: layer 0 f16, then e4m3 activations and row-scaled e4m3 weights
    a = e4m3_np(np.clip((a @ f16(W[0]).T).astype(np.float32), 0.0, 448.0))
    for l in range(1, 6):
        amax = np.abs(W[l]).max(axis=1).astype(np.float32)
        e = np.array([int(np.ceil(np.log2(float(m) / 448.0))) if m > 0 else 0 for m in amax])
        e = np.where(amax > 448.0 * np.exp2(e - 1.0), e, e - 1)  # guard ceil(log2) float edge cases
        Wq = e4m3_np(W[l] / np.exp2(e)[:, None]) * np.exp2(e)[:, None]
        y = (a @ Wq.T).astype(np.float32)
        a = e4m3_np(np.clip(y, 0.0, 448.0)) if l < 5 else f16(np.maximum(y, 0.0))
    return a[:, :3]


def _params(seed):
    rng = np.random.default_rng(seed)
    p = []
    for o, i in WIDE_SHAPES:
        p.append(rng.uniform(-1, 1, o * i) * np.sqrt(6.0 / (o + i)) * 1.6)
    return np.concatenate(p).astype(np.float32)


def test_wide_forward_modes_match_numpy(nrc, orc):
    q = nrc.synthetic.cornell_queries(600, seed=21)
    p = _params(5)
    ref32 = _np_forward(p, q, "fp32")
    y32 = orc.wide_forward(p, q, mode=orc.FP32)
    np.testing.assert_allclose(y32, ref32, rtol=2e-5, atol=1e-6)
    ymx = orc.wide_forward(p, q, mode=orc.MIXED)
    refmx = _np_forward(p, q, "mixed")
    # f16 rounding boundaries can flip on f64 summation-order differences: almost all equal, rel-L2 tiny
    assert np.mean(ymx == refmx) > 0.97
    assert np.linalg.norm(ymx - refmx) / np.linalg.norm(refmx) < 1e-3
    y8 = orc.wide_forward(p, q, mode=orc.FP8)
    ref8 = _np_forward(p, q, "fp8")
    assert np.mean(y8 == ref8) > 0.95
    assert np.linalg.norm(y8 - ref8) / np.linalg.norm(ref8) < 1e-2
    # the FP8 path is an approximation of the f16 network: a few per cent rel-L2 on these weights
    assert np.linalg.norm(y8 - ymx) / np.linalg.norm(ymx) < 0.15


def test_wide_quantize_values(orc):
    p = _params(6)
    q, e = orc.wide_quantize(p)
    W = _unpack(p)
    Q = _unpack(q)
    np.testing.assert_array_equal(Q[0], W[0].astype(np.float32).astype(np.float16).astype(np.float64))
    for l in range(1, 6):
        rows = WIDE_SHAPES[l][0]
        s = np.exp2(e[l - 1, :rows].astype(np.float64))[:, None]
        np.testing.assert_array_equal(Q[l] / s, e4m3_np(W[l] / s))
        assert (np.abs(Q[l] / s) <= 448).all()
    assert (e[4, 16:] == 0).all()


def _np_loss_grad(params, q, t, loss_scale=128.0):
    """float64 RelativeL2Luminance loss and loss-scaled gradient of the width-128 model (denominator constant)"""
    import oracle_np

    W = _unpack(params)
    a = oracle_np.encode(q)
    acts = [a]
    for l in range(5):
        a = np.maximum(a @ W[l].T, 0.0)
        acts.append(a)
    y = np.maximum(a @ W[5].T, 0.0)
    b = len(q)
    lum = 0.299 * y[:, 0] + 0.587 * y[:, 1] + 0.114 * y[:, 2]
    den = lum * lum + 0.01
    diff = y[:, :3] - t
    loss = float(np.sum(diff * diff / den[:, None]) / (3 * b))
    d = np.zeros_like(y)
    d[:, :3] = loss_scale * 2 * diff / den[:, None] / (3 * b)
    d *= y > 0
    grads = [None] * 6
    for l in range(5, -1, -1):
        grads[l] = d.T @ acts[l]
        if l:
            d = (d @ W[l]) * (acts[l] > 0)
    return loss, np.concatenate([g.reshape(-1) for g in grads])


def test_wide_grad_matches_numpy(nrc, orc):
    q, t = nrc.synthetic.cornell_batch(512, seed=31)
    p = _params(7)
    loss_ref, g_ref = _np_loss_grad(p, q, t)
    g, loss = orc.wide_grad(p, q, t, mode=orc.FP32)
    assert abs(loss - loss_ref) <= 1e-5 * abs(loss_ref)
    assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) < 1e-5
    gm, lm = orc.wide_grad(p, q, t, mode=orc.MIXED)
    assert abs(lm - loss_ref) <= 1e-2 * abs(loss_ref)
    assert np.linalg.norm(gm - g_ref) / np.linalg.norm(g_ref) < 2e-2
