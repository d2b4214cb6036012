"""InputEncoding::Hash: the exact grid-gradient exchange for data parallelism and non-finite contributions
(DESIGN.md §10).

* nrc_train_grad_fixed on two halves of a minibatch, the int64 sums added (as an all-reduce would), then
  nrc_train_apply_fixed: the grid update is bitwise the fused single-handle step over the whole minibatch (the MLP
  part differs only by the f32 summation order of its gradient). The f32 exchange (nrc_train_grad) rounds each half
  to f16 first and is not exact -- the reason for this path.
* An f16 grid contribution w * dy that is inf or NaN cannot enter the fixed-point sum: the scatter records it per
  parameter and the rounding kernels emit +inf / -inf / NaN as tcnn's f16 atomics would combine them. Checked against
  a CPU restatement from the scatter's own inputs (positions, dL/d feature), through the f32 export, the fused Adam
  and the fixed exchange.
"""
import numpy as np
import pytest

from test_gpu_hash import _exact_grid_gradient, _t, _trained_like  # noqa: F401 (shared helpers)

pytestmark = pytest.mark.gpu


def _hash_net(nrc, params):
    import torch

    n = nrc.Network()
    n.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash)
    n.set_state(nrc.StateSlot.PARAMS, params)
    n.set_state(nrc.StateSlot.INFER, params)
    return n


def _nonfinite_grid_gradient(orc, pos, dy, b):
    """_exact_grid_gradient with tcnn's f16 semantics for non-finite contributions: any inf / NaN product makes the
    parameter's gradient +inf, -inf or NaN (+inf and -inf together: NaN), whatever the finite terms."""
    finite = _exact_grid_gradient(orc, pos, _finite_halves(dy), b)
    code = np.zeros(orc.HASH_GRID_PARAMS, np.int32)
    dyh = dy.view(np.float16).reshape(16, b, 2).astype(np.float32)
    with np.errstate(all="ignore"):
        for s in range(b):
            q = np.zeros(15, np.float32)
            q[:3] = pos[s, :3]
            for lvl in range(16):
                d0, d1 = dyh[lvl, s]
                if np.isfinite(d0) and np.isfinite(d1):
                    continue
                e, w = orc.hash_corners(q, lvl)
                for c in range(8):
                    for f, dv in ((0, d0), (1, d1)):
                        v = np.float16(np.float32(w[c]) * np.float32(dv))
                        if np.isnan(v):
                            code[2 * int(e[c]) + f] |= 3
                        elif np.isinf(v):
                            code[2 * int(e[c]) + f] |= 1 if v > 0 else 2
    out = finite.copy()
    out[code == 1] = np.inf
    out[code == 2] = -np.inf
    out[code == 3] = np.nan
    return out, code


def _nonfinite_mask(dy):
    """per (level, sample) word of two f16 dL/d feature values: does either half hold inf / NaN"""
    h = dy.astype(np.uint32)
    lo, hi = h & 0xFFFF, h >> 16
    return ((lo & 0x7C00) == 0x7C00) | ((hi & 0x7C00) == 0x7C00)


def _finite_halves(dy):
    """dy with its inf / NaN halves zeroed (their contributions are the non-finite codes; |w| <= 1, so a finite
    half only ever makes finite f16 products)"""
    h = dy.astype(np.uint32)
    lo, hi = h & 0xFFFF, h >> 16
    lo = np.where((lo & 0x7C00) == 0x7C00, 0, lo)
    hi = np.where((hi & 0x7C00) == 0x7C00, 0, hi)
    return (lo | (hi << 16)).astype(np.uint32)


def test_fixed_exchange_is_the_single_gpu_grid_step(nrc, orc, dev):
    import torch

    B = nrc.BATCH_SIZE
    p0 = _trained_like(orc, seed=31)
    fused, ra, rb = (_hash_net(nrc, p0) for _ in range(3))
    try:
        q, t = nrc.synthetic.cornell_batch(B, seed=3100)
        qd, td = _t(q, dev), _t(t, dev)
        fused.train(qd, td)
        grads, fixeds = [], []
        for net, (lo, hi) in ((ra, (0, 5000)), (rb, (5000, B))):
            g = torch.full((net.grad_floats,), 5.0, device=dev)
            f = torch.full((nrc.HASH_GRID_PARAMS,), 7, dtype=torch.int64, device=dev)  # stale contents overwritten
            net.train_grad_fixed(qd[lo:hi].contiguous(), td[lo:hi].contiguous(), hi - lo, B, g, f)
            grads.append(g)
            fixeds.append(f)
        g_sum, f_sum = grads[0] + grads[1], fixeds[0] + fixeds[1]  # what the int64 / f32 all-reduce computes
        for net in (ra, rb):
            net.train_apply_fixed(g_sum, f_sum.clone())
        torch.cuda.synchronize()
        M = nrc.HASH_MLP_PARAMS
        pf = fused.get_state(nrc.StateSlot.PARAMS)
        pa, pb = ra.get_state(nrc.StateSlot.PARAMS), rb.get_state(nrc.StateSlot.PARAMS)
        np.testing.assert_array_equal(pa, pb)  # the replicas
        assert (pf[M:] != p0[M:]).sum() > 10_000
        np.testing.assert_array_equal(pa[M:], pf[M:])  # grid: bitwise the single-GPU step
        for slot in (nrc.StateSlot.ADAM_M, nrc.StateSlot.ADAM_V):
            np.testing.assert_array_equal(ra.get_state(slot)[M:], fused.get_state(slot)[M:])
        rel = np.linalg.norm(pa[:M] - pf[:M]) / np.linalg.norm(pf[:M])
        assert rel <= 3e-3  # MLP: f32 summation order only
        # the encoded sums of a finite step are the plain fixed-point sums (no markers, no clamp)
        assert int(f_sum.abs().max()) < 2 ** 41
    finally:
        for n in (fused, ra, rb):
            n.destroy()


@pytest.mark.parametrize("poison", [[1e30], [1e30, -1e30, float("nan")]])
def test_nonfinite_contributions_propagate(nrc, orc, dev, poison):
    import torch

    b = 256
    p0 = _trained_like(orc, seed=41)
    q, t = nrc.synthetic.cornell_batch(b, seed=4100)
    # poison targets of channels whose prediction is positive (the output ReLU passes their gradient)
    y = orc.hash_forward(p0, q, orc.MIXED)
    live = np.argwhere(y > 0.05)
    assert len(live) >= 3 * len(poison)
    for k, v in enumerate(poison):
        s, ch = live[3 * k]
        t[s, ch] = v
    qd, td = _t(q, dev), _t(t, dev)
    a, fused, x0, x1 = (_hash_net(nrc, p0) for _ in range(4))
    try:
        g = torch.zeros(a.grad_floats, device=dev)
        a.train_grad(qd, td, b, b, g)
        pos = torch.zeros((b, 4), dtype=torch.float32, device=dev)
        dy = torch.zeros((16, b), dtype=torch.int32, device=dev)
        nrc._lib.check(nrc._lib.lib().nrc_debug_hash_scatter_inputs(a._h, pos.data_ptr(), dy.data_ptr(), b))
        torch.cuda.synchronize()
        dy_np = dy.cpu().numpy().astype(np.uint32)
        assert _nonfinite_mask(dy_np).any(), "the poisoned targets must produce non-finite dL/d feature"
        ref, code = _nonfinite_grid_gradient(orc, pos.cpu().numpy(), dy_np, b)
        gg = g.cpu().numpy()[nrc.HASH_MLP_PARAMS:nrc.HASH_NUM_PARAMS]
        n_nf = int((code != 0).sum())
        print(f"non-finite grid gradients: {n_nf} (+inf {(code == 1).sum()}, -inf {(code == 2).sum()}, "
              f"NaN {(code == 3).sum()}); finite touched {(np.isfinite(ref) & (ref != 0)).sum()}")
        assert 0 < n_nf < (ref != 0).sum()
        np.testing.assert_array_equal(gg, ref)  # NaN positions equal, infinities signed
        # the codes were consumed: a clean step on the same handle exports finite sums only
        q2, t2 = nrc.synthetic.cornell_batch(b, seed=4101)
        a.train_grad(_t(q2, dev), _t(t2, dev), b, b, g)
        torch.cuda.synchronize()
        assert np.isfinite(g.cpu().numpy()[nrc.HASH_MLP_PARAMS:nrc.HASH_NUM_PARAMS]).all()
        # fused step and the fixed exchange: the same parameters go non-finite, the others match bitwise
        fused.train_batch(qd, td, b)
        M = nrc.HASH_MLP_PARAMS
        gs, fs = [], []
        for net, (lo, hi) in ((x0, (0, 100)), (x1, (100, b))):
            gx = torch.zeros(net.grad_floats, device=dev)
            fx = torch.zeros(nrc.HASH_GRID_PARAMS, dtype=torch.int64, device=dev)
            net.train_grad_fixed(qd[lo:hi].contiguous(), td[lo:hi].contiguous(), hi - lo, b, gx, fx)
            gs.append(gx)
            fs.append(fx)
        x0.train_apply_fixed(gs[0] + gs[1], fs[0] + fs[1])
        torch.cuda.synchronize()
        pf, px = fused.get_state(nrc.StateSlot.PARAMS)[M:], x0.get_state(nrc.StateSlot.PARAMS)[M:]
        np.testing.assert_array_equal(~np.isfinite(pf), code != 0)
        np.testing.assert_array_equal(px, pf)
    finally:
        for n in (a, fused, x0, x1):
            n.destroy()


def test_fixed_entry_points_reject_frequency(nrc, dev):
    import torch

    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    try:
        g = torch.zeros(net.grad_floats, device=dev)
        f = torch.zeros(nrc.HASH_GRID_PARAMS, dtype=torch.int64, device=dev)
        q = torch.zeros((8, 15), device=dev)
        t = torch.zeros((8, 3), device=dev)
        with pytest.raises(nrc.NrcError):
            net.train_grad_fixed(q, t, 8, 8, g, f)
        with pytest.raises(nrc.NrcError):
            net.train_apply_fixed(g, f)
    finally:
        net.destroy()
