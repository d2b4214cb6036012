"""GPU parity of the width-128 network (BASELINE.json configs[4] / SURVEY §8 C5) against the oracle
(oracle/nrc_wide_oracle.c), through the C-ABI: inference (f16 and FP8) and training.

Tolerances:
* f16 path vs ORC_MIXED (same numerics model as the 64-wide network): relative L2 <= 1e-3 and at most 0.1 % of the
  queries beyond 16 f16 ulps of their output scale (north_star tolerance);
* e4m3 conversion (the FP8 kernel's: saturating v_cvt_scalef32_pk_fp8_f32 under MODE.FP16_OVFL, ReLU on the bytes) vs
  the oracle's RNE of the clamped value: bit-exact;
* FP8 path vs ORC_FP8: relative L2 <= 2.2e-2 (70,001 queries; 3e-2 at 1 and 33) and >= 98 % of outputs within 2^-10
  relative
  (measured 1.4-1.9e-2 and 99.3 % at 70,001 queries). Not bit-exact by construction: the MX MFMA's 64-element fp8 block sum is
  not f32-exact (<= ~2.2e-5 of sum|a*b|, tools/microbench/fp8_probe.hip), so a pre-activation near an e4m3 rounding
  boundary can land one e4m3 step (2^-3 relative) away and that step propagates;
* training, as the 64-wide network (tests/test_gpu_parity.py): weight gradient vs ORC_MIXED relative L2 <= 2e-3,
  loss within 1e-3; one Adam + EMA step from the oracle's gradient: >= 99 % equal update signs, relative L2 of the
  new weights <= 1e-3 (Adam's first step is +-lr per weight, so a gradient differing in sign flips a whole step);
* FP8 vs the f16 network (the approximation FP8 makes): reported only — on these random (untrained) weights the deep
  ReLU chain amplifies the e4m3 rounding to ~0.25-0.4 relative L2, a property of the weights, not of the kernel.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WIDE_SHAPES = [(128, 80), (128, 128), (128, 128), (128, 128), (128, 128), (16, 128)]


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


def wide_params(seed, gain=1.6):
    """xavier-uniform weights scaled so that activations stay O(1) through 6 ReLU layers"""
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.uniform(-1, 1, o * i) * np.sqrt(6.0 / (o + i)) * gain
                           for o, i in WIDE_SHAPES]).astype(np.float32)


@pytest.fixture(params=["Frequency", "FrequencySH"])
def wnet(request, nrc, dev):
    import torch
    enc = getattr(nrc.InputEncoding, request.param)
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), encoding=enc, config=nrc.default_config(enc, width=128))
    yield net, enc
    net.destroy()


def run(net, nrc, dev, q, precision=None):
    import torch
    n = len(q)
    out = torch.full((n + 8, 3), 777.0, device=dev)
    if precision is None:
        net.infer(_t(q, dev), out, n)
    else:
        net.infer_precision(precision, _t(q, dev), out, n)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert (o[n:] == 777.0).all(), "infer wrote past n"
    return o[:n]


def test_fp8_conversion_bit_exact(nrc, orc, dev):
    import torch
    E = [(c & 7) * 2.0 ** -9 if (c >> 3) == 0 else (1 + (c & 7) / 8) * 2.0 ** ((c >> 3) - 7) for c in range(0x7f)]
    E = np.array(E, np.float32)
    mids = (0.5 * (E[1:].astype(np.float64) + E[:-1])).astype(np.float32)
    rng = np.random.default_rng(8)
    x = np.concatenate([E, mids, np.nextafter(mids, np.float32(0)), np.nextafter(mids, np.float32(1e9)),
                        np.exp2(rng.uniform(-14, 9.5, 200000)).astype(np.float32), [0.0, 1e-40, 500.0, 1e9]])
    x = np.concatenate([x, -x]).astype(np.float32)
    y = torch.zeros(len(x), dtype=torch.uint8, device=dev)
    for relu in (True, False):
        nrc.fp8_convert(_t(x, dev), y, len(x), relu=relu)
        torch.cuda.synchronize()
        got = y.cpu().numpy()
        lo = 0.0 if relu else -448.0
        ref = np.array([orc.e4m3(float(v)) for v in np.clip(x, lo, 448.0)])
        # decode the GPU bytes
        mag = E[got & 0x7f]
        val = np.where(got & 0x80, -mag, mag)
        assert ((got & 0x7f) != 0x7f).all(), "NaN encoding produced"
        np.testing.assert_array_equal(val, ref.astype(np.float32))


def test_wide_config_and_state(nrc, dev, wnet):
    net, enc = wnet
    assert net.num_params == nrc._lib.WIDE_NUM_PARAMS
    assert '"n_neurons":128' in net.configJson()
    p = net.get_state(nrc.StateSlot.PARAMS)
    np.testing.assert_array_equal(p, net.get_state(nrc.StateSlot.INFER))
    assert np.isfinite(p).all() and 0.05 < np.abs(p).max() < 0.3


@pytest.mark.parametrize("n", [1, 33, 4096, 70001])
def test_wide_f16_infer_parity(nrc, orc, dev, wnet, n):
    net, enc = wnet
    params = wide_params(11)
    net.set_state(nrc.StateSlot.INFER, params)
    q = nrc.synthetic.cornell_queries(n, seed=400 + n)
    o = run(net, nrc, dev, q)
    y = orc.wide_forward(params, q, orc.MIXED, encoding=int(enc))
    err = np.abs(o - y).max(axis=1)
    tol = 16.0 * 2.0 ** -11 * np.maximum(np.abs(y).max(axis=1), 1e-2)
    assert np.flatnonzero(err > tol).size <= max(1, 0.001 * n)
    assert rel(o, y) <= 1e-3, rel(o, y)


@pytest.mark.parametrize("n", [1, 33, 70001])
def test_wide_fp8_infer_parity(nrc, orc, dev, wnet, n):
    net, enc = wnet
    params = wide_params(12)
    net.set_state(nrc.StateSlot.INFER, params)
    q = nrc.synthetic.cornell_queries(n, seed=500 + n)
    o8 = run(net, nrc, dev, q, precision=nrc._lib.PRECISION_FP8)
    y8 = orc.wide_forward(params, q, orc.FP8, encoding=int(enc))
    r8 = rel(o8, y8)
    if n > 1000:
        ymx = orc.wide_forward(params, q, orc.MIXED, encoding=int(enc))
        close = float(np.mean(np.abs(o8 - y8) <= 2.0 ** -10 * np.abs(y8) + 1e-6))
        print(f"fp8 vs ORC_FP8 rel-L2 {r8:.2e} ({close:.3f} of outputs within 2^-10), ORC_FP8 vs the f16 network "
              f"{rel(y8, ymx):.2e}, GPU fp8 vs the f16 network {rel(o8, ymx):.2e}")
        assert close > 0.98
    print(f"n={n}: fp8 vs ORC_FP8 rel-L2 {r8:.3e}")
    # round 4: a frame-sized sample is held to 2.2e-2 (measured 1.4e-2 - 1.9e-2); a handful of
    # queries keeps 3e-2 (one query one e4m3 step away moves a 33-query rel-L2 by more)
    assert r8 <= (2.2e-2 if n > 1000 else 3e-2), r8


def test_wide_fp8_configured_handle(nrc, orc, dev):
    """infer() of a handle configured with infer_precision FP8 runs the FP8 kernel; re-packing follows set_state."""
    import torch
    net = nrc.Network()
    cfg = nrc.default_config(nrc.InputEncoding.Frequency, width=128, infer_precision=nrc._lib.PRECISION_FP8)
    net.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Frequency, config=cfg)
    try:
        q = nrc.synthetic.cornell_queries(5000, seed=9)
        for seed in (13, 14):
            params = wide_params(seed)
            net.set_state(nrc.StateSlot.INFER, params)
            o = run(net, nrc, dev, q)
            o8 = run(net, nrc, dev, q, precision=nrc._lib.PRECISION_FP8)
            np.testing.assert_array_equal(o, o8)
            assert rel(o, orc.wide_forward(params, q, orc.FP8)) <= 1e-2
    finally:
        net.destroy()


def test_wide_fused_accumulate(nrc, dev, wnet):
    import torch
    net, enc = wnet
    net.set_state(nrc.StateSlot.INFER, wide_params(15))
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(96, 64, (4, 4), seed=6)
    n = f.screen_size + f.num_tiles
    q = _t(f.queries_inference, dev)
    thr = _t(f.last_render_throughput, dev)
    for mode in (F.RenderMode.Full, F.RenderMode.CacheOnly):
        ref = torch.empty((n, 3), device=dev)
        net.infer(q, ref, n)
        rgba_ref = torch.full((f.screen_size, 4), 0.5, device=dev)
        F.accumulate_render_radiance(ref, thr, rgba_ref, f.screen_size, mode, 2)
        res = torch.zeros((n, 3), device=dev)
        rgba = torch.full((f.screen_size, 4), 0.5, device=dev)
        F.infer_accumulate(net, q, res, n, thr, rgba, f.screen_size, mode, 2)
        torch.cuda.synchronize()
        assert torch.equal(rgba, rgba_ref) and torch.equal(res[f.screen_size:], ref[f.screen_size:])


GB = 16384


def test_wide_grad_matches_oracle(nrc, orc, dev, wnet):
    import torch
    net, enc = wnet
    params = wide_params(21, gain=1.2)
    net.set_state(nrc.StateSlot.PARAMS, params)
    q, t = nrc.synthetic.cornell_batch(GB, seed=61)
    grad = torch.zeros(net.grad_floats, device=dev)
    net.train_grad(_t(q, dev), _t(t, dev), GB, GB, grad)
    torch.cuda.synchronize()
    g = grad.cpu().numpy()
    g_ref, l_ref = orc.wide_grad(params, q, t, mode=orc.MIXED, encoding=int(enc))
    n = nrc.WIDE_NUM_PARAMS
    assert rel(g[:n], g_ref) <= 2e-3, rel(g[:n], g_ref)
    assert abs(g[n] - l_ref) <= 1e-3 * abs(l_ref)
    # the gradient of every layer, not just the largest
    offs = [0, 10240, 26624, 43008, 59392, 75776, 77824]
    for l in range(6):
        assert rel(g[offs[l]:offs[l + 1]], g_ref[offs[l]:offs[l + 1]]) <= 5e-3, l


@pytest.mark.parametrize("b", [1000, 4000, 4001])
def test_wide_grad_ragged_batch(nrc, orc, dev, wnet, b):
    """Batches that are not a multiple of the 64-sample forward/backward block or of the 512-sample dW chunk: the
    last block's second wave has no samples (b = 4000, 4001) and the last chunk is partial."""
    import torch
    net, enc = wnet
    params = wide_params(24, gain=1.2)
    net.set_state(nrc.StateSlot.PARAMS, params)
    q, t = nrc.synthetic.cornell_batch(b, seed=64)
    grad = torch.full((net.grad_floats,), 7.0, device=dev)  # stale contents must be overwritten
    net.train_grad(_t(q, dev), _t(t, dev), b, b, grad)
    torch.cuda.synchronize()
    g = grad.cpu().numpy()
    g_ref, l_ref = orc.wide_grad(params, q, t, mode=orc.MIXED, encoding=int(enc))
    n = nrc.WIDE_NUM_PARAMS
    assert rel(g[:n], g_ref) <= 2e-3, rel(g[:n], g_ref)
    assert abs(g[n] - l_ref) <= 1e-3 * abs(l_ref)


def test_wide_train_step_matches_oracle(nrc, orc, dev, wnet):
    import torch
    net, enc = wnet
    params = wide_params(22, gain=1.2)
    net.set_state(nrc.StateSlot.PARAMS, params)
    net.set_state(nrc.StateSlot.INFER, params)
    net.step = 0
    q, t = nrc.synthetic.cornell_batch(GB, seed=62)
    loss = net.train(_t(q, dev), _t(t, dev), loss=True)
    g_ref, l_ref = orc.wide_grad(params, q, t, mode=orc.MIXED, encoding=int(enc))
    assert abs(loss - l_ref) <= 1e-3 * abs(l_ref)
    st = orc.AdamEmaState(params)
    st.apply(g_ref)
    p1 = net.get_state(nrc.StateSlot.PARAMS)
    d_gpu, d_ref = p1 - params, st.params - params
    assert np.mean(np.sign(d_gpu) == np.sign(d_ref)) >= 0.99
    assert rel(p1, st.params) <= 1e-3
    assert rel(net.get_state(nrc.StateSlot.INFER), st.infer) <= 1e-3
    assert net.step == 1


def test_wide_data_parallel_split_matches_fused_step(nrc, dev):
    """two half-batch gradients summed + apply == one fused step (the RCCL all-reduce's arithmetic)"""
    import torch
    enc = nrc.InputEncoding.Frequency
    nets = []
    for _ in range(2):
        n = nrc.Network()
        n.init(stream=torch.cuda.current_stream(), encoding=enc, config=nrc.default_config(enc, width=128))
        nets.append(n)
    try:
        params = wide_params(23, gain=1.2)
        for n in nets:
            n.set_state(nrc.StateSlot.PARAMS, params)
        q, t = nrc.synthetic.cornell_batch(GB, seed=63)
        qd, td = _t(q, dev), _t(t, dev)
        nets[0].train(qd, td)
        g = torch.zeros(nets[1].grad_floats, device=dev)
        g2 = torch.zeros_like(g)
        h = GB // 2
        nets[1].train_grad(qd, td, h, GB, g)
        nets[1].train_grad(qd[h:], td[h:], h, GB, g2)
        nets[1].train_apply(g + g2)
        torch.cuda.synchronize()
        pa, pb = nets[0].get_state(nrc.StateSlot.PARAMS), nets[1].get_state(nrc.StateSlot.PARAMS)
        assert np.mean(np.sign(pa - params) == np.sign(pb - params)) >= 0.999
        assert rel(pb, pa) <= 1e-4
    finally:
        for n in nets:
            n.destroy()


def test_wide_training_learns_and_fp8_on_trained_weights(nrc, orc, dev):
    import torch
    enc = nrc.InputEncoding.Frequency
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), encoding=enc, config=nrc.default_config(enc, width=128))
    try:
        q, t = nrc.synthetic.cornell_batch(4 * GB, seed=64)
        qd, td = _t(q, dev), _t(t, dev)
        losses = []
        for it in range(60):
            b = (it % 4) * GB
            losses.append(net.train(qd[b:], td[b:], loss=True))
        assert np.isfinite(losses).all()
        assert np.mean(losses[-4:]) < 0.8 * np.mean(losses[:4]), (losses[:4], losses[-4:])
        # inference on the trained (EMA) weights: f16 vs the oracle, FP8 vs the f16 network
        qi = nrc.synthetic.cornell_queries(20000, seed=65)
        w = net.get_state(nrc.StateSlot.INFER)
        o16 = run(net, nrc, dev, qi, precision=nrc.PRECISION_F16)
        o8 = run(net, nrc, dev, qi, precision=nrc.PRECISION_FP8)
        y = orc.wide_forward(w, qi, orc.MIXED)
        assert rel(o16, y) <= 1e-3
        r = rel(o8, o16)
        print(f"trained width-128 network: loss {losses[0]:.4g} -> {losses[-1]:.4g}; FP8 vs f16 rel-L2 {r:.3e}")
        assert r <= 0.1
    finally:
        net.destroy()


@pytest.mark.parametrize("n", [1, 1000, 4097, 70001])
def test_wide_kernel_variant_bit_identical(nrc, dev, n):
    """The 1024-thread-block debug variant (4 waves per SIMD) computes exactly what the production kernel does
    (debug library only; tests/test_gpu_debug_lib.py runs this test under it)."""
    import torch
    if not nrc._lib.is_debug_library():
        pytest.skip("A/B variant of the debug library (libnrc_amd_debug.so)")
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Frequency,
             config=nrc.default_config(nrc.InputEncoding.Frequency, width=128))
    try:
        q = nrc.synthetic.cornell_queries(n, seed=n)
        for prec in (nrc._lib.PRECISION_F16, nrc._lib.PRECISION_FP8):
            base = run(net, nrc, dev, q, prec)
            var = run(net, nrc, dev, q, prec | (1 << 4))
            assert np.array_equal(base, var), f"precision {prec}: variant differs"
    finally:
        net.destroy()


@pytest.mark.parametrize("gain", [1.6, 6.0])
def test_wide_fp8_byte_relu_variant_bit_identical(nrc, dev, gain):
    """The production FP8 kernel (round 6: ReLU on the converted e4m3 bytes, saturation by the convert under
    MODE.FP16_OVFL, tools/probe_fp8_cvt.hip) against debug variant 2 (round 5: a med3 clamp per value before the
    convert): bitwise, on xavier weights (gain 1.6) and on weights large enough that the hidden activations pass 448
    (gain 6: the clamp and the saturating convert must agree there)."""
    import torch
    if not nrc._lib.is_debug_library():
        pytest.skip("A/B variant of the debug library (libnrc_amd_debug.so)")
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Frequency,
             config=nrc.default_config(nrc.InputEncoding.Frequency, width=128))
    try:
        net.set_state(nrc.StateSlot.INFER, wide_params(13, gain))
        q = nrc.synthetic.cornell_queries(70001, seed=17)
        base = run(net, nrc, dev, q, nrc._lib.PRECISION_FP8)
        var = run(net, nrc, dev, q, nrc._lib.PRECISION_FP8 | (2 << 4))
        assert np.isfinite(base).all()
        assert np.array_equal(base, var)
    finally:
        net.destroy()
