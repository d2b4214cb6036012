"""GPU parity of the FrequencySH encoding extension (NRC_ENCODING_FREQUENCY_SH: TriangleWave + degree-4 SH of the
direction + OneBlob + Identity, 80 wide) against the oracle (orc_encode_sh / orc_forward_enc / orc_grad_enc).
Same tolerances as the Frequency model (tests/test_gpu_parity.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture()
def snet(nrc, dev):
    import torch
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.FrequencySH)
    yield net
    net.destroy()


def test_sh_encoder_parity(nrc, orc, dev, snet):
    import torch
    q = nrc.synthetic.cornell_queries(30000, seed=12)
    enc = torch.zeros((len(q), 80), device=dev)
    snet.encode_features(_t(q, dev), enc, len(q))
    torch.cuda.synchronize()
    got = enc.cpu().numpy()
    ref = orc.encode_sh(q).astype(np.float16).astype(np.float32)
    # sinf/cosf of the GPU and libm may differ by an f32 ulp: one f16 ulp + 2e-6 absolute
    bad = np.argwhere(np.abs(got - ref) > np.abs(ref) * 2.0 ** -10 + 2e-6)
    assert bad.size == 0, f"{len(bad)} features off, first {bad[:5].tolist()}"
    assert '"SphericalHarmonics"' in snet.configJson()


@pytest.mark.parametrize("n", [1, 33, 70001])
def test_sh_infer_parity(nrc, orc, dev, snet, golden, n):
    import torch
    params = golden["params_b"]
    snet.set_state(nrc.StateSlot.INFER, params)
    q = nrc.synthetic.cornell_queries(n, seed=300 + n)
    out = torch.full((n + 8, 3), 777.0, device=dev)
    snet.infer(_t(q, dev), out, n)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert (o[n:] == 777.0).all()
    y = orc.forward(params, q, orc.MIXED, encoding=orc.FREQUENCY_SH)
    err = np.abs(o[:n] - y).max(axis=1)
    tol = 16.0 * 2.0 ** -11 * np.maximum(np.abs(y).max(axis=1), 1e-2)
    assert np.flatnonzero(err > tol).size <= 0.001 * n
    assert rel(o[:n], y) <= 1e-3


def test_sh_grad_and_training(nrc, orc, dev, snet, golden):
    import torch
    params = golden["params_b"]
    snet.set_state(nrc.StateSlot.PARAMS, params)
    q, t = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=77)
    grad = torch.zeros(nrc.GRAD_FLOATS, device=dev)
    snet.train_grad(_t(q, dev), _t(t, dev), nrc.BATCH_SIZE, nrc.BATCH_SIZE, grad)
    torch.cuda.synchronize()
    g = grad.cpu().numpy()
    g_ref, l_ref = orc.grad(params, q, t, mode=orc.MIXED, encoding=orc.FREQUENCY_SH)
    assert rel(g[:nrc.NUM_PARAMS], g_ref) <= 2e-3
    assert abs(g[nrc.NUM_PARAMS] - l_ref) <= 1e-3 * abs(l_ref)
    snet.train_apply(grad)
    # a few steps learn
    losses = [snet.train(_t(q, dev), _t(t, dev), loss=True) for _ in range(5)]
    assert losses[-1] < losses[0]


def test_sh_process_frame_fused(nrc, dev, snet):
    import torch
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(96, 64, (4, 4), seed=6)
    n = f.screen_size + f.num_tiles
    q = _t(f.queries_inference, dev)
    thr = _t(f.last_render_throughput, dev)
    ref = torch.empty((n, 3), device=dev)
    snet.infer(q, ref, n)
    rgba_ref = torch.full((f.screen_size, 4), 0.5, device=dev)
    F.accumulate_render_radiance(ref, thr, rgba_ref, f.screen_size, F.RenderMode.Full, 1)
    res = torch.zeros((n, 3), device=dev)
    rgba = torch.full((f.screen_size, 4), 0.5, device=dev)
    F.infer_accumulate(snet, q, res, n, thr, rgba, f.screen_size, F.RenderMode.Full, 1)
    torch.cuda.synchronize()
    assert torch.equal(rgba, rgba_ref) and torch.equal(res[f.screen_size:], ref[f.screen_size:])
