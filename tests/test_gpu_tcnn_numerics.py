"""The opt-in tcnn-numerics inference (nrc_config.infer_precision = NRC_PRECISION_F16_ACC16).

tiny-cuda-nn's FullyFusedMLP keeps f16 accumulators (NRCNetworkConfigs.h:26-33, SURVEY App. A.5 [M]); the oracle
emulates that as ORC_TCNN (16-wide K chunks added in K order, rounded to f16 after each). The production kernel
(f32 accumulation per layer) sits 1.7e-3 - 2.1e-3 from ORC_TCNN on the random-weight golden sets
(tests/test_gpu_parity.py::test_infer_golden_and_modes). The F16_ACC16 kernel (infer_tcnn_kernel) must meet
north_star's 1e-3 relative L2 against ORC_TCNN on those same random weights, and hold per query: at most 0.1 % of
queries beyond 16 f16 ulps of their scale (the same per-query bound as the production kernel against ORC_MIXED).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.fixture(scope="module")
def torch():
    import torch as _t

    return _t


@pytest.fixture()
def tnet(nrc, torch, dev):
    cfg = nrc.default_config(nrc.InputEncoding.Frequency, infer_precision=nrc.PRECISION_F16_ACC16)
    n = nrc.Network()
    n.init(stream=torch.cuda.current_stream(), config=cfg)
    yield n
    n.destroy()


def infer(torch, dev, net, q_np):
    n = q_np.shape[0]
    out = torch.full((n + 40, 3), 12345.0, dtype=torch.float32, device=dev)
    net.infer(torch.from_numpy(np.ascontiguousarray(q_np)).to(dev), out, n)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert (o[n:] == 12345.0).all(), "wrote past n"
    return o[:n]


def per_query_ok(y, y_ref):
    err = np.abs(y - y_ref).max(axis=1)
    tol = 16.0 * 2.0 ** -11 * np.maximum(np.abs(y_ref).max(axis=1), 1e-2)
    return int((err > tol).sum())


def test_golden_random_weights_within_1e3_of_tcnn_emulation(nrc, orc, torch, dev, tnet, golden):
    tnet.set_state(nrc.StateSlot.INFER, golden["params_b"])
    for qk, yk in [("queries", "y"), ("queries_edge", "y_edge")]:
        y = infer(torch, dev, tnet, golden[qk])
        r_tcnn, r_mixed = rel(y, golden[f"{yk}_tcnn"]), rel(y, golden[f"{yk}_mixed"])
        print(f"{qk}: F16_ACC16 rel-L2 vs ORC_TCNN {r_tcnn:.2e} (vs ORC_MIXED {r_mixed:.2e})")
        assert r_tcnn <= 1e-3
        assert per_query_ok(y, golden[f"{yk}_tcnn"]) <= 0.001 * y.shape[0] + 1


@pytest.mark.parametrize("n", [1, 33, 4096, 70001])
def test_sizes_against_oracle(nrc, orc, torch, dev, tnet, golden, n):
    params = golden["params_b"]
    tnet.set_state(nrc.StateSlot.INFER, params)
    q_np = nrc.synthetic.cornell_queries(n, seed=900 + n)
    y = infer(torch, dev, tnet, q_np)
    y_ref = orc.forward(params, q_np, orc.TCNN)
    assert rel(y, y_ref) <= 1e-3
    assert per_query_ok(y, y_ref) <= 0.001 * n + 1


def test_debug_precision_entry_matches_config(nrc, torch, dev, tnet, golden):
    """nrc_debug_infer_precision(F16_ACC16) on a default-config handle runs the same kernel as a handle configured
    for it: bitwise equal outputs; the default precision differs (f32 accumulation)."""
    d = nrc.Network()
    d.init(stream=torch.cuda.current_stream())
    try:
        for net in (tnet, d):
            net.set_state(nrc.StateSlot.INFER, golden["params_b"])
        q_np = nrc.synthetic.cornell_queries(3000, seed=5)
        q = torch.from_numpy(q_np).to(dev)
        a = torch.zeros((3000, 3), device=dev)
        tnet.infer(q, a, 3000)
        b = torch.zeros((3000, 3), device=dev)
        d.infer_precision(nrc.PRECISION_F16_ACC16, q, b, 3000)
        c = torch.zeros((3000, 3), device=dev)
        d.infer(q, c, 3000)
        torch.cuda.synchronize()
        assert torch.equal(a, b) and not torch.equal(a, c)
    finally:
        d.destroy()


def test_unsupported_combinations(nrc, torch, dev, tnet):
    for enc in (nrc.InputEncoding.FrequencySH,):
        cfg = nrc.default_config(enc, infer_precision=nrc.PRECISION_F16_ACC16)
        n = nrc.Network()
        with pytest.raises(nrc.NrcError) as e:
            n.init(stream=torch.cuda.current_stream(), encoding=enc, config=cfg)
        assert e.value.status == 5
    cfg = nrc.default_config(nrc.InputEncoding.Hash, infer_precision=nrc.PRECISION_F16_ACC16)
    cfg.query_layout = nrc.QUERY_PADDED
    with pytest.raises(nrc.NrcError) as e:
        nrc.Network().init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash, config=cfg)
    assert e.value.status == 5
    cfg = nrc.default_config(nrc.InputEncoding.Frequency, width=128, infer_precision=nrc.PRECISION_F16_ACC16)
    with pytest.raises(nrc.NrcError):
        nrc.Network().init(stream=torch.cuda.current_stream(), config=cfg)
    q = torch.zeros((64, 15), device=dev)
    out = torch.zeros((64, 3), device=dev)
    thr = torch.zeros((64, 3), device=dev)
    rgba = torch.zeros((64, 4), device=dev)
    with pytest.raises(nrc.NrcError) as e:
        nrc.frame.infer_accumulate(tnet, q, out, 64, thr, rgba, 64, nrc.frame.RenderMode.Full, 0)
    assert e.value.status == 5


def test_trained_weights_full_frame(nrc, orc, torch, dev, tnet):
    """Self-trained weights (the bench's synthetic stream, 8 steps), the whole 2^21-query frame through the kernel, a
    sample of 2,056 rows against ORC_TCNN."""
    N = 1 << 21
    for f in range(2):
        q, t = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=4000 + f)
        q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
        for b in range(4):
            tnet.train(q[b * nrc.BATCH_SIZE:], t[b * nrc.BATCH_SIZE:])
    params = tnet.get_state(nrc.StateSlot.INFER)
    q_np = nrc.synthetic.cornell_queries(N, seed=4100)
    y = infer(torch, dev, tnet, q_np)
    idx = np.arange(0, N, 1021)
    y_ref = orc.forward(params, q_np[idx], orc.TCNN)
    r = rel(y[idx], y_ref)
    print(f"trained weights, 2^21 frame, {idx.size} rows: rel-L2 vs ORC_TCNN {r:.2e}")
    assert r <= 1e-3
    assert np.isfinite(y).all()


def test_process_frame_on_a_tcnn_numerics_handle(nrc, torch, dev, tnet):
    """a handle with infer_precision F16_ACC16 has no fused accumulation epilogue, so nrc_process_frame in
    Full mode (default frame params) takes infer + accumulate_render_radiance instead of failing with UNSUPPORTED; the
    frame buffer is bitwise that of the same two calls made by hand (training off, so the weights do not move)."""
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(160, 96, (8, 8), seed=11)
    S, T = f.screen_size, f.num_tiles
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    cap = F.NUM_TRAINING_RECORDS_PER_FRAME
    fb = F.FrameBuffers(t(f.queries_inference), torch.zeros((S + T, 3), device=dev), t(f.last_render_throughput),
                        torch.full((S, 4), 0.25, device=dev), F.records_to_device(f.end_vertices, dev),
                        F.records_to_device(np.zeros(cap, F.TRAINING_RECORD_DTYPE), dev),
                        [torch.zeros((cap, 15), device=dev), torch.zeros((cap, 15), device=dev)],
                        [torch.zeros((cap, 3), device=dev), torch.zeros((cap, 3), device=dev)])
    fp = F.FrameParams(S, T, 0, F.RenderMode.Full, 3, 3, 1, train=False)
    F.process_frame(tnet, fb, fp, loss=False)
    rad = torch.zeros((S + T, 3), device=dev)
    tnet.infer(t(f.queries_inference), rad, S + T)
    rgba = torch.full((S, 4), 0.25, device=dev)
    F.accumulate_render_radiance(rad, t(f.last_render_throughput), rgba, S, F.RenderMode.Full, 3,
                                 stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert torch.equal(fb.output_rgba, rgba)
    assert torch.equal(fb.results_inference[S:], rad[S:])


# ---- InputEncoding::Hash (round 5): the same f16-accumulate MLP behind the HashGrid encoding ----
@pytest.fixture()
def hnet(nrc, torch, dev):
    cfg = nrc.default_config(nrc.InputEncoding.Hash, infer_precision=nrc.PRECISION_F16_ACC16)
    n = nrc.Network()
    n.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash, config=cfg)
    yield n
    n.destroy()


def _hash_params_random(nrc, orc):
    """The Hash model's random init with the grid table drawn wide (tcnn initialises it to +-1e-4, which makes every grid
    feature ~0 and the check blind to the grid): the MLP at init, the table uniform in [-1, 1]."""
    p = orc.hash_init_params(7).copy()
    rng = np.random.default_rng(5)
    p[nrc.HASH_MLP_PARAMS:] = rng.uniform(-1.0, 1.0, p.size - nrc.HASH_MLP_PARAMS).astype(np.float32)
    return p


@pytest.mark.parametrize("n", [1, 33, 4096, 70001])
def test_hash_random_weights_within_1e3_of_tcnn_emulation(nrc, orc, torch, dev, hnet, n):
    """Hash F16_ACC16 against the Hash oracle's ORC_TCNN mode (the same feature pass, the MLP with f16 accumulation per
    16-wide K chunk in canonical K order): north_star's 1e-3 relative L2 on random weights, and the per-query bound; the
    default (f32-accumulate) Hash kernel's distance to ORC_TCNN is printed beside it."""
    params = _hash_params_random(nrc, orc)
    hnet.set_state(nrc.StateSlot.INFER, params)
    q_np = nrc.synthetic.cornell_queries(n, seed=1200 + n)
    y = infer(torch, dev, hnet, q_np)
    y_tcnn = orc.hash_forward(params, q_np, orc.TCNN)
    r = rel(y, y_tcnn)
    d = nrc.Network()
    d.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash)
    d.set_state(nrc.StateSlot.INFER, params)
    y_def = infer(torch, dev, d, q_np)
    d.destroy()
    print(f"Hash n={n}: F16_ACC16 rel-L2 vs ORC_TCNN {r:.2e}; default kernel vs ORC_TCNN {rel(y_def, y_tcnn):.2e}")
    assert r <= 1e-3
    assert per_query_ok(y, y_tcnn) <= 0.001 * n + 1


def test_hash_trained_weights_two_passes(nrc, orc, torch, dev, hnet):
    """Self-trained Hash weights (8 steps of 16,384 samples), then 2^21 + 77 queries -- two feature passes -- through the
    F16_ACC16 kernel; a sample of rows across both passes within 1e-3 of ORC_TCNN."""
    for f in range(2):
        q, t = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=4200 + f)
        q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
        for b in range(4):
            hnet.train(q[b * nrc.BATCH_SIZE:], t[b * nrc.BATCH_SIZE:])
    params = hnet.get_state(nrc.StateSlot.INFER)
    N = (1 << 21) + 77
    q_np = nrc.synthetic.cornell_queries(N, seed=4300)
    y = infer(torch, dev, hnet, q_np)
    idx = np.concatenate([np.arange(0, N, 1021), np.arange(N - 77, N)])
    y_ref = orc.hash_forward(params, q_np[idx], orc.TCNN)
    r = rel(y[idx], y_ref)
    nz = float((y_ref > 0).mean())
    print(f"Hash trained weights, {N} queries, {idx.size} rows: rel-L2 vs ORC_TCNN {r:.2e} (nonzero outputs {nz:.2f}, "
          f"max {y_ref.max():.3g})")
    assert nz > 0.1, "degenerate (all-zero) network: the comparison would be vacuous"
    assert r <= 1e-3
    assert np.isfinite(y).all()


def test_hash_debug_precision_entry_matches_config(nrc, orc, torch, dev, hnet):
    d = nrc.Network()
    d.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash)
    try:
        params = _hash_params_random(nrc, orc)
        for net in (hnet, d):
            net.set_state(nrc.StateSlot.INFER, params)
        q = torch.from_numpy(nrc.synthetic.cornell_queries(3000, seed=6)).to(dev)
        a, b, c = (torch.zeros((3000, 3), device=dev) for _ in range(3))
        hnet.infer(q, a, 3000)
        d.infer_precision(nrc.PRECISION_F16_ACC16, q, b, 3000)
        d.infer(q, c, 3000)
        torch.cuda.synchronize()
        assert torch.equal(a, b) and not torch.equal(a, c)
    finally:
        d.destroy()


@pytest.mark.parametrize("encoding", ["Frequency", "Hash"])
def test_reentry_forms_bitwise_equal(nrc, torch, dev, encoding):
    """Round 6: the f16 accumulator re-enters the f32 MFMA accumulator through four 4x4x4 identity MFMAs per block and
    chunk (knob tcnn_reentry = 1, the default) or two 32x32x16 identity MFMAs (0, the first form). Both are exact
    widenings of the same f16 values, so outputs must be bit-identical -- ragged sizes, a Hash launch past one feature
    pass (2^21 + 77 queries runs two passes) and wide random weights (large activations)."""
    enc = getattr(nrc.InputEncoding, encoding)
    cfg = nrc.default_config(enc, infer_precision=nrc.PRECISION_F16_ACC16)
    n = nrc.Network()
    n.init(stream=torch.cuda.current_stream(), encoding=enc, config=cfg)
    try:
        p = n.get_state(nrc.StateSlot.INFER)
        n.set_state(nrc.StateSlot.INFER, (p * np.float32(2.0)).astype(np.float32))
        for size in ([1, 33, 70001, (1 << 21) + 77] if encoding == "Hash" else [1, 33, 70001]):
            q = torch.from_numpy(nrc.synthetic.cornell_queries(size, seed=1300 + size)).to(dev)
            outs = []
            for kv in (0, 1):
                nrc._lib.set_knob("tcnn_reentry", kv)
                o = torch.full((size + 8, 3), 777.0, device=dev)
                n.infer(q, o, size)
                outs.append(o)
            torch.cuda.synchronize()
            assert torch.equal(outs[0], outs[1]), (encoding, size)
            assert bool((outs[1][size:] == 777.0).all())
    finally:
        nrc._lib.set_knob("tcnn_reentry", -1)
        n.destroy()
