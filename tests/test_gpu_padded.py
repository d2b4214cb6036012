"""The non-compact RadianceQuery layout (USE_COMPACT_RADIANCE_QUERY 0, /root/reference/nrc/shaders/config.h:113,
neural_radiance_caching.h:38-40, :107-111; NRCNetworkConfigs.h:61-67, :106-111) through nrc_config.query_layout.

Two kinds of check:
* equivalence, bitwise: with pad_ = 1.0 in every query, a padded handle computes exactly what a compact handle computes
  with W0's columns permuted into the compact order (the padded encoding's pad_ slot is the compact encoding's first
  constant-one slot) -- inference, the Hash feature pass, both Frequency training kernels, Hash training and the whole
  frame driver; every load offset, record stride and kernel instance of the padded path is exercised against the
  compact one;
* parity with the oracle on random pad_ values (oracle/nrc_oracle.c orc_encode_padded: the reference's padded column
  order, independent of the handle's internal order): inference at the network tolerance of test_gpu_parity.py, the
  weight gradient at the tolerances of the gradient tests (Frequency rel-L2 <= 2e-3; Hash MLP <= 2e-4, grid <= 1e-3).
Parity unpinned as for the compact layout.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FREQ_REAL, FREQ_PADCOL = 36, 66  # real columns before pad_; the compact column that carries it
HASH_REAL, HASH_PADCOL = 32, 62


@pytest.fixture(scope="module")
def torch():
    import torch as _t

    return _t


def to_dev(torch, dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def padded(q15, pad):
    """[n][15] compact records -> [n][16] padded records with pad_ = pad (scalar or [n])."""
    q = np.asarray(q15, np.float32)
    return np.ascontiguousarray(np.insert(q, 3, np.broadcast_to(np.float32(pad), (q.shape[0],)), axis=1), np.float32)


def api_column(hash_enc: bool, c: int) -> int:
    """Column of the reference's padded encoding holding the handle's internal (compact-order) column c."""
    R, E = (HASH_REAL, HASH_PADCOL) if hash_enc else (FREQ_REAL, FREQ_PADCOL)
    return c if c < R else c + 1 if c < E else R if c == E else c


def to_internal(blob, hash_enc: bool):
    """API (padded-order) parameter blob -> the compact-order blob the same handle computes with."""
    inw = 64 if hash_enc else 80
    out = np.array(blob, np.float32, copy=True)
    w0 = np.asarray(blob, np.float32)[: 64 * inw].reshape(64, inw)
    cols = [api_column(hash_enc, c) for c in range(inw)]
    out[: 64 * inw] = w0[:, cols].reshape(-1)
    return out


def make_net(nrc, torch, encoding, padded_layout: bool):
    cfg = nrc.default_config(encoding)
    cfg.query_layout = nrc.QUERY_PADDED if padded_layout else nrc.QUERY_COMPACT
    n = nrc.Network()
    n.init(stream=torch.cuda.current_stream(), encoding=encoding, config=cfg)
    return n


def infer(torch, dev, net, q_np):
    n = q_np.shape[0]
    out = torch.full((n + 32, 3), 4321.0, dtype=torch.float32, device=dev)
    net.infer(to_dev(torch, dev, q_np), out, n)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert (o[n:] == 4321.0).all()
    return o[:n]


def test_mapping_is_a_bijection_and_roundtrips(nrc, torch, dev, golden):
    for h in (False, True):
        inw = 64 if h else 80
        assert sorted(api_column(h, c) for c in range(inw)) == list(range(inw))
    net = make_net(nrc, torch, nrc.InputEncoding.Frequency, True)
    p = np.asarray(golden["params_b"], np.float32)
    net.set_state(nrc.StateSlot.PARAMS, p)
    np.testing.assert_array_equal(net.get_state(nrc.StateSlot.PARAMS), p)
    assert '{"n_dims_to_encode":1,"otype":"Identity"},{"n_bins":4' in net.configJson()
    net.destroy()


@pytest.mark.parametrize("case", ["sh", "wide", "acc16"])
def test_unsupported_combinations(nrc, torch, case):
    cfg = nrc.default_config(nrc.InputEncoding.Frequency, width=128 if case == "wide" else 64,
                             infer_precision=nrc.PRECISION_F16_ACC16 if case == "acc16" else 0)
    cfg.query_layout = nrc.QUERY_PADDED
    enc = nrc.InputEncoding.FrequencySH if case == "sh" else nrc.InputEncoding.Frequency
    net = nrc.Network()
    with pytest.raises(nrc.NrcError) as e:
        net.init(stream=torch.cuda.current_stream(), encoding=enc, config=cfg)
    assert e.value.status == 5
    cfg.query_layout = 7
    with pytest.raises(nrc.NrcError) as e:
        net.init(stream=torch.cuda.current_stream(), encoding=enc, config=cfg)
    assert e.value.status == 1


@pytest.mark.parametrize("encoding", ["Frequency", "Hash"])
def test_pad_one_equals_compact_bitwise(nrc, torch, dev, golden, encoding):
    """pad_ = 1.0: inference and training of the padded handle are bitwise the compact handle's with W0's columns
    permuted (Frequency: 16,384-sample steps on the role-split kernel and 2,048-sample steps on the decoupled-chain
    kernel; Hash: the feature-pass inference and the Hash training kernel + exact scatter)."""
    enc = getattr(nrc.InputEncoding, encoding)
    h = encoding == "Hash"
    P, C = make_net(nrc, torch, enc, True), make_net(nrc, torch, enc, False)
    p_api = P.get_state(nrc.StateSlot.PARAMS)
    if not h:
        p_api = np.asarray(golden["params_b"], np.float32)
        for slot in (nrc.StateSlot.PARAMS, nrc.StateSlot.INFER):
            P.set_state(slot, p_api)
    for slot in (nrc.StateSlot.PARAMS, nrc.StateSlot.INFER):
        C.set_state(slot, to_internal(P.get_state(slot), h))
    for n in (1, 33, 70001):
        q15 = nrc.synthetic.cornell_queries(n, seed=300 + n)
        np.testing.assert_array_equal(infer(torch, dev, P, padded(q15, 1.0)), infer(torch, dev, C, q15))
    for it, b in enumerate((16384, 2048, 16384)):
        q15, t = nrc.synthetic.cornell_batch(b, seed=310 + it)
        lp = P.train_batch(to_dev(torch, dev, padded(q15, 1.0)), to_dev(torch, dev, t), b, loss=True)
        lc = C.train_batch(to_dev(torch, dev, q15), to_dev(torch, dev, t), b, loss=True)
        assert lp == lc, (it, lp, lc)
    for slot in (nrc.StateSlot.PARAMS, nrc.StateSlot.INFER, nrc.StateSlot.ADAM_M, nrc.StateSlot.ADAM_V):
        np.testing.assert_array_equal(to_internal(P.get_state(slot), h), C.get_state(slot))
    q15 = nrc.synthetic.cornell_queries(4097, seed=333)
    np.testing.assert_array_equal(infer(torch, dev, P, padded(q15, 1.0)), infer(torch, dev, C, q15))
    P.destroy()
    C.destroy()


@pytest.mark.parametrize("n", [1, 33, 4096, 70001])
def test_padded_inference_vs_oracle(nrc, orc, torch, dev, golden, n):
    """Random pad_ values: the pad_ feature reaches layer 0 in the reference's column order."""
    params = np.asarray(golden["params_b"], np.float32)
    net = make_net(nrc, torch, nrc.InputEncoding.Frequency, True)
    net.set_state(nrc.StateSlot.INFER, params)
    q = padded(nrc.synthetic.cornell_queries(n, seed=400 + n), np.random.default_rng(n).uniform(-1, 1, n))
    y = infer(torch, dev, net, q)
    y_ref = orc.forward(params, q, orc.MIXED, encoding=orc.FREQUENCY | orc.PADDED)
    assert rel(y, y_ref) <= 1e-3
    err = np.abs(y - y_ref).max(axis=1)
    tol = 16.0 * 2.0 ** -11 * np.maximum(np.abs(y_ref).max(axis=1), 1e-2)
    assert np.count_nonzero(err > tol) <= 0.001 * n
    # the pad_ column matters: the compact-order oracle on the same values (pad_ dropped) is far off
    if n >= 4096:
        y_nopad = orc.forward(to_internal(params, False), np.delete(q, 3, axis=1), orc.MIXED)
        assert rel(y_nopad, y_ref) > 1e-2
    net.destroy()


@pytest.mark.parametrize("b", [2048, 16384])
def test_padded_gradient_vs_oracle(nrc, orc, torch, dev, golden, b):
    params = np.asarray(golden["params_b"], np.float32)
    net = make_net(nrc, torch, nrc.InputEncoding.Frequency, True)
    net.set_state(nrc.StateSlot.PARAMS, params)
    q15, t = nrc.synthetic.cornell_batch(b, seed=500 + b)
    q = padded(q15, np.random.default_rng(b).uniform(-1, 1, b))
    g = torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev)
    net.train_grad(to_dev(torch, dev, q), to_dev(torch, dev, t), b, b, g)
    torch.cuda.synchronize()
    g_int = g.cpu().numpy()[: nrc.NUM_PARAMS]
    g_ref, loss_ref = orc.grad(params, q, t, mode=orc.MIXED, encoding=orc.FREQUENCY | orc.PADDED)
    assert rel(g_int, to_internal(g_ref, False)) <= 2e-3
    assert abs(g.cpu().numpy()[nrc.NUM_PARAMS] - loss_ref) <= 1e-3 * abs(loss_ref)
    net.destroy()


def test_padded_hash_vs_oracle(nrc, orc, torch, dev):
    net = make_net(nrc, torch, nrc.InputEncoding.Hash, True)
    params = net.get_state(nrc.StateSlot.PARAMS)
    rng = np.random.default_rng(7)
    params[nrc.HASH_MLP_PARAMS:] = rng.uniform(-0.5, 0.5, nrc.HASH_GRID_PARAMS).astype(np.float32)
    for slot in (nrc.StateSlot.PARAMS, nrc.StateSlot.INFER):
        net.set_state(slot, params)
    n = 70001
    q = padded(nrc.synthetic.cornell_queries(n, seed=601), rng.uniform(-1, 1, n))
    y = infer(torch, dev, net, q)
    y_ref = orc.hash_forward(params, q, orc.MIXED, padded=True)
    assert rel(y, y_ref) <= 1e-3
    b = 16384
    q15, t = nrc.synthetic.cornell_batch(b, seed=602)
    qb = padded(q15, rng.uniform(-1, 1, b))
    g = torch.zeros(nrc.HASH_GRAD_FLOATS, dtype=torch.float32, device=dev)
    net.train_grad(to_dev(torch, dev, qb), to_dev(torch, dev, t), b, b, g)
    torch.cuda.synchronize()
    gg = g.cpu().numpy()
    g_ref, loss_ref = orc.hash_grad(params, qb, t, mode=orc.MIXED, padded=True)
    M = nrc.HASH_MLP_PARAMS
    assert rel(gg[:M], to_internal(g_ref[:M], True)) <= 2e-4
    assert rel(gg[M:nrc.HASH_NUM_PARAMS], g_ref[M:]) <= 1e-3
    net.destroy()


# ---- the frame entry points over padded records: bit-exact against the compact oracle on the same values ----------
def test_padded_permute_bitwise(nrc, orc, torch, dev):
    n_out, nrec = 65536, 40000
    rng = np.random.default_rng(11)
    qs = rng.normal(size=(n_out, 16)).astype(np.float32)
    ts = rng.normal(size=(n_out, 3)).astype(np.float32)
    qd = torch.full((n_out, 16), 3.0, device=dev)
    td = torch.full((n_out, 3), 3.0, device=dev)
    nrc.frame.permute_train_data(to_dev(torch, dev, qs), to_dev(torch, dev, ts), None, 77, 9, nrec, qd, td, n_out,
                                 padded=True)
    torch.cuda.synchronize()
    perm = orc.permutation(77, 9, n_out)
    src = perm.astype(np.int64) % nrec
    np.testing.assert_array_equal(qd.cpu().numpy(), qs[src])
    np.testing.assert_array_equal(td.cpu().numpy(), ts[src])


@pytest.mark.parametrize("mode", [0, 2, 4, 5])
def test_padded_accumulate_factored_bitwise(nrc, orc, torch, dev, mode):
    n = 100_003
    rng = np.random.default_rng(mode)
    L = rng.lognormal(-1, 1.5, (n, 3)).astype(np.float32)
    T = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    O = rng.uniform(0, 2, (n, 4)).astype(np.float32)
    q15 = nrc.synthetic.cornell_queries(n, seed=mode)
    out = to_dev(torch, dev, O)
    nrc.frame.accumulate_render_radiance_factored(to_dev(torch, dev, L), to_dev(torch, dev, padded(q15, 9.0)),
                                                  to_dev(torch, dev, T), out, n, mode, 5, padded=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), orc.accumulate(L, T, O, mode, 5, queries=q15))


def test_padded_propagate_factored_bitwise(nrc, orc, torch, dev):
    f = nrc.synthetic.cornell_frame(1920, 1080, (8, 8), seed=13, capacity=65536)
    nrec = min(f.num_training_records, 65536)
    rng = np.random.default_rng(5)
    end_rad = rng.lognormal(-1, 1, (f.num_tiles, 3)).astype(np.float32)
    end_q = nrc.synthetic.cornell_queries(f.num_tiles, seed=17)
    train_q = np.array(f.train_queries, copy=True)
    train_q[::5, 9:15] = 0.0
    tg = to_dev(torch, dev, f.train_targets)
    F = nrc.frame
    F.propagate_train_radiance_factored(F.records_to_device(f.end_vertices, dev), to_dev(torch, dev, end_rad),
                                        to_dev(torch, dev, padded(end_q, -2.0)), f.num_tiles,
                                        F.records_to_device(f.train_records, dev), tg,
                                        to_dev(torch, dev, padded(train_q, 3.0)), nrec, padded=True)
    torch.cuda.synchronize()
    want = orc.propagate(f.end_vertices, end_rad, f.train_records, f.train_targets, nrec, end_queries=end_q,
                         train_queries=train_q)
    np.testing.assert_array_equal(tg.cpu().numpy(), want)


@pytest.mark.parametrize("rf", [False, True])
def test_padded_process_frame_equals_compact(nrc, torch, dev, rf):
    """The frame driver on a padded handle with padded frame buffers (pad_ = 1.0) against a compact handle with the
    permuted weights: frame buffer, propagated targets, shuffled records, losses and weights bitwise equal."""
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(320, 240, (4, 4), seed=29, frame_index=1)
    cap = F.NUM_TRAINING_RECORDS_PER_FRAME
    out0 = np.random.default_rng(3).uniform(0, 1, (f.screen_size, 4)).astype(np.float32)
    runs = []
    for pad in (True, False):
        net = make_net(nrc, torch, nrc.InputEncoding.Frequency, pad)
        if not pad:
            for slot in (nrc.StateSlot.PARAMS, nrc.StateSlot.INFER):
                net.set_state(slot, to_internal(runs[0]["p0"], False))
        p0 = net.get_state(nrc.StateSlot.PARAMS)
        conv = (lambda a: padded(a, 1.0)) if pad else (lambda a: np.asarray(a, np.float32))
        qw = 16 if pad else 15
        tq0 = np.zeros((cap, 15), np.float32)
        tq0[: len(f.train_queries)] = f.train_queries[:cap]
        tt0 = np.zeros((cap, 3), np.float32)
        tt0[: len(f.train_targets)] = f.train_targets[:cap]
        rec = np.zeros(cap, F.TRAINING_RECORD_DTYPE)
        rec[: len(f.train_records)] = f.train_records[:cap]
        fb = F.FrameBuffers(
            queries_inference=to_dev(torch, dev, conv(f.queries_inference)),
            results_inference=torch.zeros((f.screen_size + f.num_tiles, 3), device=dev),
            last_render_throughput=to_dev(torch, dev, f.last_render_throughput),
            output_rgba=to_dev(torch, dev, out0),
            queries_cache_vis=to_dev(torch, dev, conv(f.queries_cache_vis)),
            results_cache_vis=torch.zeros((f.screen_size, 3), device=dev),
            end_vertices=F.records_to_device(f.end_vertices, dev),
            train_records=F.records_to_device(rec, dev),
            train_queries=[to_dev(torch, dev, conv(tq0)), torch.zeros((cap, qw), device=dev)],
            train_targets=[to_dev(torch, dev, tt0), torch.zeros((cap, 3), device=dev)],
            permutation=None)
        fp = F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records, F.RenderMode.Full, iteration_index=1,
                           frame_index=1, shuffle_seed=5, reflectance_factoring=rf)
        loss = F.process_frame(net, fb, fp)
        torch.cuda.synchronize()
        tq1 = fb.train_queries[1].cpu().numpy()
        runs.append({"p0": p0, "loss": loss, "rgba": fb.output_rgba.cpu().numpy(),
                     "res": fb.results_inference.cpu().numpy(), "tt0": fb.train_targets[0].cpu().numpy(),
                     "tq1": np.delete(tq1, 3, axis=1) if pad else tq1, "tt1": fb.train_targets[1].cpu().numpy(),
                     "params": to_internal(net.get_state(nrc.StateSlot.PARAMS), False) if pad
                     else net.get_state(nrc.StateSlot.PARAMS)})
        if pad:
            assert (tq1[: min(f.num_training_records, cap), 3] == 1.0).all()
        net.destroy()
    a, b = runs
    assert a["loss"] == b["loss"]
    for k in ("rgba", "res", "tt0", "tq1", "tt1", "params"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
