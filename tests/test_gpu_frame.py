"""GPU parity of the per-frame kernels around the network (include/nrc/frame.h) against the C oracle
(oracle/nrc_frame_oracle.c). Integer / copy / fma work: bit-exact. The frame driver's training leg is
checked against the oracle's training at the fp16 tolerance of the network tests."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("n", [1, 257, 100_003])
def test_accumulate_bitwise(nrc, orc, dev, mode, n):
    import torch
    rng = np.random.default_rng(n + mode)
    L = rng.lognormal(-1, 1.5, (n, 3)).astype(np.float32)
    T = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    O = rng.uniform(0, 2, (n, 4)).astype(np.float32)
    for it in (0, 13):
        out = _t(O, dev)
        nrc.frame.accumulate_render_radiance(_t(L, dev), _t(T, dev), out, n, mode, it)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), orc.accumulate(L, T, O, mode, it))


def test_accumulate_tail_untouched_and_errors(nrc, dev):
    import torch
    n = 1000
    out = torch.full((n + 64, 4), -7.0, device=dev)
    L = torch.ones((n, 3), device=dev)
    nrc.frame.accumulate_render_radiance(L, L, out, n, nrc.frame.RenderMode.CacheOnly, 0)
    torch.cuda.synchronize()
    assert torch.all(out[n:] == -7.0) and torch.all(out[:n] == 1.0)
    with pytest.raises(nrc.NrcError):
        nrc.frame.accumulate_render_radiance(L, L, out, n, 9, 0)
    with pytest.raises(nrc.NrcError):  # float4 frame buffer must be 16-byte aligned
        nrc.frame.accumulate_render_radiance(L, L, int(out.data_ptr()) + 4, n, 0, 0)


def test_copy_radiance_to_output(nrc, dev):
    import torch
    L = torch.rand((777, 3), device=dev)
    out = torch.zeros((777, 4), device=dev)
    nrc.frame.copy_radiance_to_output(L, out, 777)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :3], L) and torch.all(out[:, 3] == 1)


@pytest.mark.parametrize("shape", [(64, 48, (4, 4), 512), (1920, 1080, (8, 8), 65536), (640, 480, (2, 2), 65536)])
def test_propagate_bitwise(nrc, orc, dev, shape):
    import torch
    w, h, tile, cap = shape
    f = nrc.synthetic.cornell_frame(w, h, tile, seed=11, capacity=cap)
    nrec = min(f.num_training_records, cap)
    rng = np.random.default_rng(4)
    end_rad = rng.lognormal(-1, 1, (f.num_tiles, 3)).astype(np.float32)
    tg = _t(f.train_targets, dev)
    nrc.frame.propagate_train_radiance(nrc.frame.records_to_device(f.end_vertices, dev), _t(end_rad, dev),
                                       f.num_tiles, nrc.frame.records_to_device(f.train_records, dev), tg, nrec)
    torch.cuda.synchronize()
    want = orc.propagate(f.end_vertices, end_rad, f.train_records, f.train_targets, nrec)
    np.testing.assert_array_equal(tg.cpu().numpy(), want)


def test_propagate_hardening(nrc, orc, dev):
    """Cyclic and out-of-range links neither hang nor fault; results match the oracle."""
    import torch
    F = nrc.frame
    recs = np.zeros(4, dtype=F.TRAINING_RECORD_DTYPE)
    recs["prop_to"] = [1, 1, 99, -1]
    recs["local_throughput"] = 0.5
    ends = np.zeros(5, dtype=F.END_VERTEX_DTYPE)
    ends["start_train_record"] = [0, 2, 7, F.TRAIN_RECORD_INDEX_BUFFER_FULL, F.TRAIN_RECORD_INDEX_NONE]
    ends["radiance_mask"] = 1.0
    er = np.ones((5, 3), np.float32)
    tg = torch.zeros((4, 3), device=dev)
    F.propagate_train_radiance(F.records_to_device(ends, dev), _t(er, dev), 5, F.records_to_device(recs, dev), tg, 4)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tg.cpu().numpy(), orc.propagate(ends, er, recs, np.zeros((4, 3), np.float32), 4))


@pytest.mark.parametrize("n", [1, 3, 1000, 65536, 100_003, 1 << 22])
def test_permutation_bitwise(nrc, orc, dev, n):
    import torch
    p = torch.empty(n, dtype=torch.int32, device=dev)
    nrc.frame.generate_train_permutation(0xDEADBEEF12345, 5, p, n)
    torch.cuda.synchronize()
    got = p.cpu().numpy()
    np.testing.assert_array_equal(got, orc.permutation(0xDEADBEEF12345, 5, n))
    assert np.array_equal(np.sort(got), np.arange(n))


def _keys(kind: str, n: int) -> np.ndarray:
    rng = np.random.default_rng(n * 7 + len(kind))
    if kind == "random":      # curand's 32-bit keys: few ties
        return rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    if kind == "ties":        # many ties in every digit
        return rng.integers(0, 300, n).astype(np.uint32) * np.uint32(0x01010101)
    if kind == "equal":       # all equal: the permutation must be the identity (stable)
        return np.full(n, 0xDEADBEEF, np.uint32)
    if kind == "sorted_desc":
        return (np.uint32(0xFFFFFFFF) - np.arange(n, dtype=np.uint32)).astype(np.uint32)
    return (rng.integers(0, 4, n).astype(np.uint32) << np.uint32(30))  # only the top digit differs


@pytest.mark.parametrize("kind", ["random", "ties", "equal", "sorted_desc", "top_digit"])
@pytest.mark.parametrize("n", [65536, 1, 17, 1000, 65537, (1 << 20) + 3])
def test_sort_train_permutation_bitwise(nrc, orc, dev, kind, n):
    """the reference's shuffle contract (NRCUtil.cu:19-35), cub::DeviceRadixSort::SortPairs of
    caller-supplied u32 keys with the indices -- bit-exact against the oracle's stable LSD restatement and numpy's
    stable argsort; ties keep index order (all-equal keys give the identity)."""
    import torch
    keys = _keys(kind, n)
    kd = _t(keys.view(np.int32), dev)
    perm = torch.full((n + 64,), -5, dtype=torch.int32, device=dev)
    sk = torch.zeros(n, dtype=torch.int32, device=dev)
    nrc.frame.sort_train_permutation(kd, perm, n, sorted_keys=sk)
    torch.cuda.synchronize()
    got = perm.cpu().numpy()
    assert (got[n:] == -5).all(), "wrote past n"
    want, want_keys = orc.sort_pairs(keys)
    np.testing.assert_array_equal(got[:n], want)
    np.testing.assert_array_equal(got[:n], np.argsort(keys, kind="stable"))
    np.testing.assert_array_equal(sk.cpu().numpy().view(np.uint32), want_keys)
    np.testing.assert_array_equal(kd.cpu().numpy().view(np.uint32), keys)  # input untouched
    if kind == "equal":
        np.testing.assert_array_equal(got[:n], np.arange(n))


def test_sort_train_permutation_errors(nrc, dev):
    import torch
    keys = torch.zeros(100, dtype=torch.int32, device=dev)
    perm = torch.zeros(100, dtype=torch.int32, device=dev)
    small = torch.zeros(8, dtype=torch.uint8, device=dev)
    with pytest.raises(nrc.NrcError):
        nrc.frame.sort_train_permutation(keys, perm, 100, temp=small)
    with pytest.raises(nrc.NrcError):
        nrc.frame.sort_train_permutation(keys, perm, (1 << 24) + 1)
    nrc.frame.sort_train_permutation(keys, perm, 0)  # no-op
    assert nrc.frame.sort_train_permutation_temp_bytes(65536) >= 3 * 65536 * 4


def test_process_frame_with_shuffle_keys(nrc, orc, dev):
    """The frame driver with the renderer's keys (nrc_frame_buffers.shuffle_keys_d): the shuffled training buffers are
    bitwise those made with the oracle's key-sort permutation passed explicitly, and the whole frame (losses, weights)
    is bitwise the explicit-permutation frame."""
    import torch
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(128, 64, (4, 4), seed=8)
    keys = _keys("random", 65536)
    perm, _ = orc.sort_pairs(keys)
    res = []
    for use_keys in (True, False):
        net = nrc.Network()
        net.init(stream=torch.cuda.current_stream())
        fb, tq0, tt0, rec = _device_frame(nrc, f, dev, with_perm=None if use_keys else perm)
        if use_keys:
            fb.shuffle_keys = _t(keys.view(np.int32), dev)
        loss = F.process_frame(net, fb, F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records))
        torch.cuda.synchronize()
        res.append((loss, fb.train_queries[1].cpu().numpy(), fb.train_targets[1].cpu().numpy(),
                    net.get_state(nrc.StateSlot.PARAMS)))
        net.destroy()
    nrec = min(f.num_training_records, 65536)
    np.testing.assert_array_equal(res[0][1], tq0[perm % nrec])
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("num_records", [65536, 40000, 1, 70000, 0, -3])
@pytest.mark.parametrize("explicit", [False, True])
def test_permute_bitwise(nrc, orc, dev, num_records, explicit):
    import torch
    n_out = 65536
    rng = np.random.default_rng(num_records & 0xFFFF)
    qs = rng.normal(size=(n_out, 15)).astype(np.float32)
    ts = rng.normal(size=(n_out, 3)).astype(np.float32)
    perm = rng.permutation(n_out).astype(np.int32) if explicit else None
    qd = torch.full((n_out, 15), 3.0, device=dev)
    td = torch.full((n_out, 3), 3.0, device=dev)
    nrc.frame.permute_train_data(_t(qs, dev), _t(ts, dev), None if perm is None else _t(perm, dev), 77, 9,
                                 num_records, qd, td, n_out)
    torch.cuda.synchronize()
    wq, wt = orc.permute(qs, ts, perm, 77, 9, num_records, n_out, q_dst=np.full((n_out, 15), 3.0, np.float32),
                         t_dst=np.full((n_out, 3), 3.0, np.float32))
    np.testing.assert_array_equal(qd.cpu().numpy(), wq)
    np.testing.assert_array_equal(td.cpu().numpy(), wt)


# ---- the frame driver ---------------------------------------------------------------------------------------------
def _device_frame(nrc, f, dev, with_perm=None):
    import torch
    F = nrc.frame
    cap = F.NUM_TRAINING_RECORDS_PER_FRAME
    tq0 = np.zeros((cap, 15), np.float32)
    tq0[: len(f.train_queries)] = f.train_queries[:cap]
    tt0 = np.zeros((cap, 3), np.float32)
    tt0[: len(f.train_targets)] = f.train_targets[:cap]
    rec = np.zeros(cap, F.TRAINING_RECORD_DTYPE)
    rec[: len(f.train_records)] = f.train_records[:cap]
    return F.FrameBuffers(
        queries_inference=_t(f.queries_inference, dev),
        results_inference=torch.zeros((f.screen_size + f.num_tiles, 3), device=dev),
        last_render_throughput=_t(f.last_render_throughput, dev),
        output_rgba=torch.zeros((f.screen_size, 4), device=dev),
        queries_cache_vis=_t(f.queries_cache_vis, dev),
        results_cache_vis=torch.zeros((f.screen_size, 3), device=dev),
        end_vertices=F.records_to_device(f.end_vertices, dev),
        train_records=F.records_to_device(rec, dev),
        train_queries=[_t(tq0, dev), torch.zeros((cap, 15), device=dev)],
        train_targets=[_t(tt0, dev), torch.zeros((cap, 3), device=dev)],
        permutation=None if with_perm is None else _t(with_perm, dev)), tq0, tt0, rec


def test_process_frame_matches_oracle_pipeline(nrc, orc, dev):
    """One full frame (infer -> accumulate -> propagate -> shuffle -> 4 x train) against the oracle's steps."""
    import torch
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(320, 240, (4, 4), seed=21, frame_index=3)
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    params = orc.init_params(1337) * np.float32(1.6)
    for slot in (nrc.StateSlot.PARAMS, nrc.StateSlot.INFER):
        net.set_state(slot, params)
    fb, tq0, tt0, rec = _device_frame(nrc, f, dev)
    out0 = np.random.default_rng(0).uniform(0, 1, (f.screen_size, 4)).astype(np.float32)
    fb.output_rgba.copy_(_t(out0, dev))
    fp = F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records, F.RenderMode.Full, iteration_index=2,
                       frame_index=3, shuffle_seed=99, keep_render_results=True)
    loss = F.process_frame(net, fb, fp)
    torch.cuda.synchronize()

    # infer: the network's own per-query tolerance is covered by test_gpu_parity; here the downstream steps are
    # checked bit-exactly given the GPU's radiance.
    res = fb.results_inference.cpu().numpy()
    y_ref = orc.forward(params, f.queries_inference, orc.MIXED)
    assert np.linalg.norm(res - y_ref) / np.linalg.norm(y_ref) < 1e-3
    np.testing.assert_array_equal(fb.output_rgba.cpu().numpy(),
                                  orc.accumulate(res[: f.screen_size], f.last_render_throughput, out0, 0, 2))
    nrec = min(f.num_training_records, 65536)
    tt_prop = orc.propagate(f.end_vertices, res[f.screen_size:], rec, tt0, nrec)
    np.testing.assert_array_equal(fb.train_targets[0].cpu().numpy(), tt_prop)
    qd, td = orc.permute(tq0, tt_prop, None, 99, 3, nrec, 65536)
    np.testing.assert_array_equal(fb.train_queries[1].cpu().numpy(), qd)
    np.testing.assert_array_equal(fb.train_targets[1].cpu().numpy(), td)

    # training: 4 oracle steps on the same shuffled batches
    st = orc.AdamEmaState(params)
    losses = []
    for b in range(4):
        s = slice(b * 16384, (b + 1) * 16384)
        g, lb = orc.grad(st.params, qd[s], td[s])
        st.apply(g)
        losses.append(lb)
    # same tolerances as test_gpu_parity.test_train_step_matches_oracle_and_learns (fp16 network)
    assert abs(loss - np.mean(losses)) <= 2e-2 * abs(np.mean(losses))
    assert net.step == 4
    p_gpu = net.get_state(nrc.StateSlot.PARAMS)
    assert np.linalg.norm(p_gpu - st.params) / np.linalg.norm(st.params) <= 1e-3
    net.destroy()


def test_process_frame_modes(nrc, orc, dev):
    import torch
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(128, 64, (4, 4), seed=2)
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    params = net.get_state(nrc.StateSlot.INFER)

    # NoCache: render queries are not inferred, the frame buffer is untouched, training still runs
    fb, *_ = _device_frame(nrc, f, dev)
    fb.results_inference.fill_(-1.0)
    fb.output_rgba.fill_(5.0)
    loss = F.process_frame(net, fb, F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records,
                                                  F.RenderMode.NoCache))
    torch.cuda.synchronize()
    assert torch.all(fb.results_inference[: f.screen_size] == -1.0)
    assert torch.all(fb.results_inference[f.screen_size:] != -1.0)
    assert torch.all(fb.output_rgba == 5.0)
    assert np.isfinite(loss) and net.step == 4

    # CacheFirstVertex: output = radiance at the first non-specular vertex
    net.init(stream=torch.cuda.current_stream())
    net.set_state(nrc.StateSlot.INFER, params)
    fb, *_ = _device_frame(nrc, f, dev)
    loss = F.process_frame(net, fb, F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records,
                                                  F.RenderMode.CacheFirstVertex, train=False))
    torch.cuda.synchronize()
    assert loss == 0.0 and net.step == 0
    vis = fb.results_cache_vis.cpu().numpy()
    assert np.linalg.norm(vis - orc.forward(params, f.queries_cache_vis, orc.MIXED)) / np.linalg.norm(vis) < 1e-3
    np.testing.assert_array_equal(fb.output_rgba.cpu().numpy()[:, :3], vis)

    # no records: no training (Device.cpp:2507)
    fb, *_ = _device_frame(nrc, f, dev)
    assert F.process_frame(net, fb, F.FrameParams(f.screen_size, f.num_tiles, 0)) == 0.0
    assert net.step == 0

    # explicit (caller-made) permutation: shuffled buffers follow it exactly
    perm = np.random.default_rng(5).permutation(65536).astype(np.int32)
    fb, tq0, tt0, rec = _device_frame(nrc, f, dev, with_perm=perm)
    F.process_frame(net, fb, F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records), loss=False)
    torch.cuda.synchronize()
    nrec = min(f.num_training_records, 65536)
    np.testing.assert_array_equal(fb.train_queries[1].cpu().numpy(), tq0[perm % nrec])

    net.destroy()
    with pytest.raises(nrc.NrcError):
        F.process_frame(net, fb, F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records))


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("n,n_acc", [(100_003, 90_001), (4096, 4096), (777, 0), (2_097_152 + 32_400, 2_097_152)])
def test_infer_accumulate_fused_bitwise(nrc, dev, mode, n, n_acc):
    """Fused inference epilogue == nrc_infer + nrc_accumulate_render_radiance, bit for bit; render radiance is not
    written, train-suffix radiance is."""
    import torch
    F = nrc.frame
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    q = _t(nrc.synthetic.cornell_queries(n, seed=n), dev)
    rng = np.random.default_rng(n_acc)
    thr = _t(rng.uniform(0, 1, (max(n_acc, 1), 3)).astype(np.float32), dev)
    rgba0 = _t(rng.uniform(0, 1, (max(n_acc, 1), 4)).astype(np.float32), dev)
    ref_res = torch.empty((n, 3), device=dev)
    net.infer(q, ref_res, n)
    ref_rgba = rgba0.clone()
    F.accumulate_render_radiance(ref_res, thr, ref_rgba, n_acc, mode, 5)
    res = torch.full((n, 3), -3.0, device=dev)
    rgba = rgba0.clone()
    F.infer_accumulate(net, q, res, n, thr, rgba, n_acc, mode, 5)
    torch.cuda.synchronize()
    assert torch.equal(rgba, ref_rgba)
    assert torch.equal(res[n_acc:], ref_res[n_acc:])
    assert torch.all(res[:n_acc] == -3.0)
    with pytest.raises(nrc.NrcError):
        F.infer_accumulate(net, q, res, n, thr, rgba, n_acc, F.RenderMode.DebugThroughputOnly, 0)
    net.destroy()


@pytest.mark.parametrize("encoding", ["Frequency", "Hash"])
def test_process_frame_fused_equals_unfused(nrc, dev, encoding):
    """The default (fused, one loss sync) frame == the reference-shaped unfused frame: same frame buffer, same
    train-suffix radiance, same losses and weights. Hash (round 5): the frame driver over the Hash handle's feature
    pass + MLP pass with the fused accumulation, and its training steps (scatter partials, one optimizer launch)."""
    import torch
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(256, 192, (4, 4), seed=8, frame_index=1)
    out = []
    for keep in (False, True):
        net = nrc.Network()
        net.init(stream=torch.cuda.current_stream(), encoding=getattr(nrc.InputEncoding, encoding))
        fb, *_ = _device_frame(nrc, f, dev)
        fb.output_rgba.fill_(0.25)
        losses = [F.process_frame(net, fb, F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records,
                                                         F.RenderMode.Full, iteration_index=it, frame_index=it,
                                                         keep_render_results=keep)) for it in range(3)]
        torch.cuda.synchronize()
        out.append((losses, fb.output_rgba.cpu().numpy(), fb.results_inference[f.screen_size:].cpu().numpy(),
                    net.get_state(nrc.StateSlot.INFER)))
        net.destroy()
    (l0, o0, r0, w0), (l1, o1, r1, w1) = out
    assert l0 == l1
    np.testing.assert_array_equal(o0, o1)
    np.testing.assert_array_equal(r0, r1)
    np.testing.assert_array_equal(w0, w1)


# ---- USE_REFLECTANCE_FACTORING 1 (frame.h *_factored, nrc_frame_params.reflectance_factoring): bit-exact vs the oracle
@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("n", [1, 100_003])
def test_accumulate_factored_bitwise(nrc, orc, dev, mode, n):
    import torch
    rng = np.random.default_rng(n + 7 * mode)
    L = rng.lognormal(-1, 1.5, (n, 3)).astype(np.float32)
    T = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    O = rng.uniform(0, 2, (n, 4)).astype(np.float32)
    q = nrc.synthetic.cornell_queries(n, seed=n + mode)
    for it in (0, 13):
        out = _t(O, dev)
        nrc.frame.accumulate_render_radiance_factored(_t(L, dev), _t(q, dev), _t(T, dev), out, n, mode, it)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), orc.accumulate(L, T, O, mode, it, queries=q))


@pytest.mark.parametrize("shape", [(64, 48, (4, 4), 512), (1920, 1080, (8, 8), 65536)])
def test_propagate_factored_bitwise(nrc, orc, dev, shape):
    import torch
    w, h, tile, cap = shape
    f = nrc.synthetic.cornell_frame(w, h, tile, seed=13, capacity=cap)
    nrec = min(f.num_training_records, cap)
    rng = np.random.default_rng(5)
    end_rad = rng.lognormal(-1, 1, (f.num_tiles, 3)).astype(np.float32)
    end_q = nrc.synthetic.cornell_queries(f.num_tiles, seed=17)
    train_q = np.array(f.train_queries, copy=True)
    train_q[::5, 9:15] = 0.0  # zero reflectance on some records: safeDiv's zero branch
    tg = _t(f.train_targets, dev)
    nrc.frame.propagate_train_radiance_factored(nrc.frame.records_to_device(f.end_vertices, dev), _t(end_rad, dev),
                                                _t(end_q, dev), f.num_tiles,
                                                nrc.frame.records_to_device(f.train_records, dev), tg,
                                                _t(train_q, dev), nrec)
    torch.cuda.synchronize()
    want = orc.propagate(f.end_vertices, end_rad, f.train_records, f.train_targets, nrec, end_queries=end_q,
                         train_queries=train_q)
    np.testing.assert_array_equal(tg.cpu().numpy(), want)


def test_process_frame_reflectance_factoring(nrc, orc, dev):
    """The frame driver with reflectance_factoring: unfused inference, the factored accumulation with the render
    queries, the factored propagation with the tile queries (inference buffer after the pixels) and the records'
    queries as traced; the shuffle and training unchanged. Every step after inference bit-exact vs the oracle."""
    import torch
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(320, 240, (4, 4), seed=23, frame_index=2)
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    fb, tq0, tt0, rec = _device_frame(nrc, f, dev)
    out0 = np.random.default_rng(1).uniform(0, 1, (f.screen_size, 4)).astype(np.float32)
    fb.output_rgba.copy_(_t(out0, dev))
    fp = F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records, F.RenderMode.Full, iteration_index=3,
                       frame_index=2, shuffle_seed=7, reflectance_factoring=True)
    F.process_frame(net, fb, fp)
    torch.cuda.synchronize()
    res = fb.results_inference.cpu().numpy()
    S = f.screen_size
    np.testing.assert_array_equal(fb.output_rgba.cpu().numpy(),
                                  orc.accumulate(res[:S], f.last_render_throughput, out0, 0, 3,
                                                 queries=f.queries_inference[:S]))
    nrec = min(f.num_training_records, 65536)
    tt_prop = orc.propagate(f.end_vertices, res[S:], rec, tt0, nrec, end_queries=f.queries_inference[S:],
                            train_queries=tq0)
    np.testing.assert_array_equal(fb.train_targets[0].cpu().numpy(), tt_prop)
    qd, td = orc.permute(tq0, tt_prop, None, 7, 2, nrec, 65536)
    np.testing.assert_array_equal(fb.train_targets[1].cpu().numpy(), td)
    assert net.step == 4
    # CacheFirstVertex: the cache-vis radiance times the cache-vis queries' reflectance
    fb.output_rgba.zero_()
    fp2 = F.FrameParams(f.screen_size, f.num_tiles, 0, F.RenderMode.CacheFirstVertex, reflectance_factoring=True,
                        train=False)
    F.process_frame(net, fb, fp2, loss=False)
    torch.cuda.synchronize()
    cv = fb.results_cache_vis.cpu().numpy()
    np.testing.assert_array_equal(fb.output_rgba.cpu().numpy(),
                                  orc.accumulate(cv, cv, np.zeros((S, 4), np.float32), 4, 0, queries=f.queries_cache_vis))
    net.destroy()
