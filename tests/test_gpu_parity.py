"""GPU parity: the gfx950 path through the C-ABI against the CPU oracle (oracle/nrc_oracle.c).

Tolerances (north_star: "outputs within 1e-3 relative-L2" of the network; fp16 arithmetic):
* inference outputs vs the ORC_MIXED oracle (same numerics model: f16 operands, f32 accumulate,
  f16 activations/outputs): relative L2 <= 1e-3, max |diff| <= 2 f16 ulps of the output scale;
* encoding vs oracle (f32, before the f16 cast): |diff| <= 4e-6;
* weight gradient vs ORC_MIXED: relative L2 <= 2e-3 (f16 deltas, different summation order);
* Adam + EMA from an identical gradient: relative <= 1e-6 (f32, same operation order);
* tcnn-emulation (ORC_TCNN, f16 accumulation) and exact f32 (ORC_FP32) distances are asserted at the measured
  bound (<= 2.5e-3; measured 1.7e-3 - 2.1e-3) and reported — parity with tcnn itself is unpinned (DESIGN.md §4-5,
  sensitivity table profiles/r02_sensitivity/).
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
def net(nrc, torch, dev):
    n = nrc.Network()
    n.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Frequency)
    yield n
    n.destroy()


def to_dev(torch, dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def run_infer(nrc, torch, dev, net, q_np, sentinel=True):
    n = q_np.shape[0]
    q = to_dev(torch, dev, q_np)
    out = torch.full((n + 64, 3), 12345.0, dtype=torch.float32, device=dev)
    net.infer(q, out, n)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    if sentinel:
        assert (o[n:] == 12345.0).all(), "infer wrote past n (the reference's tail overrun must not happen)"
    return o[:n]


def test_init_weights_match_oracle_init(nrc, orc, net):
    np.testing.assert_array_equal(net.get_state(nrc.StateSlot.PARAMS), orc.init_params(1337))
    np.testing.assert_array_equal(net.get_state(nrc.StateSlot.INFER), orc.init_params(1337))
    assert net.step == 0


def test_encode_parity(nrc, orc, torch, dev, golden):
    for q_np in [golden["queries"][:256], golden["queries_edge"], nrc.synthetic.cornell_queries(5000, seed=21)]:
        n = q_np.shape[0]
        enc = torch.zeros((n, 80), dtype=torch.float32, device=dev)
        nrc.encode(to_dev(torch, dev, q_np), enc, n)
        torch.cuda.synchronize()
        np.testing.assert_allclose(enc.cpu().numpy(), orc.encode(q_np), rtol=0, atol=4e-6)


@pytest.mark.parametrize("encoder", [0, 1, 2])
def test_encode_fast_parity(nrc, orc, torch, dev, golden, encoder):
    """The encoder inside the MLP kernels (closed-form OneBlob, direct (0) or omod doubling-chain (1) triangle
    wave; 2: encoder v3, tent-map triangle wave and clamped OneBlob wrap; f16 packing) against the oracle's tcnn-literal encoding rounded to f16: every feature of every query
    within one f16 ulp (plus 2e-6 absolute for the f32 evaluation-order differences)."""
    L = nrc._lib.lib()
    for q_np in [golden["queries"], golden["queries_edge"], nrc.synthetic.cornell_queries(20000, seed=22)]:
        n = q_np.shape[0]
        enc = torch.zeros((n, 80), dtype=torch.float32, device=dev)
        nrc._lib.check(L.nrc_debug_encode_fast_variant(encoder, to_dev(torch, dev, q_np).data_ptr(), enc.data_ptr(),
                                                       n, None))
        torch.cuda.synchronize()
        ref = orc.encode(q_np).astype(np.float16).astype(np.float32)
        got = enc.cpu().numpy()
        tol = np.abs(ref) * 2.0 ** -10 + 2e-6
        bad = np.argwhere(np.abs(got - ref) > tol)
        assert bad.size == 0, f"{len(bad)} features off, first (query, feature): {bad[:5].tolist()}"


@pytest.mark.parametrize("variant", [0, 23, 30, 39, 40, 41, 42, 47, 48, 61, 62, 63, 64])
def test_every_infer_variant_per_sample(nrc, orc, torch, dev, net, golden, variant):
    """Per-query max error (not an aggregate) for every kernel variant kept for A/B at sizes
    that exercise partial tiles / single blocks. The product library holds variant 47 only; the A/B variants are
    checked when the debug library is loaded (tests/test_gpu_debug_lib.py runs this test under it)."""
    if variant != 47 and not nrc._lib.is_debug_library():
        pytest.skip("A/B variant of the debug library (libnrc_amd_debug.so)")
    net.set_state(nrc.StateSlot.INFER, golden["params_b"])
    L = nrc._lib.lib()
    for n in [1, 33, 1000, 70001]:
        q_np = nrc.synthetic.cornell_queries(n, seed=700 + n)
        out = torch.full((n + 8, 3), 777.0, device=dev)
        nrc._lib.check(L.nrc_debug_infer_variant(net._h, variant, to_dev(torch, dev, q_np).data_ptr(), out.data_ptr(),
                                                 n, int(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        assert (o[n:] == 777.0).all()
        y_ref = orc.forward(golden["params_b"], q_np, orc.MIXED)
        err = np.abs(o[:n] - y_ref).max(axis=1)
        # The encoding amplifies tiny differences (d tri / dx reaches 2 * 2^11): in the oracle itself a 1e-6
        # position change moves 1.7 % of these queries by > 16 output ulps. Bound: at most 0.1 % of the
        # queries beyond 16 ulps of their scale (a wrong query or tile fails it), rel-L2 <= 1e-3 overall.
        tol = 16.0 * 2.0 ** -11 * np.maximum(np.abs(y_ref).max(axis=1), 1e-2)
        bad = np.flatnonzero(err > tol)
        assert bad.size <= 0.001 * n, f"variant {variant} n={n}: {bad.size} queries off, e.g. {bad[:5]} {o[bad[:2]]} vs {y_ref[bad[:2]]}"
        assert rel(o[:n], y_ref) <= 1e-3


@pytest.mark.parametrize("n", [1, 2, 31, 32, 33, 127, 1000, 4096, 65537])
def test_infer_parity_sizes(nrc, orc, torch, dev, net, golden, n):
    params = golden["params_b"]
    net.set_state(nrc.StateSlot.INFER, params)
    q_np = nrc.synthetic.cornell_queries(n, seed=100 + n)
    y = run_infer(nrc, torch, dev, net, q_np)
    y_ref = orc.forward(params, q_np, orc.MIXED)
    assert rel(y, y_ref) <= 1e-3
    scale = float(np.abs(y_ref).max())
    assert np.abs(y - y_ref).max() <= 2.0 * 2.0 ** -10 * max(scale, 1e-3)


def test_infer_golden_and_modes(nrc, orc, torch, dev, net, golden):
    net.set_state(nrc.StateSlot.INFER, golden["params_b"])
    for qk, yk in [("queries", "y"), ("queries_edge", "y_edge")]:
        y = run_infer(nrc, torch, dev, net, golden[qk])
        r_mixed = rel(y, golden[f"{yk}_mixed"])
        r_tcnn = rel(y, golden[f"{yk}_tcnn"])
        r_fp32 = rel(y, golden[f"{yk}_fp32"])
        print(f"{qk}: rel-L2 vs mixed {r_mixed:.2e}, vs tcnn-emulation {r_tcnn:.2e}, vs fp32 {r_fp32:.2e}")
        assert r_mixed <= 1e-3
        # Measured bounds: the f16-accumulation emulation ORC_TCNN [M] sits 1.74e-3 / 2.08e-3 (these
        # two query sets, golden weights) from ORC_MIXED, i.e. from this kernel's numerics, and exact f32 math
        # 1.86e-3 / 1.76e-3: the default path does NOT meet north_star's 1e-3 against the f16-accumulate reading of
        # tcnn, only against ORC_MIXED. With trained weights the ORC_TCNN distance is 5e-4 - 7e-4
        # (profiles/r02_sensitivity/sensitivity.json).
        assert r_tcnn <= 2.5e-3 and r_fp32 <= 2.5e-3


def test_infer_unaligned_and_offset_buffers(nrc, orc, torch, dev, net, golden):
    # RadianceQuery rows are only 4-byte aligned in the reference: start at an odd float offset
    net.set_state(nrc.StateSlot.INFER, golden["params_b"])
    n = 777
    q_np = nrc.synthetic.cornell_queries(n, seed=5)
    buf = torch.zeros(n * 15 + 1, dtype=torch.float32, device=dev)
    buf[1:] = to_dev(torch, dev, q_np.reshape(-1))
    out = torch.zeros(n * 3 + 1, dtype=torch.float32, device=dev)
    net.infer(buf.data_ptr() + 4, out.data_ptr() + 4, n)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert o[0] == 0.0
    assert rel(o[1:].reshape(n, 3), orc.forward(golden["params_b"], q_np, orc.MIXED)) <= 1e-3


def test_infer_zero_is_noop(nrc, torch, dev, net):
    out = torch.full((4, 3), 7.0, device=dev)
    net.infer(out, out, 0)
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == 7.0).all()


def test_infer_large_batch_properties(nrc, orc, torch, dev, net, golden):
    """Full C2 size (2^21): per-query independence (a permutation of the queries permutes the
    outputs bit for bit), determinism, and oracle agreement on a strided sample."""
    net.set_state(nrc.StateSlot.INFER, golden["params_b"])
    n = 1 << 21
    q_np = nrc.synthetic.cornell_queries(n, seed=2)
    q = to_dev(torch, dev, q_np)
    out1 = torch.empty((n, 3), device=dev)
    out2 = torch.empty((n, 3), device=dev)
    net.infer(q, out1, n)
    net.infer(q, out2, n)
    perm = torch.randperm(n, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    outp = torch.empty((n, 3), device=dev)
    net.infer(q[perm].contiguous(), outp, n)
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    assert torch.equal(outp, out1[perm])
    idx = np.arange(0, n, 997)
    y = out1.cpu().numpy()[idx]
    assert rel(y, orc.forward(golden["params_b"], q_np[idx], orc.MIXED)) <= 1e-3
    assert np.isfinite(y).all()


@pytest.mark.parametrize("b", [1, 100, 128, 1000, 1024, 4096])
def test_train_grad_parity(nrc, orc, torch, dev, net, golden, b):
    params = golden["params_b"]
    net.set_state(nrc.StateSlot.PARAMS, params)
    q_np, t_np = nrc.synthetic.cornell_batch(b, seed=300 + b)
    grad = torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev)
    net.train_grad(to_dev(torch, dev, q_np), to_dev(torch, dev, t_np), b, b, grad)
    torch.cuda.synchronize()
    g = grad.cpu().numpy()
    g_ref, loss_ref = orc.grad(params, q_np, t_np, mode=orc.MIXED)
    g32, _ = orc.grad(params, q_np, t_np, mode=orc.FP32)
    print(f"b={b}: grad rel vs mixed {rel(g[:nrc.NUM_PARAMS], g_ref):.2e}, vs fp32 {rel(g[:nrc.NUM_PARAMS], g32):.2e}")
    assert rel(g[:nrc.NUM_PARAMS], g_ref) <= 2e-3
    assert abs(g[nrc.NUM_PARAMS] - loss_ref) <= 1e-3 * abs(loss_ref)
    # padded output rows 3..15 get exactly zero data gradient
    w5 = g[21504:22528].reshape(16, 64)
    assert (w5[3:] == 0).all()


def test_train_grad_global_normalisation(nrc, orc, torch, dev, net, golden):
    """A rank's gradient is normalised by the global batch: sum over shards == full-batch gradient."""
    net.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
    B = 2048
    q_np, t_np = nrc.synthetic.cornell_batch(B, seed=9)
    q, t = to_dev(torch, dev, q_np), to_dev(torch, dev, t_np)
    full = torch.zeros(nrc.GRAD_FLOATS, device=dev)
    net.train_grad(q, t, B, B, full)
    parts = torch.zeros(nrc.GRAD_FLOATS, device=dev)
    for k in range(4):
        g = torch.zeros(nrc.GRAD_FLOATS, device=dev)
        s = k * (B // 4)
        net.train_grad(q[s:s + B // 4], t[s:s + B // 4], B // 4, B, g)
        parts += g
    torch.cuda.synchronize()
    assert rel(parts.cpu().numpy(), full.cpu().numpy()) <= 1e-5


def test_adam_ema_apply_matches_oracle(nrc, orc, torch, dev, net, golden):
    params = golden["params_b"]
    net.set_state(nrc.StateSlot.PARAMS, params)
    st = orc.AdamEmaState(params)
    rng = np.random.default_rng(1)
    for step in range(3):
        g = np.zeros(nrc.GRAD_FLOATS, np.float32)
        g[:nrc.NUM_PARAMS] = rng.normal(0, 1.0, nrc.NUM_PARAMS).astype(np.float32)
        g[nrc.NUM_PARAMS] = 0.5
        loss = net.train_apply(to_dev(torch, dev, g), loss=True)
        st.apply(g[:nrc.NUM_PARAMS])
        assert loss == 0.5
    for slot, ref in [(nrc.StateSlot.PARAMS, st.params), (nrc.StateSlot.ADAM_M, st.m), (nrc.StateSlot.ADAM_V, st.v),
                      (nrc.StateSlot.EMA, st.ema), (nrc.StateSlot.INFER, st.infer)]:
        np.testing.assert_allclose(net.get_state(slot), ref, rtol=1e-6, atol=1e-12)
    assert net.step == 3


def test_fused_step_equals_grad_plus_apply(nrc, torch, dev, golden):
    q_np, t_np = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=4)
    nets = []
    for _ in range(2):
        n = nrc.Network()
        n.init(stream=torch.cuda.current_stream())
        n.set_state(nrc.StateSlot.PARAMS, golden["params_b"])
        nets.append(n)
    q, t = to_dev(torch, dev, q_np), to_dev(torch, dev, t_np)
    l1 = nets[0].train(q, t, loss=True)
    grad = torch.zeros(nrc.GRAD_FLOATS, device=dev)
    nets[1].train_grad(q, t, nrc.BATCH_SIZE, nrc.BATCH_SIZE, grad)
    l2 = nets[1].train_apply(grad, loss=True)
    assert l1 == l2
    for slot in nrc.StateSlot:
        np.testing.assert_array_equal(nets[0].get_state(slot), nets[1].get_state(slot))
    for n in nets:
        n.destroy()


def test_train_step_matches_oracle_and_learns(nrc, orc, torch, dev, net, golden):
    """Several reference-shaped steps (exactly BATCH_SIZE samples each) track the oracle."""
    params = golden["params_b"]
    net.set_state(nrc.StateSlot.PARAMS, params)
    st = orc.AdamEmaState(params)
    losses, losses_ref = [], []
    for it in range(6):
        q_np, t_np = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=500 + it)
        l_gpu = net.train(to_dev(torch, dev, q_np), to_dev(torch, dev, t_np), loss=True)
        g, l_ref = orc.grad(st.params, q_np, t_np, mode=orc.MIXED)
        st.apply(g)
        losses.append(l_gpu)
        losses_ref.append(l_ref)
    print("losses gpu", losses, "oracle", losses_ref)
    np.testing.assert_allclose(losses, losses_ref, rtol=2e-2)
    assert rel(net.get_state(nrc.StateSlot.PARAMS), st.params) <= 1e-3
    assert rel(net.get_state(nrc.StateSlot.INFER), st.infer) <= 1e-3
    assert losses[-1] < losses[0]


def test_set_hyper_params_changes_the_step(nrc, orc, torch, dev, net, golden):
    """setHyperParams (NRCNetwork.cu:90-94, changed at runtime from the GUI, Application.cpp:1032) takes effect on
    the next step: 2 steps at the default LR 1e-3, LR -> 5e-4, 2 more steps; the oracle runs the same schedule."""
    params = golden["params_b"]
    net.set_state(nrc.StateSlot.PARAMS, params)
    st = orc.AdamEmaState(params)
    for it in range(4):
        if it == 2:
            net.setHyperParams(nrc.HyperParams(learningRate=5e-4))
            st.lr = 5e-4
            assert net.getLearningRate() == np.float32(5e-4)
        q_np, t_np = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=900 + it)
        net.train(to_dev(torch, dev, q_np), to_dev(torch, dev, t_np))
        g, _ = orc.grad(st.params, q_np, t_np, mode=orc.MIXED)
        st.apply(g)
    p_gpu = net.get_state(nrc.StateSlot.PARAMS)
    assert rel(p_gpu, st.params) <= 1e-3
    assert rel(net.get_state(nrc.StateSlot.INFER), st.infer) <= 1e-3
    # and the LR change is visible in the update itself: the same 4-step schedule at a constant 1e-3 lands elsewhere
    st_const = orc.AdamEmaState(params)
    for it in range(4):
        q_np, t_np = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=900 + it)
        g, _ = orc.grad(st_const.params, q_np, t_np, mode=orc.MIXED)
        st_const.apply(g)
    d_sched = rel(p_gpu, st.params)
    d_const = rel(p_gpu, st_const.params)
    assert d_const > 5 * d_sched, (d_sched, d_const)


def test_set_config_on_a_live_handle_keeps_the_model(nrc, orc, torch, dev, net, golden):
    """setConfig only replaces the config (NRCNetwork.cu:96-99): a live Frequency network that is asked for the Hash
    config keeps inferring and training as the Frequency oracle, with its learning rate."""
    import json

    params = golden["params_b"]
    net.set_state(nrc.StateSlot.PARAMS, params)
    net.set_state(nrc.StateSlot.INFER, params)
    net.setHyperParams(nrc.HyperParams(learningRate=7e-4))
    net.setConfig(nrc.InputEncoding.Hash)
    assert net.getLearningRate() == np.float32(7e-4)
    assert json.loads(net.config_json())["encoding"]["nested"][0]["otype"] == "HashGrid"
    q_np = nrc.synthetic.cornell_queries(3000, seed=31)
    y = run_infer(nrc, torch, dev, net, q_np)
    assert rel(y, orc.forward(params, q_np, orc.MIXED)) <= 1e-3
    st = orc.AdamEmaState(params, lr=7e-4)
    q_np, t_np = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=32)
    net.train(to_dev(torch, dev, q_np), to_dev(torch, dev, t_np))
    g, _ = orc.grad(st.params, q_np, t_np, mode=orc.MIXED)
    st.apply(g)
    assert rel(net.get_state(nrc.StateSlot.PARAMS), st.params) <= 1e-3
    assert net.num_params == nrc.NUM_PARAMS
    # the next init uses its own encoding argument, as init_ does (NRCNetwork.cu:106-112)
    net.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Frequency)
    assert json.loads(net.config_json())["encoding"]["nested"][0]["otype"] == "TriangleWave"


def test_training_is_deterministic(nrc, torch, dev, golden):
    q_np, t_np = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=8)
    states = []
    for _ in range(2):
        n = nrc.Network()
        n.init(stream=torch.cuda.current_stream())
        for _ in range(3):
            n.train(to_dev(torch, dev, q_np), to_dev(torch, dev, t_np))
        states.append(n.get_state(nrc.StateSlot.INFER))
        n.destroy()
    np.testing.assert_array_equal(states[0], states[1])


def test_error_behaviour(nrc, torch, dev):
    n = nrc.Network()
    with pytest.raises(nrc.NrcError):
        n.init(encoding=7)  # Unsupported input encoding: std::invalid_argument in the reference
    n.init(stream=torch.cuda.current_stream())
    with pytest.raises(ValueError):
        n.infer(None, None, 4)
    with pytest.raises(nrc.NrcError):
        n.train_batch(0, 0, 0)
    assert abs(n.getLearningRate() - 1e-3) < 1e-9
    n.setHyperParams(nrc.HyperParams(learningRate=5e-4))
    assert abs(n.getLearningRate() - 5e-4) < 1e-9
    with pytest.raises(nrc.NrcError):
        n.setHyperParams(nrc.HyperParams(learningRate=float("nan")))
    n.destroy()
    n.destroy()
    x = torch.zeros(16 * 15, device=dev)
    assert n.infer(x, x, 16) is None  # silent after destroy, like NRCNetwork.cu:66
    n.init(stream=torch.cuda.current_stream())  # re-init revives (Device.cpp:2415-2421)
    n.destroy()


def test_cpp_shim_end_to_end(tmp_path):
    """Builds the C++ replay driver (tests/cpp/replay_driver.cpp) against libnrc_amd.so and runs it."""
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    exe = tmp_path / "replay_driver"
    lib_dir = root / "neural-radiance-caching_amd"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", f"-I{root / 'include'}",
                        str(root / "tests" / "cpp" / "replay_driver.cpp"), f"-L{lib_dir}", "-lnrc_amd",
                        f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "replay ok" in r.stdout


def test_pooled_variant_bitwise_and_reusable(nrc, torch, dev, net, golden):
    """Debug library (A/B variant, rejected on speed). Variant 41 (pooled cross-CU tile draws) computes every tile exactly as 39 does, only the tile -> wave mapping
    differs: outputs are bit-identical. Its two counter sets alternate between launches and each launch zeroes the
    set it does not use, so back-to-back launches of different sizes, interleaved with non-pooled launches on the
    same handle, must all see fresh counters (a stale set would skip tiles: the 777 sentinel would survive)."""
    if not nrc._lib.is_debug_library():
        pytest.skip("A/B variant of the debug library (libnrc_amd_debug.so)")
    net.set_state(nrc.StateSlot.INFER, golden["params_b"])
    L = nrc._lib.lib()
    sp = int(torch.cuda.current_stream().cuda_stream)
    sizes = [1 << 21, 31, 1 << 21, 100_003, 1, 1 << 20, 1 << 21]
    for i, n in enumerate(sizes):
        q = to_dev(torch, dev, nrc.synthetic.cornell_queries(n, seed=900 + i))
        a = torch.full((n, 3), 777.0, device=dev)
        b = torch.full((n, 3), 777.0, device=dev)
        nrc._lib.check(L.nrc_debug_infer_variant(net._h, 39, q.data_ptr(), a.data_ptr(), n, sp))
        nrc._lib.check(L.nrc_debug_infer_variant(net._h, 41, q.data_ptr(), b.data_ptr(), n, sp))
        if i % 2:
            net.infer(q, torch.empty_like(b), n)  # the handle's own launch (product default) in between
        torch.cuda.synchronize()
        assert torch.equal(a, b), f"n={n}: {int((a != b).any(dim=1).sum())} rows differ"


@pytest.mark.parametrize("pair", [(47, 63), (62, 64)])
def test_early_first_tile_variants_bitwise(nrc, torch, dev, net, golden, pair):
    """Round 6: variants 63 / 64 take a wave's first tile by wave index and load its queries before the weight copy
    (kAblEarlyQ); the tiles and the per-query arithmetic are those of 47 / 62, so every row must be bit-identical,
    including launches with fewer tiles than waves and ragged tails."""
    if not nrc._lib.is_debug_library():
        pytest.skip("A/B variant of the debug library (libnrc_amd_debug.so)")
    net.set_state(nrc.StateSlot.INFER, golden["params_b"])
    L = nrc._lib.lib()
    sp = int(torch.cuda.current_stream().cuda_stream)
    for n in [1, 33, 1000, 70001, (1 << 19) + 5]:
        q = to_dev(torch, dev, nrc.synthetic.cornell_queries(n, seed=900 + n))
        outs = []
        for v in pair:
            o = torch.full((n + 8, 3), 777.0, device=dev)
            nrc._lib.check(L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), o.data_ptr(), n, sp))
            outs.append(o)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]), f"n={n}"
