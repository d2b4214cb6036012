"""CPU tests of the per-frame oracle (oracle/nrc_frame_oracle.c) against independent Python restatements,
and of the synthetic frame generator's invariants."""
import numpy as np
import pytest

MASK32 = 0xFFFFFFFF


def _mix32(x: int) -> int:
    x ^= x >> 16
    x = (x * 0x7FEB352D) & MASK32
    x ^= x >> 15
    x = (x * 0x846CA68B) & MASK32
    x ^= x >> 16
    return x


def _perm_py(seed: int, frame: int, n: int) -> list[int]:
    """DESIGN.md §9 spec, pure Python."""
    keys = [_mix32((seed & MASK32) ^ _mix32((seed >> 32) ^ _mix32((frame + 0x9E3779B9 * (r + 1)) & MASK32)))
            for r in range(4)]
    b = 2
    while b < 32 and (1 << b) < n:
        b += 1
    b += b & 1
    h = b // 2
    mask = (1 << h) - 1

    def f(x):
        L, R = x >> h, x & mask
        for r in range(4):
            L, R = R, L ^ (_mix32(R ^ keys[r]) & mask)
        return (L << h) | R

    out = []
    for d in range(n):
        x = f(d)
        while x >= n:
            x = f(x)
        out.append(x)
    return out


@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 100, 1000, 4096, 5000])
def test_permutation_matches_python_spec(orc, n):
    seed, frame = 0x123456789ABCDEF, 7
    assert orc.permutation(seed, frame, n).tolist() == _perm_py(seed, frame, n)


@pytest.mark.parametrize("n", [65536, 100003, 1 << 20])
def test_permutation_is_bijection(orc, n):
    p = orc.permutation(42, 3, n)
    assert np.array_equal(np.sort(p), np.arange(n))
    # differs across frames and seeds, and is not close to the identity
    assert not np.array_equal(p, orc.permutation(42, 4, n))
    assert not np.array_equal(p, orc.permutation(43, 3, n))
    assert np.mean(p == np.arange(n)) < 1e-3


def test_permutation_decorrelates(orc):
    """Neighbouring destinations come from far-apart sources (the purpose of the shuffle)."""
    p = orc.permutation(1, 0, 65536).astype(np.int64)
    gaps = np.abs(np.diff(p))
    assert np.median(gaps) > 10000
    assert abs(np.corrcoef(np.arange(65536), p)[0, 1]) < 0.02


def test_accumulate_matches_numpy(orc):
    rng = np.random.default_rng(0)
    n = 999
    L = rng.lognormal(-1, 1.5, (n, 3)).astype(np.float32)
    T = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    O = rng.uniform(0, 2, (n, 4)).astype(np.float32)
    for it in [0, 1, 6, 1000]:
        w = np.float32(1.0) / np.float32(it + 1)
        got = orc.accumulate(L, T, O, 0, it)
        want = (O[:, :3].astype(np.float64) + (T * L).astype(np.float64) * np.float64(w)).astype(np.float32)
        np.testing.assert_array_max_ulp(got[:, :3], want, maxulp=1)
        assert np.all(got[:, 3] == 1.0)
    np.testing.assert_array_equal(orc.accumulate(L, T, O, 2, 5)[:, :3], L * T)
    np.testing.assert_array_equal(orc.accumulate(L, T, O, 4, 5)[:, :3], L)
    np.testing.assert_array_equal(orc.accumulate(L, T, O, 5, 5)[:, :3], T)
    for mode in (1, 3):  # NoCache / CacheFirstVertex: untouched
        np.testing.assert_array_equal(orc.accumulate(L, T, O, mode, 5), O)


def _propagate_py(ends, end_rad, recs, targets, nrec):
    t = targets.astype(np.float64).copy()
    for k in range(len(ends)):
        last = end_rad[k].astype(np.float64) * float(ends["radiance_mask"][k])
        i = int(ends["start_train_record"][k])
        steps = 0
        while 0 <= i < nrec and steps < nrec:
            t[i] = np.float32(t[i] + recs["local_throughput"][i].astype(np.float64) * last)
            last = t[i].copy()
            i = int(recs["prop_to"][i])
            steps += 1
    return t.astype(np.float32)


def test_propagate_matches_python(nrc, orc):
    f = nrc.synthetic.cornell_frame(64, 48, (4, 4), seed=5, capacity=512)
    rng = np.random.default_rng(1)
    end_rad = rng.lognormal(-1, 1, (f.num_tiles, 3)).astype(np.float32)
    nrec = min(f.num_training_records, 512)
    got = orc.propagate(f.end_vertices, end_rad, f.train_records, f.train_targets, nrec)
    want = _propagate_py(f.end_vertices, end_rad, f.train_records, f.train_targets, nrec)
    np.testing.assert_array_max_ulp(got, want, maxulp=2)
    assert not np.array_equal(got, f.train_targets)


def test_propagate_hardening(nrc, orc):
    """Out-of-range starts / links end a chain; a cyclic chain is cut after num_records steps."""
    F = nrc.frame
    recs = np.zeros(4, dtype=F.TRAINING_RECORD_DTYPE)
    recs["prop_to"] = [1, 1, 99, -1]  # record 1 links to itself; record 2 links out of range
    recs["local_throughput"] = 0.5
    ends = np.zeros(4, dtype=F.END_VERTEX_DTYPE)
    ends["start_train_record"] = [0, 2, 7, F.TRAIN_RECORD_INDEX_BUFFER_FULL]
    ends["radiance_mask"] = 1.0
    er = np.ones((4, 3), np.float32)
    t = orc.propagate(ends, er, recs, np.zeros((4, 3), np.float32), 4)
    # tile 0: 0 -> 1 -> 1 -> 1 (4 steps in total): t1 = .25, then .25 + .5 * .25, then .375 + .5 * .375
    assert t[0, 0] == 0.5
    assert t[1, 0] == np.float32(0.5625)
    assert t[2, 0] == 0.5 and t[3, 0] == 0.0


def test_permute_matches_numpy(nrc, orc):
    rng = np.random.default_rng(2)
    n_out = 1024
    qs = rng.normal(size=(n_out, 15)).astype(np.float32)
    ts = rng.normal(size=(n_out, 3)).astype(np.float32)
    perm = rng.permutation(n_out).astype(np.int32)
    for nr in [n_out, 700, 1, 5000]:
        qd, td = orc.permute(qs, ts, perm, 0, 0, nr, n_out)
        s = perm % min(nr, n_out)
        np.testing.assert_array_equal(qd, qs[s])
        np.testing.assert_array_equal(td, ts[s])
    qd, td = orc.permute(qs, ts, None, 9, 2, 700, n_out)
    s = orc.permutation(9, 2, n_out) % 700
    np.testing.assert_array_equal(qd, qs[s])
    # num_records <= 0: destination untouched
    qd0 = np.full((n_out, 15), 7.0, np.float32)
    qd, _ = orc.permute(qs, ts, perm, 0, 0, 0, n_out, q_dst=qd0)
    np.testing.assert_array_equal(qd, qd0)


def test_synthetic_frame_invariants(nrc):
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(160, 96, (4, 4), seed=3, capacity=1536)
    assert f.num_tiles == 40 * 24 and f.screen_size == 160 * 96
    assert f.num_training_records > 1536  # this configuration overflows the record buffer
    nrec = min(f.num_training_records, 1536)
    visits = np.zeros(nrec, np.int64)
    for s in f.end_vertices["start_train_record"]:
        assert s >= F.TRAIN_RECORD_INDEX_NONE
        i = int(s)
        while i >= 0:
            visits[i] += 1
            i = int(f.train_records["prop_to"][i])
    assert np.all(visits == 1)  # chains are disjoint, acyclic and cover every allocated record
    assert set(np.unique(f.end_vertices["radiance_mask"])) <= {0.0, 1.0}
    assert f.queries_inference.shape == (f.screen_size + f.num_tiles, 15)
    assert f.train_records.dtype.itemsize == 28 and f.end_vertices.dtype.itemsize == 16


def test_sh_encoding_oracle_matches_numpy(nrc, orc):
    """FrequencySH extension (oracle/nrc_oracle.c orc_encode_sh) against a float64 numpy restatement."""
    q = nrc.synthetic.cornell_queries(512, seed=8).astype(np.float64)
    enc = orc.encode_sh(q.astype(np.float32)).astype(np.float64)
    th, ph = q[:, 3], q[:, 4]
    x, y, z = np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)
    sh = np.stack([np.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
                   -0.48860251190291987 * x, 1.0925484305920792 * x * y, -1.0925484305920792 * y * z,
                   0.94617469575755997 * z * z - 0.31539156525251999, -1.0925484305920792 * x * z,
                   0.54627421529603959 * (x * x - y * y), 0.59004358992664352 * y * (-3 * x * x + y * y),
                   2.8906114426405538 * x * y * z, 0.45704579946446572 * y * (1 - 5 * z * z),
                   0.3731763325901154 * z * (5 * z * z - 3), 0.45704579946446572 * x * (1 - 5 * z * z),
                   1.4453057213202769 * z * (x * x - y * y), 0.59004358992664352 * x * (-x * x + 3 * y * y)], 1)
    np.testing.assert_allclose(enc[:, 36:52], sh, atol=2e-6)
    # the orthonormal real SH: sum of squares of degree-l band is (2l+1)/(4 pi)
    for l, (a, b) in enumerate([(0, 1), (1, 4), (4, 9), (9, 16)]):
        np.testing.assert_allclose((sh[:, a:b] ** 2).sum(1), (2 * l + 1) / (4 * np.pi), rtol=1e-12)
    freq = orc.encode(q.astype(np.float32)).astype(np.float64)
    np.testing.assert_array_equal(enc[:, :36], freq[:, :36])          # triangle wave unchanged
    np.testing.assert_array_equal(enc[:, 52:68], freq[:, 44:60])      # OneBlob of normal + roughness
    np.testing.assert_array_equal(enc[:, 68:74], freq[:, 60:66])      # identity
    assert np.all(enc[:, 74:] == 1.0)
    # forward / grad entry points accept the encoding
    p = orc.init_params(3)
    y_sh = orc.forward(p, q[:64].astype(np.float32), orc.FP32, encoding=orc.FREQUENCY_SH)
    y_f = orc.forward(p, q[:64].astype(np.float32), orc.FP32)
    assert not np.array_equal(y_sh, y_f)


def _refl(q):
    """RadianceQuery::reflectance() = diffuse + specular (neural_radiance_caching.h:118), compact record."""
    return (q[:, 9:12] + q[:, 12:15]).astype(np.float32)


def test_accumulate_factored_matches_numpy(nrc, orc):
    """USE_REFLECTANCE_FACTORING 1 (nrc_helpers.cu:95-97, 111-113, 118-120): the radiance times the render query's
    reflectance, after the throughput product; DebugThroughputOnly ignores it."""
    rng = np.random.default_rng(3)
    n = 777
    L = rng.lognormal(-1, 1.5, (n, 3)).astype(np.float32)
    T = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    O = rng.uniform(0, 2, (n, 4)).astype(np.float32)
    q = nrc.synthetic.cornell_queries(n, seed=3)
    R = _refl(q)
    for it in (0, 5):
        w = np.float32(1.0) / np.float32(it + 1)
        got = orc.accumulate(L, T, O, 0, it, queries=q)
        want = (O[:, :3].astype(np.float64) + ((T * L) * R).astype(np.float64) * np.float64(w)).astype(np.float32)
        np.testing.assert_array_max_ulp(got[:, :3], want, maxulp=1)
    np.testing.assert_array_equal(orc.accumulate(L, T, O, 2, 5, queries=q)[:, :3], (L * T) * R)
    np.testing.assert_array_equal(orc.accumulate(L, T, O, 4, 5, queries=q)[:, :3], L * R)
    np.testing.assert_array_equal(orc.accumulate(L, T, O, 5, 5, queries=q)[:, :3], T)
    for mode in (1, 3):
        np.testing.assert_array_equal(orc.accumulate(L, T, O, mode, 5, queries=q), O)


def _propagate_factored_py(ends, end_rad, end_q, recs, targets, train_q, nrec):
    t = targets.astype(np.float32).copy()
    for k in range(len(ends)):
        last = (end_rad[k] * np.float32(ends["radiance_mask"][k])) * _refl(end_q[k:k + 1])[0]
        i = int(ends["start_train_record"][k])
        steps = 0
        while 0 <= i < nrec and steps < nrec:
            R = _refl(train_q[i:i + 1])[0]
            v = (t[i] * R).astype(np.float64) + recs["local_throughput"][i].astype(np.float64) * last.astype(np.float64)
            v = v.astype(np.float32)
            with np.errstate(divide="ignore", invalid="ignore"):
                t[i] = np.where(R != 0, v / np.where(R != 0, R, 1), np.float32(0))
            last = v
            i = int(recs["prop_to"][i])
            steps += 1
    return t


def test_propagate_factored_matches_python(nrc, orc):
    """USE_REFLECTANCE_FACTORING 1 (nrc_helpers.cu:156-160, 189-214): targets hold radiance / reflectance, the chain
    carries the radiance; a zero reflectance component gives a zero target (safeDiv, :28-35)."""
    f = nrc.synthetic.cornell_frame(64, 48, (4, 4), seed=7, capacity=512)
    rng = np.random.default_rng(8)
    end_rad = rng.lognormal(-1, 1, (f.num_tiles, 3)).astype(np.float32)
    end_q = nrc.synthetic.cornell_queries(f.num_tiles, seed=9)
    nrec = min(f.num_training_records, 512)
    train_q = np.array(f.train_queries, copy=True)
    train_q[::7, 9:15] = 0.0  # some records with zero reflectance: safeDiv's zero branch
    got = orc.propagate(f.end_vertices, end_rad, f.train_records, f.train_targets, nrec, end_queries=end_q,
                        train_queries=train_q)
    want = _propagate_factored_py(f.end_vertices, end_rad, end_q, f.train_records, f.train_targets, train_q, nrec)
    np.testing.assert_array_max_ulp(got, want, maxulp=2)
    plain = orc.propagate(f.end_vertices, end_rad, f.train_records, f.train_targets, nrec)
    assert not np.array_equal(got, plain)


@pytest.mark.parametrize("n", [0, 1, 2, 1000, 65536])
def test_sort_pairs_is_the_stable_argsort(orc, n):
    """orc_sort_pairs (NRCUtil.cu:19-35, cub SortPairs over the indices): numpy's stable argsort of the same keys, with
    ties (a small key range) and all-equal keys (identity)."""
    rng = np.random.default_rng(n)
    for keys in (rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
                 rng.integers(0, 5, n).astype(np.uint32) * np.uint32(0x10001),
                 np.full(n, 7, np.uint32)):
        perm, sk = orc.sort_pairs(keys)
        np.testing.assert_array_equal(perm, np.argsort(keys, kind="stable"))
        np.testing.assert_array_equal(sk, np.sort(keys))
    assert orc.sort_pairs(np.full(n, 3, np.uint32))[0].tolist() == list(range(n))
