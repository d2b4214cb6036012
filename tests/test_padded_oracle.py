"""The oracle's non-compact RadianceQuery path (oracle/nrc_oracle.c orc_encode_padded, nrc_hash_oracle.c
orc_hash_*_layout; the reference's USE_COMPACT_RADIANCE_QUERY 0 encodings, NRCNetworkConfigs.h:61-67, :106-111),
checked on the CPU against the compact path it restates with one more column:
* the padded encoding is the compact one with pad_ inserted at column 36 and one constant-one column fewer;
* with pad_ = 1.0 a padded network equals the compact network whose W0 columns are permuted by the mapping
  tests/test_gpu_padded.py applies to the GPU handle (so both sides of that test rest on the same column map)."""
import numpy as np

from test_gpu_padded import padded, to_internal


def test_padded_encoding_is_the_compact_one_plus_pad(orc):
    q15 = np.random.default_rng(0).uniform(-2, 2, (257, 15)).astype(np.float32)
    pad = np.random.default_rng(1).uniform(-1, 1, 257).astype(np.float32)
    e = orc.encode_padded(padded(q15, pad))
    c = orc.encode(q15)
    np.testing.assert_array_equal(e[:, :36], c[:, :36])
    np.testing.assert_array_equal(e[:, 36], pad)
    np.testing.assert_array_equal(e[:, 37:67], c[:, 36:66])
    assert (e[:, 67:] == 1.0).all() and (c[:, 66:] == 1.0).all()


def test_padded_network_with_pad_one_is_the_permuted_compact_network(nrc, orc):
    rng = np.random.default_rng(2)
    p_api = orc.init_params(7) * np.float32(1.5)
    q15, t = nrc.synthetic.cornell_batch(512, seed=3)
    q16 = padded(q15, 1.0)
    for mode in (orc.FP32, orc.MIXED):
        y_pad = orc.forward(p_api, q16, mode, encoding=orc.FREQUENCY | orc.PADDED, threads=4)
        y_cmp = orc.forward(to_internal(p_api, False), q15, mode, threads=4)
        np.testing.assert_array_equal(y_pad, y_cmp)
    g_pad, l_pad = orc.grad(p_api, q16, t, mode=orc.MIXED, encoding=orc.FREQUENCY | orc.PADDED, threads=4)
    g_cmp, l_cmp = orc.grad(to_internal(p_api, False), q15, t, mode=orc.MIXED, threads=4)
    assert l_pad == l_cmp
    np.testing.assert_array_equal(to_internal(g_pad, False), g_cmp)
    # and pad_ is a real input: other values change the outputs
    y_r = orc.forward(p_api, padded(q15, rng.uniform(-1, 1, 512)), orc.MIXED, encoding=orc.FREQUENCY | orc.PADDED)
    assert not np.array_equal(y_r, y_pad)


def test_padded_hash_with_pad_one_is_the_permuted_compact_network(nrc, orc):
    rng = np.random.default_rng(4)
    p_api = np.zeros(nrc.HASH_NUM_PARAMS, np.float32)
    p_api[: nrc.HASH_MLP_PARAMS] = rng.normal(0, 0.15, nrc.HASH_MLP_PARAMS)
    p_api[nrc.HASH_MLP_PARAMS:] = rng.uniform(-0.5, 0.5, nrc.HASH_GRID_PARAMS)
    q15, t = nrc.synthetic.cornell_batch(256, seed=5)
    q16 = padded(q15, 1.0)
    p_int = to_internal(p_api, True)
    np.testing.assert_array_equal(orc.hash_forward(p_api, q16, orc.MIXED, threads=4, padded=True),
                                  orc.hash_forward(p_int, q15, orc.MIXED, threads=4))
    g_pad, l_pad = orc.hash_grad(p_api, q16, t, mode=orc.MIXED, threads=4, padded=True)
    g_cmp, l_cmp = orc.hash_grad(p_int, q15, t, mode=orc.MIXED, threads=4)
    assert l_pad == l_cmp
    np.testing.assert_array_equal(to_internal(g_pad, True), g_cmp)
