"""Recorded sample-stream format (include/nrc/stream.h): the numpy implementation and the C-ABI reader/writer
agree byte for byte on host buffers; corrupt files are rejected. No GPU needed."""
import ctypes

import numpy as np
import pytest


def _frame(nrc, seed=0, frame_index=0, w=48, h=32, extra=True):
    S = nrc.stream
    f = nrc.synthetic.cornell_frame(w, h, (4, 4), seed=seed, frame_index=frame_index)
    secs = S.frame_sections(f)
    hdr = S.FrameHeader(frame_index, 3 * frame_index, 2, f.screen_size, f.num_tiles, f.num_training_records,
                        shuffle_seed=0xABCDEF0123)
    if extra:
        rng = np.random.default_rng(seed)
        secs[S.PERMUTATION] = rng.permutation(S.CAPACITY).astype(np.int32)
        secs[S.RESULTS_INFERENCE] = rng.normal(size=(f.screen_size + f.num_tiles, 3)).astype(np.float32)
        secs[S.OUTPUT_RGBA] = rng.normal(size=(f.screen_size, 4)).astype(np.float32)
        secs[S.LOSSES] = rng.normal(size=4).astype(np.float32)
    return hdr, secs


def test_numpy_writer_c_reader_roundtrip(nrc, tmp_path):
    S = nrc.stream
    p = tmp_path / "a.nrcs"
    frames = [_frame(nrc, seed=i, frame_index=i, extra=(i != 1)) for i in range(3)]
    with S.StreamWriter(p, 48, 32) as w:
        for h, secs in frames:
            w.write_frame(h, secs)
    with S.CStream(p) as cs:
        assert (cs.width, cs.height) == (48, 32)
        for h, secs in frames:
            got = cs.next_frame()
            assert got.frame_index == h.frame_index and got.num_training_records == h.num_training_records
            assert got.sections == sum(1 << k for k in secs)
            # read sections out of order, twice
            for sec in sorted(secs, reverse=True) + sorted(secs):
                a = cs.read_section(sec)
                assert a.tobytes() == np.ascontiguousarray(secs[sec]).tobytes(), S.SECTION_NAMES[sec]
            for missing in (k for k in range(S.SECTION_COUNT) if k not in secs):
                with pytest.raises(nrc.NrcError):
                    cs.read_section(missing)
        assert cs.next_frame() is None
        assert cs.next_frame() is None


def test_c_writer_numpy_reader_roundtrip(nrc, tmp_path):
    S = nrc.stream
    p = tmp_path / "b.nrcs"
    frames = [_frame(nrc, seed=7 + i, frame_index=i) for i in range(2)]
    with S.CStream(p, "w", 48, 32) as cs:
        for h, secs in frames:
            cs.write_frame(h, {k: np.ascontiguousarray(v) for k, v in secs.items()})
    got = list(S.read_stream(p))
    assert len(got) == 2
    for (h, secs), (gh, gsecs) in zip(frames, got):
        assert (gh.frame_index, gh.iteration_index, gh.render_mode, gh.shuffle_seed) == \
               (h.frame_index, h.iteration_index, h.render_mode, h.shuffle_seed)
        assert set(gsecs) == set(secs)
        for k in secs:
            assert gsecs[k].tobytes() == np.ascontiguousarray(secs[k]).tobytes()
    # byte-identical files from the two writers
    q = tmp_path / "c.nrcs"
    with S.StreamWriter(q, 48, 32) as w:
        for h, secs in frames:
            w.write_frame(h, secs)
    assert p.read_bytes() == q.read_bytes()


def test_section_bytes_agree(nrc):
    S = nrc.stream
    L = S._sigs()
    rng = np.random.default_rng(0)
    for _ in range(50):
        h = S.FrameHeader(0, 0, 0, int(rng.integers(0, 1 << 22)), int(rng.integers(0, 1 << 18)),
                          int(rng.integers(-5, 100000)))
        for sec in range(S.SECTION_COUNT):
            assert L.nrc_stream_section_bytes(ctypes.byref(S._to_c(h)), sec) == S.section_bytes(h, sec)


def test_corrupt_streams_rejected(nrc, tmp_path):
    S = nrc.stream
    p = tmp_path / "ok.nrcs"
    h, secs = _frame(nrc)
    with S.StreamWriter(p) as w:
        w.write_frame(h, secs)
    data = p.read_bytes()
    bad_magic = tmp_path / "bad_magic.nrcs"
    bad_magic.write_bytes(b"X" + data[1:])
    with pytest.raises(nrc.NrcError):
        S.CStream(bad_magic)
    truncated = tmp_path / "trunc.nrcs"
    truncated.write_bytes(data[:-100])
    with S.CStream(truncated) as cs:
        cs.next_frame()
        with pytest.raises(nrc.NrcError):
            cs.read_section(S.LOSSES)  # the last section runs past the end of the file
    bad_tag = tmp_path / "bad_tag.nrcs"
    bad_tag.write_bytes(data[:64] + b"XXXX" + data[68:])
    with S.CStream(bad_tag) as cs, pytest.raises(nrc.NrcError):
        cs.next_frame()
    with pytest.raises(nrc.NrcError):
        S.CStream(tmp_path / "missing.nrcs")
    empty = tmp_path / "empty.nrcs"
    with S.StreamWriter(empty):
        pass
    with S.CStream(empty) as cs:
        assert cs.next_frame() is None
    assert list(S.read_stream(empty)) == []


def test_record_synthetic_stream(nrc, tmp_path):
    S = nrc.stream
    p = tmp_path / "syn.nrcs"
    S.record_synthetic(p, 3, 64, 48, seed=5)
    frames = list(S.read_stream(p))
    assert [h.frame_index for h, _ in frames] == [0, 1, 2]
    f1 = nrc.synthetic.cornell_frame(64, 48, (4, 4), seed=5, frame_index=1)
    h, secs = frames[1]
    np.testing.assert_array_equal(secs[S.QUERIES_INFERENCE], f1.queries_inference)
    assert secs[S.TRAIN_RECORDS].tobytes() == f1.train_records[: h.nrec].tobytes()


def test_padded_query_layout_roundtrip(nrc, tmp_path):
    """A stream of padded RadianceQuery records (nrc_stream_create_layout, USE_COMPACT_RADIANCE_QUERY 0): the file header
    says 64-byte queries, the query sections are 16 floats wide, the reader reports the layout and returns the bytes."""
    S = nrc.stream
    p = tmp_path / "padded.nrcs"
    h, secs = _frame(nrc, seed=3, frame_index=1)
    for k in (S.QUERIES_INFERENCE, S.QUERIES_CACHE_VIS, S.TRAIN_QUERIES):
        q = np.asarray(secs[k], np.float32)
        secs[k] = np.ascontiguousarray(np.insert(q, 3, np.arange(len(q), dtype=np.float32), axis=1))
    with S.CStream(p, "w", 48, 32, query_layout=1) as cs:
        assert cs.query_layout == 1
        cs.write_frame(h, secs)
    assert int.from_bytes(p.read_bytes()[16:20], "little") == 64  # query_bytes in the file header
    with S.CStream(p) as cs:
        assert cs.query_layout == 1 and cs.query_dims == 16
        got = cs.next_frame()
        assert got.sections == sum(1 << k for k in secs)
        for k in secs:
            assert cs.read_section(k).tobytes() == np.ascontiguousarray(secs[k]).tobytes(), S.SECTION_NAMES[k]
    with pytest.raises(nrc.NrcError):
        S.CStream(tmp_path / "x.nrcs", "w", query_layout=2)
