"""GPU side of the recorded sample stream: sections stream straight into / out of
device buffers, and a recorded frame sequence replays bit-identically through the Python replayer and the
C++ stand-in renderer (neural-radiance-caching_amd/nrc_replay)."""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
REPLAY_BIN = ROOT / "neural-radiance-caching_amd" / "nrc_replay"


def test_device_sections_roundtrip(nrc, dev, tmp_path):
    import torch
    S = nrc.stream
    p = tmp_path / "h.nrcs"
    S.record_synthetic(p, 2, 96, 64, seed=3)
    host = list(S.read_stream(p))
    # read into device buffers
    with S.CStream(p) as cs:
        for h, secs in host:
            assert cs.next_frame() == h
            for sec, a in secs.items():
                d = torch.empty(a.nbytes // 4, dtype=torch.int32, device=dev)
                cs.read_section(sec, d, torch.cuda.current_stream())
                torch.cuda.synchronize()
                assert d.cpu().numpy().tobytes() == a.tobytes()
    # record from device buffers (the renderer's dump points) -> identical file
    q = tmp_path / "d.nrcs"
    with S.CStream(q, "w", 96, 64) as cs:
        for h, secs in host:
            cs.write_frame(h, {k: torch.from_numpy(np.array(v).view(np.uint8)).to(dev)
                               for k, v in secs.items()}, torch.cuda.current_stream())
    assert q.read_bytes() == p.read_bytes()


def _fresh_net(nrc):
    import torch
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    return net


def test_replay_python_matches_cpp_replayer(nrc, dev, tmp_path):
    """The same recorded frames through the Python replayer and the C++ replayer: identical losses, radiance and
    frame buffer (both drive nrc_process_frame from the same C-ABI; kernels are deterministic)."""
    assert REPLAY_BIN.exists(), "nrc_replay not built (make -C neural-radiance-caching_amd)"
    S = nrc.stream
    p = tmp_path / "r.nrcs"
    S.record_synthetic(p, 4, 320, 240, seed=9)
    net = _fresh_net(nrc)
    res = S.replay(p, net, dev, keep_outputs=True)
    assert net.step == 16 and all(np.isfinite(res.losses))
    net.destroy()

    out_f, res_f = tmp_path / "out.f32", tmp_path / "res.f32"
    r = subprocess.run([str(REPLAY_BIN), str(p), "--dump-output", str(out_f), "--dump-results", str(res_f)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines()]
    cpp_losses = [x["loss"] for x in lines if "frame" in x]
    assert lines[-1]["train_steps"] == 16
    np.testing.assert_array_equal(np.float32(cpp_losses), np.float32(res.losses))
    np.testing.assert_array_equal(np.fromfile(out_f, np.float32).reshape(-1, 4), res.output_rgba)
    np.testing.assert_array_equal(np.fromfile(res_f, np.float32).reshape(-1, 3), res.results_inference[-1])


def test_replay_reproduces_recorded_outputs(nrc, dev, tmp_path):
    """Record a replay's outputs into the stream (RESULTS_INFERENCE / LOSSES sections), replay again from a fresh
    network: the recorded radiance is reproduced exactly."""
    S = nrc.stream
    p = tmp_path / "a.nrcs"
    S.record_synthetic(p, 3, 160, 120, seed=1)
    net = _fresh_net(nrc)
    first = S.replay(p, net, dev, keep_outputs=True)
    net.destroy()
    q = tmp_path / "b.nrcs"
    with S.StreamWriter(q, 160, 120) as w:
        for i, (h, secs) in enumerate(S.read_stream(p)):
            secs = dict(secs)
            secs[S.RESULTS_INFERENCE] = first.results_inference[i]
            secs[S.LOSSES] = np.full(4, first.losses[i], np.float32)
            w.write_frame(h, secs)
    net = _fresh_net(nrc)
    second = S.replay(q, net, dev)
    net.destroy()
    assert second.mismatches["results_inference"] == 0.0
    assert second.losses == first.losses


def test_replay_with_recorded_permutation_and_modes(nrc, dev, tmp_path):
    """A caller-made permutation recorded in the stream is used as is; NoCache frames leave the frame buffer alone."""
    import torch
    S = nrc.stream
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(128, 96, (4, 4), seed=4)
    perm = np.random.default_rng(2).permutation(S.CAPACITY).astype(np.int32)
    p = tmp_path / "p.nrcs"
    with S.StreamWriter(p) as w:
        secs = S.frame_sections(f)
        secs[S.PERMUTATION] = perm
        w.write_frame(S.FrameHeader(0, 0, int(F.RenderMode.NoCache), f.screen_size, f.num_tiles,
                                    f.num_training_records), secs)
    net = _fresh_net(nrc)
    rp_res = S.replay(p, net, dev)
    assert np.all(rp_res.output_rgba == 0.0)  # NoCache: never accumulated
    # the same frame through process_frame with the permutation passed explicitly: identical weights
    cap = S.CAPACITY
    nrec = min(f.num_training_records, cap)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    pad = lambda a, w: np.concatenate([a[:nrec], np.zeros((cap - nrec, w), np.float32)])  # noqa: E731
    rec = np.zeros(cap, F.TRAINING_RECORD_DTYPE)
    rec[:nrec] = f.train_records[:nrec]
    fb = F.FrameBuffers(t(f.queries_inference), torch.zeros((f.screen_size + f.num_tiles, 3), device=dev),
                        t(f.last_render_throughput), torch.zeros((f.screen_size, 4), device=dev),
                        F.records_to_device(f.end_vertices, dev), F.records_to_device(rec, dev),
                        [t(pad(f.train_queries, 15)), torch.zeros((cap, 15), device=dev)],
                        [t(pad(f.train_targets, 3)), torch.zeros((cap, 3), device=dev)], permutation=t(perm))
    net2 = _fresh_net(nrc)
    F.process_frame(net2, fb, F.FrameParams(f.screen_size, f.num_tiles, f.num_training_records,
                                            F.RenderMode.NoCache))
    np.testing.assert_array_equal(net.get_state(nrc.StateSlot.PARAMS), net2.get_state(nrc.StateSlot.PARAMS))
    np.testing.assert_array_equal(fb.train_queries[1].cpu().numpy(), pad(f.train_queries, 15)[perm % nrec])
    net.destroy()
    net2.destroy()


def test_replay_ranks1_rccl_matches_plain_replay(nrc, dev, tmp_path):
    """nrc_replay --ranks 1 (a forked rank with a world-1 RCCL communicator, nrc_process_frame_shard + nrc_train_dp)
    reproduces the plain replay bit for bit: losses, frame buffer and radiance."""
    S = nrc.stream
    p = tmp_path / "k.nrcs"
    S.record_synthetic(p, 3, 160, 120, seed=5)
    outs = {}
    for mode, extra in (("plain", []), ("ranks1", ["--ranks", "1"])):
        out_f, res_f = tmp_path / f"out_{mode}.f32", tmp_path / f"res_{mode}.f32"
        r = subprocess.run([str(REPLAY_BIN), str(p), "--dump-output", str(out_f), "--dump-results", str(res_f)] + extra,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]  # RCCL may log to stdout
        assert lines[-1]["train_steps"] == 12 and lines[-1]["world"] == 1
        outs[mode] = ([x["loss"] for x in lines if "frame" in x], out_f.read_bytes(), res_f.read_bytes())
    assert outs["plain"][0] == outs["ranks1"][0]
    assert outs["plain"][1] == outs["ranks1"][1] and outs["plain"][2] == outs["ranks1"][2]


def test_cpp_replayer_padded_stream_equals_compact(nrc, dev, tmp_path):
    """A stream of padded RadianceQuery records (USE_COMPACT_RADIANCE_QUERY 0, pad_ = 1.0 in every record) replays
    through nrc_replay -- which sizes its buffers and makes its handle from the stream's query layout -- with losses,
    radiance and frame buffer bitwise those of the compact stream of the same frames: a padded handle with pad_ = 1
    computes what a compact handle computes (tests/test_gpu_padded.py), and both start from the same seeded weights."""
    assert REPLAY_BIN.exists(), "nrc_replay not built (make -C neural-radiance-caching_amd)"
    S = nrc.stream
    p, q = tmp_path / "compact.nrcs", tmp_path / "padded.nrcs"
    S.record_synthetic(p, 3, 160, 120, seed=4)
    with S.CStream(q, "w", 160, 120, query_layout=1) as cs:
        for h, secs in S.read_stream(p):
            for k in (S.QUERIES_INFERENCE, S.QUERIES_CACHE_VIS, S.TRAIN_QUERIES):
                if k in secs:
                    a = np.asarray(secs[k], np.float32)
                    secs[k] = np.ascontiguousarray(np.insert(a, 3, np.float32(1.0), axis=1))
            cs.write_frame(h, {k: np.ascontiguousarray(v) for k, v in secs.items()})
    outs = []
    for path in (p, q):
        out_f, res_f = tmp_path / (path.stem + ".out"), tmp_path / (path.stem + ".res")
        r = subprocess.run([str(REPLAY_BIN), str(path), "--dump-output", str(out_f), "--dump-results", str(res_f)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        losses = [json.loads(x)["loss"] for x in r.stdout.splitlines() if '"frame"' in x]
        outs.append((losses, np.fromfile(out_f, np.float32), np.fromfile(res_f, np.float32)))
    assert len(outs[0][0]) == 3 and all(np.isfinite(outs[0][0]))
    assert outs[0][0] == outs[1][0]
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    np.testing.assert_array_equal(outs[0][2], outs[1][2])
