"""Recorded NRC sample streams (include/nrc/stream.h) and the frame replayer.

* ``StreamWriter`` / ``read_stream``: the file format in numpy (an independent implementation of the
  layout the C-ABI reader/writer in csrc/nrc_stream.cpp implements; tests cross-check the two).
* ``CStream``: the C-ABI reader/writer (what a C++ renderer links), for host or device buffers.
* ``replay``: feeds every recorded frame through ``nrc_process_frame`` (infer -> accumulate ->
  propagate -> shuffle -> 4 x train) on the GPU, the stand-in for the reference's ``Device::render``
  after the OptiX trace (/root/reference/nrc/src/Device.cpp:2493-2515).
* ``record_synthetic``: writes a synthetic Cornell frame sequence (synthetic.cornell_frame).
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass, field

import numpy as np

from ._lib import check, lib
from .frame import (END_VERTEX_DTYPE, NUM_BATCHES, NUM_TRAINING_RECORDS_PER_FRAME, TRAINING_RECORD_DTYPE,
                    FrameBuffers, FrameParams, RenderMode, process_frame)

VERSION = 1
MAGIC = b"NRCSTRM\0"
FRAME_TAG = b"FRME"
CAPACITY = NUM_TRAINING_RECORDS_PER_FRAME

(QUERIES_INFERENCE, LAST_RENDER_THROUGHPUT, QUERIES_CACHE_VIS, END_VERTICES, TRAIN_RECORDS, TRAIN_QUERIES,
 TRAIN_TARGETS, PERMUTATION, RESULTS_INFERENCE, OUTPUT_RGBA, LOSSES, SHUFFLE_KEYS) = range(12)
SECTION_COUNT = 12
SECTION_NAMES = ["queries_inference", "last_render_throughput", "queries_cache_vis", "end_vertices",
                 "train_records", "train_queries", "train_targets", "permutation", "results_inference",
                 "output_rgba", "losses", "shuffle_keys"]

_FILE_HDR = struct.Struct("<8s10I2Q")       # 64 B
_FRAME_HDR = struct.Struct("<4s2Ii2IiI4x2Q12x")  # tag + nrc_stream_frame_header (48) + 12 pad = 64 B
assert _FILE_HDR.size == 64 and _FRAME_HDR.size == 64


@dataclass
class FrameHeader:
    """nrc_stream_frame_header (include/nrc/stream.h)."""
    frame_index: int = 0
    iteration_index: int = 0
    render_mode: int = int(RenderMode.Full)
    screen_size: int = 0
    num_tiles: int = 0
    num_training_records: int = 0
    sections: int = 0
    shuffle_seed: int = 0
    payload_bytes: int = 0

    @property
    def nrec(self) -> int:
        return max(0, min(self.num_training_records, CAPACITY))


def section_shape(h: FrameHeader, sec: int, query_dims: int = 15):
    """(count, dtype, row shape) of a section (query_dims: 15 compact / 16 padded RadianceQuery records)."""
    s, t, n, qd = h.screen_size, h.num_tiles, h.nrec, int(query_dims)
    return {
        QUERIES_INFERENCE: (s + t, np.float32, (qd,)), LAST_RENDER_THROUGHPUT: (s, np.float32, (3,)),
        QUERIES_CACHE_VIS: (s, np.float32, (qd,)), END_VERTICES: (t, END_VERTEX_DTYPE, ()),
        TRAIN_RECORDS: (n, TRAINING_RECORD_DTYPE, ()), TRAIN_QUERIES: (n, np.float32, (qd,)),
        TRAIN_TARGETS: (n, np.float32, (3,)), PERMUTATION: (CAPACITY, np.int32, ()),
        RESULTS_INFERENCE: (s + t, np.float32, (3,)), OUTPUT_RGBA: (s, np.float32, (4,)),
        LOSSES: (NUM_BATCHES, np.float32, ()), SHUFFLE_KEYS: (CAPACITY, np.uint32, ()),
    }[sec]


def section_bytes(h: FrameHeader, sec: int) -> int:
    n, dt, row = section_shape(h, sec)
    return int(n) * np.dtype(dt).itemsize * int(np.prod(row, dtype=np.int64))


class StreamWriter:
    """numpy writer of the stream format."""

    def __init__(self, path, width: int = 0, height: int = 0):
        self._f = open(path, "wb")
        self._f.write(_FILE_HDR.pack(MAGIC, VERSION, 64, 60, 28, 16, 12, width, height, CAPACITY, 0, 0, 0))

    def write_frame(self, header: FrameHeader, sections: dict[int, np.ndarray]) -> None:
        h = FrameHeader(**{**header.__dict__})
        h.sections, h.payload_bytes = 0, 0
        blobs = []
        for sec in range(SECTION_COUNT):
            a = sections.get(sec)
            if a is None:
                continue
            n, dt, row = section_shape(h, sec)
            a = np.ascontiguousarray(a, dtype=dt).reshape((n,) + row)
            h.sections |= 1 << sec
            h.payload_bytes += a.nbytes
            blobs.append(a)
        self._f.write(_FRAME_HDR.pack(FRAME_TAG, h.frame_index, h.iteration_index, h.render_mode,
                                      h.screen_size, h.num_tiles, h.num_training_records, h.sections,
                                      h.shuffle_seed, h.payload_bytes))
        for a in blobs:
            self._f.write(a.tobytes())

    def close(self) -> None:
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_stream(path):
    """Yield (FrameHeader, {section: array}) for every frame; arrays are views of a memory map."""
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    magic, version, hb, qb, rb, evb, f3b, w, h_, cap, *_ = _FILE_HDR.unpack(bytes(mm[:64]))
    if magic != MAGIC or version != VERSION or (hb, qb, rb, evb, f3b, cap) != (64, 60, 28, 16, 12, CAPACITY):
        raise ValueError(f"{path}: not a version-{VERSION} NRC stream")
    off = 64
    while off < len(mm):
        tag, fi, it, mode, scr, tiles, nrec, secs, seed, payload = _FRAME_HDR.unpack(bytes(mm[off:off + 64]))
        if tag != FRAME_TAG:
            raise ValueError(f"{path}: corrupt frame tag at {off}")
        h = FrameHeader(fi, it, mode, scr, tiles, nrec, secs, seed, payload)
        off += 64
        out, p = {}, off
        for sec in range(SECTION_COUNT):
            if secs & (1 << sec):
                n, dt, row = section_shape(h, sec)
                nb = section_bytes(h, sec)
                out[sec] = np.frombuffer(mm, dtype=np.uint8, count=nb, offset=p).view(dt).reshape((n,) + row)
                p += nb
        if p - off > payload:
            raise ValueError(f"{path}: frame payload shorter than its sections")
        off += payload
        yield h, out


# ---- C-ABI reader / writer ----------------------------------------------------------------------------
class _CHeader(ctypes.Structure):
    _fields_ = [("frame_index", ctypes.c_uint32), ("iteration_index", ctypes.c_uint32),
                ("render_mode", ctypes.c_int32), ("screen_size", ctypes.c_uint32), ("num_tiles", ctypes.c_uint32),
                ("num_training_records", ctypes.c_int32), ("sections", ctypes.c_uint32),
                ("query_layout", ctypes.c_uint32), ("shuffle_seed", ctypes.c_uint64), ("payload_bytes", ctypes.c_uint64)]


def _sigs():
    L = lib()
    if getattr(L, "_stream_sigs", False):
        return L
    vp, u32, st = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.nrc_stream_section_bytes.restype = ctypes.c_uint64
    L.nrc_stream_section_bytes.argtypes = [ctypes.POINTER(_CHeader), ctypes.c_int]
    for name, args in {
        "nrc_stream_create": [ctypes.c_char_p, u32, u32, ctypes.POINTER(vp)],
        "nrc_stream_create_layout": [ctypes.c_char_p, u32, u32, u32, ctypes.POINTER(vp)],
        "nrc_stream_query_layout": [vp, ctypes.POINTER(u32)],
        "nrc_stream_open": [ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(u32), ctypes.POINTER(u32)],
        "nrc_stream_close": [vp],
        "nrc_stream_write_frame": [vp, ctypes.POINTER(_CHeader), ctypes.POINTER(vp), vp],
        "nrc_stream_next_frame": [vp, ctypes.POINTER(_CHeader), ctypes.POINTER(ctypes.c_int)],
        "nrc_stream_read_section": [vp, ctypes.c_int, vp, vp],
    }.items():
        fn = getattr(L, name)
        fn.restype = st
        fn.argtypes = args
    L._stream_sigs = True
    return L


def _addr(x) -> int:
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        assert x.flags.c_contiguous
        return x.ctypes.data
    return int(x.data_ptr())


def _to_c(h: FrameHeader) -> _CHeader:
    return _CHeader(h.frame_index, h.iteration_index, h.render_mode, h.screen_size, h.num_tiles,
                    h.num_training_records, h.sections, 0, h.shuffle_seed, h.payload_bytes)


def _from_c(c: _CHeader) -> FrameHeader:
    return FrameHeader(c.frame_index, c.iteration_index, c.render_mode, c.screen_size, c.num_tiles,
                       c.num_training_records, c.sections, c.shuffle_seed, c.payload_bytes)


class CStream:
    """The C-ABI stream (csrc/nrc_stream.cpp). Buffers may be numpy arrays or device tensors / addresses.
    query_layout (writing): 0 compact (15-float records), 1 padded (16-float, USE_COMPACT_RADIANCE_QUERY 0); a reader
    takes it from the file."""

    def __init__(self, path, mode: str = "r", width: int = 0, height: int = 0, query_layout: int = 0):
        L = _sigs()
        self._h = ctypes.c_void_p()
        if mode == "w":
            check(L.nrc_stream_create_layout(str(path).encode(), width, height, int(query_layout),
                                             ctypes.byref(self._h)))
            self.width, self.height = width, height
        else:
            w, h = ctypes.c_uint32(), ctypes.c_uint32()
            check(L.nrc_stream_open(str(path).encode(), ctypes.byref(self._h), ctypes.byref(w), ctypes.byref(h)))
            self.width, self.height = w.value, h.value
        ql = ctypes.c_uint32()
        check(L.nrc_stream_query_layout(self._h, ctypes.byref(ql)))
        self.query_layout = ql.value
        self.query_dims = 16 if ql.value == 1 else 15
        self._cur = None

    def write_frame(self, header: FrameHeader, sections: dict, stream=None) -> None:
        ptrs = (ctypes.c_void_p * SECTION_COUNT)()
        for sec, a in sections.items():
            if a is not None:
                ptrs[sec] = _addr(a)
        s = None if stream is None else int(getattr(stream, "cuda_stream", stream))
        check(_sigs().nrc_stream_write_frame(self._h, ctypes.byref(_to_c(header)), ptrs, s))

    def next_frame(self) -> FrameHeader | None:
        c, eos = _CHeader(), ctypes.c_int()
        check(_sigs().nrc_stream_next_frame(self._h, ctypes.byref(c), ctypes.byref(eos)))
        self._cur = None if eos.value else _from_c(c)
        return self._cur

    def read_section(self, sec: int, dst=None, stream=None):
        """Into dst (numpy array / device tensor / address); with dst None a new numpy array is returned."""
        if dst is None:
            n, dt, row = section_shape(self._cur, sec, self.query_dims)
            dst = np.empty((n,) + row, dtype=dt)
        s = None if stream is None else int(getattr(stream, "cuda_stream", stream))
        check(_sigs().nrc_stream_read_section(self._h, sec, _addr(dst), s))
        return dst

    def close(self) -> None:
        if self._h:
            check(_sigs().nrc_stream_close(self._h))
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ---- synthetic recording and replay ------------------------------------------------------------------
def frame_sections(f) -> dict[int, np.ndarray]:
    """A synthetic.SyntheticFrame as stream sections (trace outputs only)."""
    n = min(f.num_training_records, CAPACITY)
    return {QUERIES_INFERENCE: f.queries_inference, LAST_RENDER_THROUGHPUT: f.last_render_throughput,
            QUERIES_CACHE_VIS: f.queries_cache_vis, END_VERTICES: f.end_vertices,
            TRAIN_RECORDS: f.train_records[:n], TRAIN_QUERIES: f.train_queries[:n],
            TRAIN_TARGETS: f.train_targets[:n]}


def record_synthetic(path, frames: int, width: int = 320, height: int = 240, tile=(4, 4), seed: int = 0,
                     render_mode: RenderMode = RenderMode.Full, shuffle_seed: int = 1) -> None:
    from .synthetic import cornell_frame
    with StreamWriter(path, width, height) as w:
        for i in range(frames):
            f = cornell_frame(width, height, tile, seed=seed, frame_index=i)
            w.write_frame(FrameHeader(i, i, int(render_mode), f.screen_size, f.num_tiles, f.num_training_records,
                                      shuffle_seed=shuffle_seed), frame_sections(f))


@dataclass
class ReplayResult:
    losses: list = field(default_factory=list)
    results_inference: list = field(default_factory=list)  # per frame, when keep_outputs
    output_rgba: np.ndarray | None = None
    mismatches: dict = field(default_factory=dict)         # section name -> max |diff| vs recorded


class Replayer:
    """Device buffers sized for a stream, reused across its frames (the reference's ControlBlock)."""

    def __init__(self, device, max_screen: int, max_tiles: int):
        import torch
        self.dev = device
        z = lambda *s, dtype=torch.float32: torch.zeros(s, dtype=dtype, device=device)  # noqa: E731
        self.queries_inference = z(max_screen + max_tiles, 15)
        self.results_inference = z(max_screen + max_tiles, 3)
        self.last_render_throughput = z(max_screen, 3)
        self.output_rgba = z(max_screen, 4)
        self.queries_cache_vis = z(max_screen, 15)
        self.results_cache_vis = z(max_screen, 3)
        self.end_vertices = z(max_tiles, 4, dtype=torch.int32)
        self.train_records = z(CAPACITY, 7, dtype=torch.int32)
        self.train_queries = [z(CAPACITY, 15), z(CAPACITY, 15)]
        self.train_targets = [z(CAPACITY, 3), z(CAPACITY, 3)]
        self.permutation = z(CAPACITY, dtype=torch.int32)
        self.shuffle_keys = z(CAPACITY, dtype=torch.int32)  # u32 keys, held as int32 bytes

    def buffers(self, has_perm: bool, has_keys: bool = False) -> FrameBuffers:
        return FrameBuffers(self.queries_inference, self.results_inference, self.last_render_throughput,
                            self.output_rgba, self.end_vertices, self.train_records, self.train_queries,
                            self.train_targets, self.queries_cache_vis, self.results_cache_vis,
                            self.permutation if has_perm else None, self.shuffle_keys if has_keys else None)


def replay(path, net, device, keep_outputs: bool = False, loss: bool = True) -> ReplayResult:
    """Replay every frame of a recorded stream through the network (process_frame), reading sections with the
    C-ABI reader straight into device buffers. The frame buffer accumulates across frames, as in the renderer."""
    import torch
    # size the device buffers from the headers (one pass over the headers only)
    hdrs = []
    with CStream(path) as cs:
        while (h := cs.next_frame()) is not None:
            hdrs.append(h)
    if not hdrs:
        return ReplayResult()
    rp = Replayer(device, max(h.screen_size for h in hdrs), max(h.num_tiles for h in hdrs))
    res = ReplayResult()
    targets = {QUERIES_INFERENCE: rp.queries_inference, LAST_RENDER_THROUGHPUT: rp.last_render_throughput,
               QUERIES_CACHE_VIS: rp.queries_cache_vis, END_VERTICES: rp.end_vertices,
               TRAIN_RECORDS: rp.train_records, TRAIN_QUERIES: rp.train_queries[0],
               TRAIN_TARGETS: rp.train_targets[0], PERMUTATION: rp.permutation, SHUFFLE_KEYS: rp.shuffle_keys}
    stream = torch.cuda.current_stream()
    with CStream(path) as cs:
        while (h := cs.next_frame()) is not None:
            # Device::render zeroes the targets before the trace (Device.cpp:2471-2476)
            rp.train_targets[0].zero_()
            for sec, dst in targets.items():
                if h.sections & (1 << sec):
                    cs.read_section(sec, dst, stream)
            l = process_frame(net, rp.buffers(bool(h.sections & (1 << PERMUTATION)), bool(h.sections & (1 << SHUFFLE_KEYS))),
                              FrameParams(h.screen_size, h.num_tiles, h.num_training_records,
                                          RenderMode(h.render_mode), h.iteration_index, h.frame_index,
                                          h.shuffle_seed), loss=loss)
            res.losses.append(l)
            n = h.screen_size + h.num_tiles
            if keep_outputs:
                res.results_inference.append(rp.results_inference[:n].cpu().numpy())
            if h.sections & (1 << RESULTS_INFERENCE):
                rec = torch.from_numpy(cs.read_section(RESULTS_INFERENCE)).to(device)
                d = float((rp.results_inference[:n] - rec).abs().max())
                res.mismatches["results_inference"] = max(res.mismatches.get("results_inference", 0.0), d)
    torch.cuda.synchronize()
    res.output_rgba = rp.output_rgba[: hdrs[-1].screen_size].cpu().numpy()
    return res
