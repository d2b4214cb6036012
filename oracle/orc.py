"""ctypes binding of the C oracle (oracle/nrc_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker. The product package never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liborc.so"

FP32, MIXED, TCNN, FP8 = 0, 1, 2, 3
NUM_PARAMS = 22528
WIDE_NUM_PARAMS = 77824

_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        fp = ctypes.POINTER(ctypes.c_float)
        L.orc_f16_round.restype = ctypes.c_float
        L.orc_f16_round.argtypes = [ctypes.c_float]
        L.orc_encode.argtypes = [fp, ctypes.c_int64, fp]
        L.orc_forward.argtypes = [fp, fp, ctypes.c_int64, ctypes.c_int, fp, ctypes.c_int]
        L.orc_grad.restype = ctypes.c_double
        L.orc_grad.argtypes = [fp, fp, fp, ctypes.c_int64, ctypes.c_double, ctypes.c_float,
                               ctypes.c_int, fp, ctypes.c_int]
        L.orc_adam_ema.argtypes = [fp, fp, fp, fp, fp, ctypes.c_uint32, fp, ctypes.c_float,
                                   ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                   ctypes.c_float, ctypes.c_float, ctypes.c_int64]
        L.orc_init_params.argtypes = [fp, ctypes.c_uint64]
        L.orc_encode_sh.argtypes = [fp, ctypes.c_int64, fp]
        L.orc_encode_padded.argtypes = [fp, ctypes.c_int64, fp]
        L.orc_forward_enc.argtypes = [ctypes.c_int, fp, fp, ctypes.c_int64, ctypes.c_int, fp, ctypes.c_int]
        L.orc_grad_enc.restype = ctypes.c_double
        L.orc_grad_enc.argtypes = [ctypes.c_int, fp, fp, fp, ctypes.c_int64, ctypes.c_double, ctypes.c_float,
                                   ctypes.c_int, fp, ctypes.c_int]
        vp, u32, u64, i64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64
        L.orc_accumulate.argtypes = [vp, vp, vp, i64, ctypes.c_int, u32]
        L.orc_propagate.argtypes = [vp, vp, i64, vp, vp, i64]
        L.orc_accumulate_factored.argtypes = [vp, vp, vp, vp, i64, ctypes.c_int, u32]
        L.orc_propagate_factored.argtypes = [vp, vp, vp, i64, vp, vp, vp, i64]
        L.orc_feistel_keys.argtypes = [u64, u32, vp]
        L.orc_permutation.argtypes = [u64, u32, vp, u32]
        L.orc_sort_pairs.argtypes = [vp, vp, vp, u32]
        L.orc_permute.argtypes = [vp, vp, vp, u64, u32, ctypes.c_int32, vp, vp, u32]
        L.orc_hash_encode.argtypes = [vp, vp, i64, ctypes.c_int, vp]
        L.orc_hash_forward.argtypes = [vp, vp, i64, ctypes.c_int, vp, ctypes.c_int]
        L.orc_hash_grad.restype = ctypes.c_double
        L.orc_hash_grad.argtypes = [vp, vp, vp, i64, ctypes.c_double, ctypes.c_float, ctypes.c_int, vp, ctypes.c_int]
        L.orc_hash_forward_layout.argtypes = [ctypes.c_int, vp, vp, i64, ctypes.c_int, vp, ctypes.c_int]
        L.orc_hash_grad_layout.restype = ctypes.c_double
        L.orc_hash_grad_layout.argtypes = [ctypes.c_int, vp, vp, vp, i64, ctypes.c_double, ctypes.c_float, ctypes.c_int,
                                           vp, ctypes.c_int]
        L.orc_hash_adam_ema.argtypes = [vp, vp, vp, vp, vp, vp, u32, vp] + [ctypes.c_float] * 7
        L.orc_hash_init_params.argtypes = [vp, u64]
        L.orc_hash_corners.argtypes = [vp, ctypes.c_int, vp, vp]
        L.orc_f16_round_double.restype = ctypes.c_float
        L.orc_f16_round_double.argtypes = [ctypes.c_double]
        L.orc_wide_forward.argtypes = [ctypes.c_int, vp, vp, i64, ctypes.c_int, vp, ctypes.c_int]
        L.orc_e4m3.restype = ctypes.c_float
        L.orc_e4m3.argtypes = [ctypes.c_float]
        L.orc_fp8_row_exponent.restype = ctypes.c_int
        L.orc_fp8_row_exponent.argtypes = [ctypes.c_float]
        L.orc_wide_quantize.argtypes = [vp, vp, vp]
        L.orc_wide_grad.restype = ctypes.c_double
        L.orc_wide_grad.argtypes = [ctypes.c_int, vp, vp, vp, i64, ctypes.c_double, ctypes.c_float, ctypes.c_int, vp,
                                    ctypes.c_int]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def host_cores() -> tuple[int, str]:
    """Host cores this process may use: the CPUs of its affinity mask, bounded by a cgroup-v2 CPU quota when one is
    set (a quota of Q us per P us runs at most ceil(Q / P) threads at a time). Returns (cores, how it was found)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = f"{aff} CPUs in the affinity mask"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
            if quota < aff:
                how += f", cgroup cpu.max quota {quota}"
                aff = quota
    except (OSError, ValueError):
        pass
    return max(1, min(256, aff)), how  # nrc_oracle.c runs at most 256 pthreads


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def default_threads() -> int:
    return host_cores()[0]


def encode(queries: np.ndarray) -> np.ndarray:
    q = np.ascontiguousarray(queries, dtype=np.float32)
    n = q.shape[0]
    out = np.empty((n, 80), dtype=np.float32)
    if n:
        lib().orc_encode(_p(q), n, _p(out))
    return out


FREQUENCY, HASH, FREQUENCY_SH = 0, 1, 2
# encoding kind flag: non-compact 16-float RadianceQuery records (USE_COMPACT_RADIANCE_QUERY 0; ORC_KIND_PADDED)
PADDED = 16


def encode_padded(queries: np.ndarray) -> np.ndarray:
    """[n][16] non-compact queries -> [n][80] in the reference's padded order (nrc_oracle.c orc_encode_padded)."""
    q = np.ascontiguousarray(queries, dtype=np.float32)
    out = np.empty((q.shape[0], 80), dtype=np.float32)
    if q.shape[0]:
        lib().orc_encode_padded(_p(q), q.shape[0], _p(out))
    return out


def encode_sh(queries: np.ndarray) -> np.ndarray:
    q = np.ascontiguousarray(queries, dtype=np.float32)
    out = np.empty((q.shape[0], 80), dtype=np.float32)
    if q.shape[0]:
        lib().orc_encode_sh(_p(q), q.shape[0], _p(out))
    return out


def forward(params: np.ndarray, queries: np.ndarray, mode: int = MIXED, threads: int | None = None,
            encoding: int = FREQUENCY) -> np.ndarray:
    q = np.ascontiguousarray(queries, dtype=np.float32)
    p = np.ascontiguousarray(params, dtype=np.float32)
    n = q.shape[0]
    out = np.zeros((n, 3), dtype=np.float32)
    if n:
        lib().orc_forward_enc(encoding, _p(p), _p(q), n, mode, _p(out), threads or default_threads())
    return out


def grad(params, queries, targets, n_total=None, loss_scale=128.0, mode=MIXED, threads=None, encoding=FREQUENCY):
    q = np.ascontiguousarray(queries, dtype=np.float32)
    t = np.ascontiguousarray(targets, dtype=np.float32)
    p = np.ascontiguousarray(params, dtype=np.float32)
    b = q.shape[0]
    if n_total is None:
        n_total = 3.0 * b
    g = np.zeros(NUM_PARAMS, dtype=np.float32)
    loss = lib().orc_grad_enc(encoding, _p(p), _p(q), _p(t), b, float(n_total), float(loss_scale), mode, _p(g),
                              threads or default_threads())
    return g, float(loss)


class AdamEmaState:
    """tcnn Adam + EMA optimizer state, restated (oracle/nrc_oracle.c orc_adam_ema)."""

    def __init__(self, params: np.ndarray, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, l2_reg=1e-6,
                 ema_decay=0.99, loss_scale=128.0):
        self.params = np.array(params, dtype=np.float32)
        self.m = np.zeros_like(self.params)
        self.v = np.zeros_like(self.params)
        self.ema = np.zeros_like(self.params)
        self.infer = self.params.copy()
        self.step = 0
        self.lr, self.beta1, self.beta2, self.eps = lr, beta1, beta2, eps
        self.l2_reg, self.ema_decay, self.loss_scale = l2_reg, ema_decay, loss_scale

    def apply(self, g: np.ndarray) -> None:
        self.step += 1
        g = np.ascontiguousarray(g, dtype=np.float32)
        lib().orc_adam_ema(_p(self.params), _p(self.m), _p(self.v), _p(self.ema), _p(self.infer),
                           self.step, _p(g), self.loss_scale, self.lr, self.beta1, self.beta2,
                           self.eps, self.l2_reg, self.ema_decay, self.params.size)


def init_params(seed: int = 1337) -> np.ndarray:
    p = np.empty(NUM_PARAMS, dtype=np.float32)
    lib().orc_init_params(_p(p), seed)
    return p


def f16_round(x: float) -> float:
    return lib().orc_f16_round(x)


# ---- per-frame kernels around the network (oracle/nrc_frame_oracle.c) -----------------------------
def _v(a: np.ndarray) -> int:
    assert a.flags.c_contiguous
    return a.ctypes.data


def accumulate(radiance: np.ndarray, throughput: np.ndarray, rgba: np.ndarray, mode: int,
               iteration_index: int, queries: np.ndarray | None = None) -> np.ndarray:
    """accumulate_render_radiance (nrc_helpers.cu:77-129); returns an updated copy of rgba [n, 4]. queries (the render
    queries [n, 15]): the USE_REFLECTANCE_FACTORING 1 form."""
    r = np.ascontiguousarray(radiance, dtype=np.float32)
    t = np.ascontiguousarray(throughput, dtype=np.float32)
    o = np.array(rgba, dtype=np.float32, order="C")
    if queries is None:
        lib().orc_accumulate(_v(r), _v(t), _v(o), o.shape[0], int(mode), int(iteration_index))
    else:
        q = np.ascontiguousarray(queries, dtype=np.float32)
        lib().orc_accumulate_factored(_v(r), _v(t), _v(q), _v(o), o.shape[0], int(mode), int(iteration_index))
    return o


def propagate(end_vertices: np.ndarray, end_radiance: np.ndarray, records: np.ndarray, targets: np.ndarray,
              num_records: int, end_queries: np.ndarray | None = None,
              train_queries: np.ndarray | None = None) -> np.ndarray:
    """propagate_train_radiance (nrc_helpers.cu:131-224); end_vertices / records are the structured
    dtypes of nrc_amd.frame (16 B / 28 B). Returns an updated copy of targets [n, 3]. end_queries [tiles, 15] and
    train_queries [records, 15]: the USE_REFLECTANCE_FACTORING 1 form."""
    ev = np.ascontiguousarray(end_vertices)
    er = np.ascontiguousarray(end_radiance, dtype=np.float32)
    rec = np.ascontiguousarray(records)
    assert ev.dtype.itemsize == 16 and rec.dtype.itemsize == 28
    t = np.array(targets, dtype=np.float32, order="C")
    if end_queries is None:
        lib().orc_propagate(_v(ev), _v(er), ev.shape[0], _v(rec), _v(t), int(num_records))
    else:
        eq = np.ascontiguousarray(end_queries, dtype=np.float32)
        tq = np.ascontiguousarray(train_queries, dtype=np.float32)
        lib().orc_propagate_factored(_v(ev), _v(er), _v(eq), ev.shape[0], _v(rec), _v(t), _v(tq), int(num_records))
    return t


def permutation(seed: int, frame: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int32)
    if n:
        lib().orc_permutation(int(seed), int(frame), _v(out), int(n))
    return out


def sort_pairs(keys: np.ndarray):
    """The reference's shuffle (NRCUtil.cu:19-35): (permutation, sorted keys) of cub::DeviceRadixSort::SortPairs over the
    u32 keys and the indices (stable LSD radix sort)."""
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    perm = np.empty(k.size, np.int32)
    sk = np.empty(k.size, np.uint32)
    if k.size:
        lib().orc_sort_pairs(_v(k), _v(sk), _v(perm), int(k.size))
    return perm, sk


def permute(q_src: np.ndarray, t_src: np.ndarray, perm, seed: int, frame: int, num_records: int, n_out: int,
            q_dst: np.ndarray | None = None, t_dst: np.ndarray | None = None):
    """permute_train_data (nrc_helpers.cu:226-249); perm None = the Feistel permutation of (seed, frame)."""
    qs = np.ascontiguousarray(q_src, dtype=np.float32)
    ts = np.ascontiguousarray(t_src, dtype=np.float32)
    qd = np.zeros((n_out, 15), np.float32) if q_dst is None else np.array(q_dst, dtype=np.float32, order="C")
    td = np.zeros((n_out, 3), np.float32) if t_dst is None else np.array(t_dst, dtype=np.float32, order="C")
    pp = None if perm is None else np.ascontiguousarray(perm, dtype=np.int32)
    lib().orc_permute(_v(qs), _v(ts), None if pp is None else _v(pp), int(seed), int(frame), int(num_records),
                      _v(qd), _v(td), int(n_out))
    return qd, td


# ---- InputEncoding::Hash model (oracle/nrc_hash_oracle.c) --------------------------------------------
HASH_MLP_PARAMS = 21504
HASH_GRID_PARAMS = 991232
HASH_NUM_PARAMS = HASH_MLP_PARAMS + HASH_GRID_PARAMS


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def hash_init_params(seed: int = 1337) -> np.ndarray:
    p = np.empty(HASH_NUM_PARAMS, dtype=np.float32)
    lib().orc_hash_init_params(_v(p), seed)
    return p


def hash_encode(params, queries, mode: int = MIXED) -> np.ndarray:
    q, p = _f32(queries), _f32(params)
    out = np.zeros((q.shape[0], 64), np.float32)
    if q.shape[0]:
        lib().orc_hash_encode(_v(p), _v(q), q.shape[0], mode, _v(out))
    return out


def hash_forward(params, queries, mode: int = MIXED, threads: int | None = None, padded: bool = False) -> np.ndarray:
    q, p = _f32(queries), _f32(params)
    out = np.zeros((q.shape[0], 3), np.float32)
    if q.shape[0]:
        lib().orc_hash_forward_layout(int(padded), _v(p), _v(q), q.shape[0], mode, _v(out), threads or default_threads())
    return out


def hash_grad(params, queries, targets, n_total=None, loss_scale=128.0, mode=MIXED, threads=None, padded: bool = False):
    q, t, p = _f32(queries), _f32(targets), _f32(params)
    b = q.shape[0]
    g = np.zeros(HASH_NUM_PARAMS, np.float32)
    loss = lib().orc_hash_grad_layout(int(padded), _v(p), _v(q), _v(t), b, float(3.0 * b if n_total is None else n_total),
                                      float(loss_scale), mode, _v(g), threads or default_threads())
    return g, float(loss)


def hash_corners(query, level: int):
    q = _f32(query).reshape(15)
    e = np.zeros(8, np.uint32)
    w = np.zeros(8, np.float32)
    lib().orc_hash_corners(_v(q), level, _v(e), _v(w))
    return e, w


class HashAdamEmaState:
    """tcnn Adam (matrix part with l2, sparse non-matrix grid part with per-entry steps) + EMA."""

    def __init__(self, params, lr=1e-2, beta1=0.9, beta2=0.999, eps=1e-15, l2_reg=1e-6, ema_decay=0.99,
                 loss_scale=128.0):
        self.params = np.array(params, dtype=np.float32)
        self.m = np.zeros_like(self.params)
        self.v = np.zeros_like(self.params)
        self.ema = np.zeros_like(self.params)
        self.infer = self.params.copy()
        self.grid_steps = np.zeros(HASH_GRID_PARAMS, np.uint32)
        self.step = 0
        self.hp = (lr, beta1, beta2, eps, l2_reg, ema_decay)
        self.loss_scale = loss_scale

    def apply(self, g) -> None:
        self.step += 1
        g = _f32(g)
        lr, b1, b2, eps, l2, dec = self.hp
        lib().orc_hash_adam_ema(_v(self.params), _v(self.m), _v(self.v), _v(self.ema), _v(self.infer),
                                _v(self.grid_steps), self.step, _v(g), self.loss_scale, lr, b1, b2, eps, l2, dec)


# ---- width-128 network (nrc_wide_oracle.c) ----
def wide_forward(params, queries, mode: int = MIXED, threads: int | None = None, encoding: int = FREQUENCY) -> np.ndarray:
    params = _f32(params)
    queries = _f32(queries)
    assert params.size == WIDE_NUM_PARAMS
    n = queries.shape[0]
    out = np.zeros((n, 3), np.float32)
    lib().orc_wide_forward(int(encoding), _v(params), _v(queries), n, mode, _v(out), threads or default_threads())
    return out


def e4m3(x: float) -> float:
    return lib().orc_e4m3(float(x))


def fp8_row_exponent(amax: float) -> int:
    return lib().orc_fp8_row_exponent(float(amax))


def wide_quantize(params):
    """(quantized weight values incl. row scales [77824], row exponents [5][128]) of the FP8 inference path"""
    params = _f32(params)
    q = np.zeros(WIDE_NUM_PARAMS, np.float32)
    e = np.zeros((5, 128), np.int32)
    lib().orc_wide_quantize(_v(params), _v(q), _v(e))
    return q, e


def wide_grad(params, queries, targets, n_total=None, loss_scale=128.0, mode=MIXED, threads=None, encoding=FREQUENCY):
    """(loss-scaled gradient [77824], loss) of one width-128 minibatch"""
    params, queries, targets = _f32(params), _f32(queries), _f32(targets)
    b = queries.shape[0]
    g = np.zeros(WIDE_NUM_PARAMS, np.float32)
    loss = lib().orc_wide_grad(int(encoding), _v(params), _v(queries), _v(targets), b,
                               float(n_total if n_total is not None else 3.0 * b), float(loss_scale), mode, _v(g),
                               threads or default_threads())
    return g, loss
