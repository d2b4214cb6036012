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

FP32, MIXED, TCNN = 0, 1, 2
NUM_PARAMS = 22528

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
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def default_threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def encode(queries: np.ndarray) -> np.ndarray:
    q = np.ascontiguousarray(queries, dtype=np.float32)
    n = q.shape[0]
    out = np.empty((n, 80), dtype=np.float32)
    if n:
        lib().orc_encode(_p(q), n, _p(out))
    return out


def forward(params: np.ndarray, queries: np.ndarray, mode: int = MIXED, threads: int | None = None) -> np.ndarray:
    q = np.ascontiguousarray(queries, dtype=np.float32)
    p = np.ascontiguousarray(params, dtype=np.float32)
    n = q.shape[0]
    out = np.zeros((n, 3), dtype=np.float32)
    if n:
        lib().orc_forward(_p(p), _p(q), n, mode, _p(out), threads or default_threads())
    return out


def grad(params, queries, targets, n_total=None, loss_scale=128.0, mode=MIXED, threads=None):
    q = np.ascontiguousarray(queries, dtype=np.float32)
    t = np.ascontiguousarray(targets, dtype=np.float32)
    p = np.ascontiguousarray(params, dtype=np.float32)
    b = q.shape[0]
    if n_total is None:
        n_total = 3.0 * b
    g = np.zeros(NUM_PARAMS, dtype=np.float32)
    loss = lib().orc_grad(_p(p), _p(q), _p(t), b, float(n_total), float(loss_scale), mode, _p(g),
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
