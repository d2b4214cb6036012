"""Independent float64 numpy restatement of the NRC forward / RelativeL2Luminance / backward.

TEST INFRASTRUCTURE ONLY. Written separately from oracle/nrc_oracle.c (vectorised over samples,
float64 throughout) so that the two restatements check each other (tests/test_oracle.py).
Semantics follow SURVEY.md Appendix A (tcnn as configured by NRCNetworkConfigs.h:11-83).
"""
from __future__ import annotations

import numpy as np

LAYER_SHAPES = [(64, 80), (64, 64), (64, 64), (64, 64), (64, 64), (16, 64)]


def unpack(params: np.ndarray) -> list[np.ndarray]:
    out, off = [], 0
    for o, i in LAYER_SHAPES:
        out.append(np.asarray(params[off:off + o * i], dtype=np.float64).reshape(o, i))
        off += o * i
    return out


def encode(q: np.ndarray) -> np.ndarray:
    q = np.asarray(q, dtype=np.float64)
    n = q.shape[0]
    e = np.empty((n, 80))
    k = 2.0 ** np.arange(12)
    u = q[:, 0:3, None] * k[None, None, :]  # (n, 3, 12), dimension-major
    e[:, 0:36] = np.abs(2.0 * (u - np.floor(u)) - 1.0).reshape(n, 36)

    x = q[:, 3:9]  # (n, 6)
    lb = np.arange(4) / 4.0

    def qcdf(v):
        u = v * 4.0
        return np.clip(u * (15.0 - 10.0 * u * u + 3.0 * u ** 4) / 16.0 + 0.5, 0.0, 1.0)

    d = lb[None, None, :] - x[:, :, None]
    left = qcdf(d) + qcdf(d - 1.0) + qcdf(d + 1.0)  # (n, 6, 4)
    right = np.concatenate([left[:, :, 1:], left[:, :, :1] + 1.0], axis=2)
    e[:, 36:60] = (right - left).reshape(n, 24)
    e[:, 60:66] = q[:, 9:15]
    e[:, 66:80] = 1.0
    return e


def forward(params: np.ndarray, q: np.ndarray) -> tuple[np.ndarray, list[np.ndarray]]:
    W = unpack(params)
    a = encode(q)
    acts = [a]
    for l in range(5):
        a = np.maximum(a @ W[l].T, 0.0)
        acts.append(a)
    y = np.maximum(a @ W[5].T, 0.0)
    return y, acts


def loss_and_grad(params, q, t, n_total=None, loss_scale=128.0):
    """Returns (loss, loss_scale * dL/dW) in float64 (denominator treated as constant)."""
    W = unpack(params)
    t = np.asarray(t, dtype=np.float64)
    b = q.shape[0]
    if n_total is None:
        n_total = 3.0 * b
    y, acts = forward(params, q)
    lum = 0.299 * y[:, 0] + 0.587 * y[:, 1] + 0.114 * y[:, 2]
    den = lum * lum + 0.01
    diff = y[:, :3] - t
    loss = float(np.sum(diff * diff / den[:, None]) / n_total)
    d = np.zeros_like(y)
    d[:, :3] = loss_scale * 2.0 * diff / den[:, None] / n_total
    d *= (y > 0.0)
    grads = [None] * 6
    for l in range(5, -1, -1):
        grads[l] = d.T @ acts[l]
        if l == 0:
            break
        d = (d @ W[l]) * (acts[l] > 0.0)
    return loss, np.concatenate([g.reshape(-1) for g in grads])
