"""Seeded synthetic Cornell-box radiance queries and training targets.

Stands in for the renderer's query writers: it produces the exact byte layout the reference's
closest-hit programs write (``RadianceQuery``, 15 packed f32, /root/reference/nrc/shaders/
neural_radiance_caching.h:100-118) with the value distributions of ``nrc::addQuery``
(/root/reference/nrc/shaders/hit.cu:589-617):

* position: a uniform point on one of the six Cornell walls (±10 box,
  /root/reference/data/scene_mdl_cornell.txt:45-56) scaled by 0.005 (hit.cu:596-597);
* direction / normal: (theta, phi) = (2 asin(|d - z|/2), atan2(y, x))
  (cartesianToSphericalUnitVector, shader_common.h:320-333); the wall normal is flipped to face
  the outgoing direction;
* roughness: (1, 1) for diffuse events (hit.cu:481-483, 90 %), U[0,1]^2 otherwise;
* diffuse albedo: white / red / green Cornell materials + U[-0.05, 0.05] jitter;
* specular albedo: 0 (90 %) or U[0,1]^3;
* targets: lognormal(mu=-1, sigma=1.5) radiance per channel.
"""
from __future__ import annotations

import numpy as np

SEED = 20240611
_WHITE = (0.8, 0.8, 0.8)
_RED = (0.8, 0.1, 0.1)
_GREEN = (0.1, 0.8, 0.1)


def _spherical(d: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """cartesianToSphericalUnitVector (shader_common.h:320-333), evaluated in f32."""
    d = d.astype(np.float32)
    zm1 = d[:, 2] - np.float32(1.0)
    dist = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + zm1 * zm1)
    theta = np.float32(2.0) * np.arcsin(np.minimum(np.float32(0.5) * dist, np.float32(1.0)))
    phi = np.arctan2(d[:, 1], d[:, 0])
    return theta.astype(np.float32), phi.astype(np.float32)


def cornell_queries(n: int, seed: int = SEED) -> np.ndarray:
    """n RadianceQuery records as an (n, 15) float32 array (row = 60 contiguous bytes)."""
    rng = np.random.default_rng(seed)
    q = np.empty((n, 15), dtype=np.float32)
    if n == 0:
        return q
    wall = rng.integers(0, 6, size=n)
    axis = wall // 2
    sign = np.where(wall % 2 == 0, -1.0, 1.0)
    pos = rng.uniform(-10.0, 10.0, size=(n, 3))
    pos[np.arange(n), axis] = 10.0 * sign
    q[:, 0:3] = (pos * 0.005).astype(np.float32)

    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    q[:, 3], q[:, 4] = _spherical(d)

    nrm = np.zeros((n, 3))
    nrm[np.arange(n), axis] = -sign  # inward-facing wall normal
    flip = np.sum(nrm * d, axis=1) < 0.0
    nrm[flip] *= -1.0
    q[:, 5], q[:, 6] = _spherical(nrm)

    glossy = rng.random(n) < 0.1
    rough = np.ones((n, 2))
    rough[glossy] = rng.random((int(glossy.sum()), 2))
    q[:, 7:9] = rough.astype(np.float32)

    mats = np.array([_WHITE, _RED, _GREEN])
    q[:, 9:12] = (mats[rng.integers(0, 3, size=n)] + rng.uniform(-0.05, 0.05, size=(n, 3))).astype(np.float32)

    spec_on = rng.random(n) < 0.1
    spec = np.zeros((n, 3))
    spec[spec_on] = rng.random((int(spec_on.sum()), 3))
    q[:, 12:15] = spec.astype(np.float32)
    return q


def cornell_targets(n: int, seed: int = SEED) -> np.ndarray:
    """n float3 training targets, (n, 3) float32, lognormal(mu=-1, sigma=1.5)."""
    rng = np.random.default_rng(seed + 7919)
    return rng.lognormal(mean=-1.0, sigma=1.5, size=(n, 3)).astype(np.float32)


def cornell_batch(n: int, seed: int = SEED) -> tuple[np.ndarray, np.ndarray]:
    return cornell_queries(n, seed), cornell_targets(n, seed)
