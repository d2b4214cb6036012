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


# ---- one frame of the renderer's NRC buffers (stands in for the OptiX trace) --------------------------------
class SyntheticFrame:
    """Host arrays of one frame, in the reference's layouts (neural_radiance_caching.h:57-187).

    Emulates what the trace leaves behind (hit.cu:975-1027, miss.cu:140-160, raygeneration.cu:122-136):
    one training path per full tile; each non-Dirac vertex of it atomically allocates a TrainingRecord
    (bounce-major order, shuffled within a bounce like concurrent atomics) linked by ``prop_to`` to the
    previous one; once the 65,536-record buffer is full the path ends there by self-training; other paths
    end self-training (mask 1) or, with probability TRAIN_UNBIASED_RATIO = 1/16, unbiased (mask 0).
    ``num_training_records`` is the raw atomic counter, so it can exceed the capacity.
    """

    def __init__(self, **kw):
        self.__dict__.update(kw)


def cornell_frame(width: int = 64, height: int = 48, tile: tuple[int, int] = (4, 4), seed: int = SEED,
                  frame_index: int = 0, capacity: int = 65536, mean_records: float = 2.0,
                  max_records_per_path: int = 8) -> SyntheticFrame:
    from .frame import END_VERTEX_DTYPE, TRAINING_RECORD_DTYPE

    rng = np.random.default_rng([seed, frame_index, 0x4E5243])
    tx, ty = tile
    tiles_x, tiles_y = width // tx, height // ty  # boundary tiles are discarded (raygeneration.cu:122-129)
    screen, tiles = width * height, tiles_x * tiles_y

    n_vert = np.minimum(rng.geometric(1.0 / (mean_records + 1.0), size=tiles) - 1, max_records_per_path)
    last = np.full(tiles, -1, dtype=np.int64)
    full = np.zeros(tiles, dtype=bool)
    recs = np.zeros(capacity, dtype=TRAINING_RECORD_DTYPE)
    counter = 0
    for b in range(int(n_vert.max(initial=0))):
        t = np.flatnonzero((n_vert > b) & ~full)
        t = rng.permutation(t)
        idx = counter + np.arange(len(t))
        counter += len(t)
        ok = idx < capacity
        full[t[~ok]] = True
        t, idx = t[ok], idx[ok]
        recs["prop_to"][idx] = last[t]
        recs["local_throughput"][idx] = rng.uniform(0.05, 0.9, size=(len(t), 3)).astype(np.float32)
        recs["tile_index"][idx] = t
        recs["pixel_index"][idx] = (t // tiles_x) * ty * width + (t % tiles_x) * tx
        recs["prop_length"][idx] = b + 1
        last[t] = idx
    allocated = min(counter, capacity)

    ends = np.zeros(tiles, dtype=END_VERTEX_DTYPE)
    ends["start_train_record"] = last
    unbiased = (rng.random(tiles) < 1.0 / 16.0) & ~full
    ends["radiance_mask"] = np.where(unbiased, 0.0, 1.0).astype(np.float32)
    ends["tile_index"] = np.arange(tiles)

    train_q = np.zeros((capacity, 15), dtype=np.float32)
    train_q[:allocated] = cornell_queries(allocated, seed=int(rng.integers(1 << 31)))
    train_t = np.zeros((capacity, 3), dtype=np.float32)
    lit = np.flatnonzero(rng.random(allocated) < 0.1)  # emission / env hits added during the trace
    train_t[lit] = rng.lognormal(-1.0, 1.5, size=(len(lit), 3)).astype(np.float32)

    thr = rng.uniform(0.0, 1.0, size=(screen, 3)).astype(np.float32)
    thr[rng.random(screen) < 0.05] = 0.0  # paths that missed early (miss.cu:150-155)
    return SyntheticFrame(
        width=width, height=height, tile=tile, screen_size=screen, num_tiles=tiles,
        num_training_records=counter, frame_index=frame_index,
        queries_inference=cornell_queries(screen + tiles, seed=int(rng.integers(1 << 31))),
        last_render_throughput=thr,
        queries_cache_vis=cornell_queries(screen, seed=int(rng.integers(1 << 31))),
        end_vertices=ends, train_records=recs, train_queries=train_q, train_targets=train_t)
