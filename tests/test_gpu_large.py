"""Launches whose RadianceQuery buffer is larger than 4 GiB (72,000,123 records: 4.32 GB compact, 4.61 GB padded).

The boundary takes n as uint32_t (`nrc_c.h`, the reference's `infer(float*, float*, uint32_t)`, NRCNetwork.h:49-51), so a
caller may hand over buffers past 2^32 bytes; every kernel must address them through 64-bit bases (the raw-buffer
descriptors are built per tile, their 32-bit record counts cover one tile). Property checked at that size, independent of
the oracle's speed: each query is an independent unit, so a launch over a buffer made of copies of one
base block must return the base block's outputs, bit for bit, in every copy and in the ragged tail -- for the product
inference kernel (compact and padded records), the width-128 f16 / FP8 kernels and the Hash feature pass + MLP pass --
and write nothing past n. The base block's own outputs are checked against the oracle by the other GPU tests.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

# ≈10 GB of device buffers, a few seconds (profiles/r04_end/pytest_gpu_large.log); NRC_TEST_LARGE=0 skips them
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("NRC_TEST_LARGE", "1") == "0", reason="NRC_TEST_LARGE=0")]

BASE = 1 << 20
N = 72_000_123  # 68 copies of BASE + a ragged tail of 697,387 rows; 60 N > 2^32


@pytest.fixture(scope="module")
def torch():
    import torch as t
    return t


def _tiled(torch, base, n):
    copies = -(-n // base.shape[0])
    return base.repeat(copies, 1)[:n].contiguous()


def _check(torch, out, ref, n):
    """out [n + 8, 3] against ref [BASE, 3]: every full copy, the tail, the sentinel rows."""
    full = n // BASE
    body = out[: full * BASE].view(full, BASE, 3)
    same = (body == ref.unsqueeze(0)).all(dim=2).all(dim=1)
    assert bool(same.all()), f"copies differing from the base block: {torch.nonzero(~same).flatten()[:8].tolist()}"
    tail = n - full * BASE
    assert torch.equal(out[full * BASE: n], ref[:tail]), "ragged tail differs from the base block"
    assert bool((out[n:] == 4321.0).all()), "written past n"


def _run(torch, dev, fn, qb, n):
    ref = torch.empty((BASE, 3), dtype=torch.float32, device=dev)
    fn(qb, ref, BASE)
    q = _tiled(torch, qb, n)
    assert q.numel() * 4 > 1 << 32
    out = torch.full((n + 8, 3), 4321.0, dtype=torch.float32, device=dev)
    fn(q, out, n)
    torch.cuda.synchronize()
    del q
    return out, ref


@pytest.mark.parametrize("layout", ["compact", "padded"])
def test_infer_past_4gib(nrc, orc, torch, dev, layout):
    cfg = nrc.default_config(nrc.InputEncoding.Frequency)
    cfg.query_layout = nrc.QUERY_PADDED if layout == "padded" else nrc.QUERY_COMPACT
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), config=cfg)
    try:
        net.set_state(nrc.StateSlot.INFER, orc.init_params(1337) * np.float32(1.6))
        q15 = nrc.synthetic.cornell_queries(BASE, seed=41)
        if layout == "padded":
            q15 = np.insert(q15, 3, np.random.default_rng(2).uniform(-1, 1, BASE).astype(np.float32), axis=1)
        qb = torch.from_numpy(np.ascontiguousarray(q15, np.float32)).to(dev)
        out, ref = _run(torch, dev, net.infer, qb, N)
        _check(torch, out, ref, N)
    finally:
        net.destroy()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("prec", ["f16", "fp8"])
def test_wide_infer_past_4gib(nrc, torch, dev, prec):
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), config=nrc.default_config(nrc.InputEncoding.Frequency, width=128))
    try:
        p = nrc.PRECISION_FP8 if prec == "fp8" else nrc.PRECISION_F16
        qb = torch.from_numpy(nrc.synthetic.cornell_queries(BASE, seed=42)).to(dev)
        out, ref = _run(torch, dev, lambda q, o, n: net.infer_precision(p, q, o, n), qb, N)
        _check(torch, out, ref, N)
    finally:
        net.destroy()
        torch.cuda.empty_cache()


def test_hash_infer_past_4gib(nrc, orc, torch, dev):
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream(), encoding=nrc.InputEncoding.Hash)
    try:
        params = orc.hash_init_params(1337)
        params[orc.HASH_MLP_PARAMS:] = np.random.default_rng(5).uniform(-1.0, 1.0, orc.HASH_GRID_PARAMS).astype(np.float32)
        net.set_state(nrc.StateSlot.INFER, params)
        qb = torch.from_numpy(nrc.synthetic.cornell_queries(BASE, seed=43)).to(dev)
        out, ref = _run(torch, dev, net.infer, qb, N)
        _check(torch, out, ref, N)
    finally:
        net.destroy()
        torch.cuda.empty_cache()
