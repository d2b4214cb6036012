"""Generates tests/golden/nrc_golden.npz from the C oracle (oracle/nrc_oracle.c).

The reference holds no fixtures for this path: these vectors pin the oracle
and the GPU build against regressions; they are not tcnn outputs (parity unpinned).
Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def edge_queries() -> np.ndarray:
    """Hand-picked queries that exercise the encodings' saturation / wrap branches."""
    rows = []
    for x in [0.0, 1e-9, -1e-9, 0.05, -0.05, 0.2, 0.49999997, 0.5, 0.99999994]:
        for ang in [0.0, 0.125, 0.25, 0.6, 1.0, 1.5, 1.75, 2.0, 3.14159265, -0.3, -0.75, -1.0, -3.14159265]:
            rows.append([x, -x, 0.5 * x, ang, -ang, ang * 0.5, 3.0 - ang, 1.0, min(abs(ang), 1.0),
                         0.8, 0.1, 0.1, 0.0, 0.25, 1.0])
    return np.asarray(rows, dtype=np.float32)


def main() -> None:
    nrc = nrc_loader.load()
    orc = nrc_loader.load_oracle()
    q = nrc.synthetic.cornell_queries(4096, seed=1)
    qe = edge_queries()
    t = nrc.synthetic.cornell_targets(1024, seed=1)
    params = orc.init_params(1337)
    # a "trained-looking" parameter set: scaled init so that outputs are not tiny
    rng = np.random.default_rng(3)
    params_b = (params * np.float32(1.6) + rng.normal(0, 0.01, params.shape)).astype(np.float32)
    out = {"queries": q, "queries_edge": qe, "targets": t, "params": params, "params_b": params_b,
           "enc": orc.encode(q[:256]), "enc_edge": orc.encode(qe)}
    for name, mode in [("fp32", orc.FP32), ("mixed", orc.MIXED), ("tcnn", orc.TCNN)]:
        out[f"y_{name}"] = orc.forward(params_b, q, mode)
        out[f"y_edge_{name}"] = orc.forward(params_b, qe, mode)
        g, loss = orc.grad(params_b, q[:1024], t, mode=mode)
        out[f"grad_{name}"] = g
        out[f"loss_{name}"] = np.float64(loss)
    st = orc.AdamEmaState(params_b)
    st.apply(out["grad_mixed"])
    out["adam1_params"], out["adam1_m"], out["adam1_v"] = st.params.copy(), st.m.copy(), st.v.copy()
    out["adam1_ema"], out["adam1_infer"] = st.ema.copy(), st.infer.copy()
    path = ROOT / "tests" / "golden" / "nrc_golden.npz"
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({path.stat().st_size} bytes)")


if __name__ == "__main__":
    main()
