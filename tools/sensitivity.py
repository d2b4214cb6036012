"""Sensitivity of the network output to the spec choices the oracle had to make without tiny-cuda-nn's source
(tags [M]/[L]): how far the outputs move if tcnn's actual choice were another plausible one.

Weights are trained by the oracle (oracle/nrc_oracle.c, MIXED numerics, Adam + EMA as configured by
NRCNetworkConfigs.h:11-83) on the seeded synthetic Cornell stream for several step counts; every alternative is then
evaluated on 16,384 held-out queries with a float64 MLP on f16-rounded operands (numpy), against the spec choice run
through the same code. Output: one JSON document (profiles/r02_sensitivity/sensitivity.json), summarised in
DESIGN.md §4. CPU only; test infrastructure (imports the oracle).

    python tools/sensitivity.py [--steps 4,16,64,256] [--out profiles/r02_sensitivity/sensitivity.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402

LAYERS = [(64, 80), (64, 64), (64, 64), (64, 64), (64, 64), (16, 64)]


def f16(a):
    return np.asarray(a, np.float32).astype(np.float16).astype(np.float64)


def unpack(params):
    out, off = [], 0
    for o, i in LAYERS:
        out.append(f16(params[off:off + o * i]).reshape(o, i))
        off += o * i
    return out


def tri_variants(u):
    fr = u - np.floor(u)
    return {
        "spec |2 frac(u) - 1| (period 1, [0,1], floor-based frac)": np.abs(2.0 * fr - 1.0),
        "fmod-based frac (negative inputs keep their sign)": np.abs(2.0 * np.fmod(u, 1.0) - 1.0),
        "phase-shifted 1 - |2 frac(u) - 1| (0 at integers)": 1.0 - np.abs(2.0 * fr - 1.0),
        "range [-1, 1]: 2 |2 frac(u) - 1| - 1": 2.0 * np.abs(2.0 * fr - 1.0) - 1.0,
        "sine-like triangle, peak at u = 1/4, range [-1, 1]": 1.0 - 4.0 * np.abs(u + 0.25 - np.floor(u + 0.75)),
    }


def qcdf(v):
    u = v * 4.0
    return np.clip(u * (15.0 - 10.0 * u * u + 3.0 * u ** 4) / 16.0 + 0.5, 0.0, 1.0)


def one_blob(x, wrap=True):
    lb = np.arange(4) / 4.0
    d = lb[None, None, :] - x[:, :, None]
    if wrap:  # spec (oracle one_blob): period-1 wrap of the kernel, last bin closed by left_cdf(0) + 1
        left = qcdf(d) + qcdf(d - 1.0) + qcdf(d + 1.0)
        right = np.concatenate([left[:, :, 1:], left[:, :, :1] + 1.0], axis=2)
    else:  # no wrap: bin b = K(b/4 + 1/4 - x) - K(b/4 - x)
        left = qcdf(d)
        right = qcdf(d + 0.25)
    return (right - left).reshape(x.shape[0], -1)


SPEC_TRI = "spec |2 frac(u) - 1| (period 1, [0,1], floor-based frac)"


def encode(q, tri=SPEC_TRI, pad=1.0, wrap=True):
    n = q.shape[0]
    e = np.empty((n, 80))
    u = q[:, 0:3, None] * (2.0 ** np.arange(12))[None, None, :]
    e[:, 0:36] = tri_variants(u)[tri].reshape(n, 36)
    e[:, 36:60] = one_blob(q[:, 3:9], wrap)
    e[:, 60:66] = q[:, 9:15]
    e[:, 66:80] = pad
    return e


def forward(params, e, f16_accumulate=False):
    W = unpack(params)
    a = f16(e)
    for l in range(6):
        if f16_accumulate:  # tcnn WMMA with f16 accumulators [M]: round after every 16-wide K chunk
            z = np.zeros((a.shape[0], W[l].shape[0]))
            for c in range(0, a.shape[1], 16):
                z = f16(z + a[:, c:c + 16] @ W[l][:, c:c + 16].T)
        else:
            z = a @ W[l].T
        a = f16(np.maximum(z, 0.0))
    return a[:, :3]


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="4,16,64,256")
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r02_sensitivity" / "sensitivity.json"))
    args = ap.parse_args()
    nrc = nrc_loader.load()
    orc = nrc_loader.load_oracle()
    steps = sorted(int(s) for s in args.steps.split(","))
    q_eval = nrc.synthetic.cornell_queries(16384, seed=4242).astype(np.float64)
    st = orc.AdamEmaState(orc.init_params(1337))
    base_enc = encode(q_eval)
    tri_names = list(tri_variants(np.zeros(1)).keys())
    results = []
    t0 = time.time()
    done = 0
    for target in steps:
        while done < target:
            tq, tt = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=10_000 + done)
            g, _ = orc.grad(st.params, tq, tt, mode=orc.MIXED)
            st.apply(g)
            done += 1
        w_inf = st.infer  # debiased EMA: the inference weights of the spec
        y = forward(w_inf, base_enc)
        row = {"train_steps": done, "output_rms": float(np.sqrt(np.mean(y ** 2))), "rel_l2": {}}
        r = row["rel_l2"]
        for name in tri_names[1:]:
            r[f"TriangleWave [L]: {name}"] = rel(forward(w_inf, encode(q_eval, tri=name)), y)
        r["Composite padding [M]: 0.0 instead of 1.0"] = rel(forward(w_inf, encode(q_eval, pad=0.0)), y)
        r["OneBlob [M]: no period-1 wrap of the kernel"] = rel(forward(w_inf, encode(q_eval, wrap=False)), y)
        r["EMA [L]: raw EMA (no 1 - 0.99^t debias) as the inference weights"] = rel(forward(st.ema, base_enc), y)
        r["EMA [L]: training weights (no EMA) for inference"] = rel(forward(st.params, base_enc), y)
        r["FullyFusedMLP [M]: f16 accumulation per 16-wide K chunk (ORC_TCNN)"] = rel(forward(w_inf, base_enc, True), y)
        results.append(row)
        print(json.dumps(row), flush=True)
    doc = {"what": __doc__.strip().splitlines()[0], "eval_queries": int(q_eval.shape[0]),
           "train": "oracle MIXED numerics, Adam(1e-3) + EMA(0.99), 16,384-sample synthetic Cornell minibatches",
           "rows": results, "seconds": round(time.time() - t0, 1)}
    out = Path(args.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(doc, indent=1) + "\n")


if __name__ == "__main__":
    main()
