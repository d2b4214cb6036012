"""Timing of the width-128 network (BASELINE.json configs[4]) on one MI355X: f16 and FP8 inference
over synthetic Cornell queries, HIP events on the launch stream.

    python tools/bench_wide.py [--queries 8388608] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402

FLOP_Q = 2 * (66 * 128 + 4 * 128 * 128 + 128 * 3)  # 148,736 algorithmic FLOP per query


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--queries", type=int, nargs="+", default=[1 << 21, 1 << 23])
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    net = nrc.Network()
    net.init(stream=stream, encoding=nrc.InputEncoding.Frequency,
             config=nrc.default_config(nrc.InputEncoding.Frequency, width=128))
    rows = []
    for n in args.queries:
        q = torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=1)).to(dev)
        out = torch.empty((n, 3), device=dev)
        for prec, name in ((0, "f16"), (1, "fp8")):
            fn = lambda: net.infer_precision(prec, q, out, n, stream=stream)  # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / args.iters * 1e3
            tf = FLOP_Q * n / (us * 1e-6) / 1e12
            peak = 2500.0 if prec == 0 else 5000.0
            rows.append({"precision": name, "queries": n, "infer_us": round(us, 2), "Gq_per_s": round(n / us / 1e3, 3),
                         "tflops_alg": round(tf, 1), "frac_of_dense_peak": round(tf / peak, 4), "peak_tflops": peak})
            print(json.dumps(rows[-1]), flush=True)
    # training step: 16,384 samples (fwd + loss + bwd + dW + Adam/EMA + image repacks)
    tq, tt = nrc.synthetic.cornell_batch(4 * nrc.BATCH_SIZE, seed=2)
    tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
    for i in range(4):
        net.train(tq[i * nrc.BATCH_SIZE:], tt[i * nrc.BATCH_SIZE:])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(40):
        net.train(tq[(i % 4) * nrc.BATCH_SIZE:], tt[(i % 4) * nrc.BATCH_SIZE:])
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 40 * 1e3
    train_flop = nrc.BATCH_SIZE * (3 * FLOP_Q - 2 * 66 * 128)  # fwd + dW + dX of layers 1..5
    print(json.dumps({"train_step_us": round(us, 2), "train_tflops_alg": round(train_flop / (us * 1e-6) / 1e12, 1)}),
          flush=True)
    net.destroy()


if __name__ == "__main__":
    main()
