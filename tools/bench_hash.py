"""Timing of the InputEncoding::Hash model on one MI355X: inference over 2^21 synthetic
Cornell queries and the 16,384-sample training step, HIP events on the network's stream.

    python tools/bench_hash.py [--iters 50] [--knob hash_infer=1]
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--queries", type=int, default=1 << 21)
    ap.add_argument("--knob", action="append", default=[], help="name=value A/B knob of the library (repeatable)")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    for kv in args.knob:
        k, v = kv.split("=")
        nrc._lib.set_knob(k, int(v))
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    net = nrc.Network()
    net.init(stream=stream, encoding=nrc.InputEncoding.Hash)
    n = args.queries
    q = torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=1)).to(dev)
    out = torch.empty((n, 3), device=dev)
    tq, tt = nrc.synthetic.cornell_batch(4 * nrc.BATCH_SIZE, seed=2)
    tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
    for f in range(8):  # a few steps so that the grid is no longer at its +-1e-4 init
        net.train(tq[(f % 4) * nrc.BATCH_SIZE:], tt[(f % 4) * nrc.BATCH_SIZE:])

    def timed(fn, iters):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(iters):
            fn(i)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3

    infer_us = timed(lambda i=0: net.infer(q, out, n), args.iters)
    train_us = timed(lambda i=0: net.train(tq[(i % 4) * nrc.BATCH_SIZE:], tt[(i % 4) * nrc.BATCH_SIZE:]), 40)
    net.destroy()
    flop_q = 2 * (62 * 64 + 4 * 64 * 64 + 64 * 3)
    print(json.dumps({"encoding": "Hash", "knobs": args.knob, "queries": n, "infer_us": infer_us, "Gq_per_s": n / infer_us / 1e3,
                      "mlp_tflops_alg": flop_q * n / (infer_us * 1e-6) / 1e12,
                      "gathers_per_query": 16 * 8, "train_step_us": train_us}, indent=1))


if __name__ == "__main__":
    main()
