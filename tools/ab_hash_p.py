"""In-process interleaved A/B of a Hash-inference knob (default: the feature pass's query-range count P, knob
hash_feat_p; debug library: hash_feat_abl=8, the round-3 arithmetic): inference over 2^21 synthetic Cornell queries,
HIP events on the network's stream; outputs must be bitwise equal across the values.

    python tools/ab_hash_p.py [--knob hash_feat_p] [--ps 16,32,64] [--rounds 5] [--iters 20]
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
    ap.add_argument("--ps", default="16,32,64", help="knob values")
    ap.add_argument("--knob", default="hash_feat_p")
    ap.add_argument("--set", action="append", default=[], help="name=value knob held for the whole run")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--queries", type=int, default=1 << 21)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    for kv in args.set:
        k, v = kv.split("=")
        nrc._lib.set_knob(k, int(v))
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    net = nrc.Network()
    net.init(stream=stream, encoding=nrc.InputEncoding.Hash)
    n = args.queries
    q = torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=1)).to(dev)
    tq, tt = nrc.synthetic.cornell_batch(4 * nrc.BATCH_SIZE, seed=2)
    tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
    for b in range(4):
        net.train(tq[b * nrc.BATCH_SIZE:], tt[b * nrc.BATCH_SIZE:])
    ps = [int(p) for p in args.ps.split(",")]
    outs = {}
    for p in ps:
        nrc._lib.set_knob(args.knob, p)
        outs[p] = torch.empty((n, 3), device=dev)
        net.infer(q, outs[p], n)
    torch.cuda.synchronize()
    equal = {p: bool(torch.equal(outs[p], outs[ps[0]])) for p in ps}
    times = {p: [] for p in ps}
    for _ in range(args.rounds):
        for p in ps:
            nrc._lib.set_knob(args.knob, p)
            for _ in range(3):
                net.infer(q, outs[p], n)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                net.infer(q, outs[p], n)
            e1.record(stream)
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) / args.iters * 1e3)
    nrc._lib.set_knob(args.knob, -1)
    res = {p: {"median_us": float(np.median(times[p])), "min_us": float(np.min(times[p])),
               "bitwise_equal_to_first": equal[p]} for p in ps}
    print(json.dumps({"queries": n, "knob": args.knob, "held": args.set, "by_value": res}))
    net.destroy()


if __name__ == "__main__":
    main()
