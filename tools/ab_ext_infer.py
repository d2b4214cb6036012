"""In-process A/B of the Hash and FrequencySH inference kernels: per-block LDS work queue (default) against the
round-1 fixed-tiles-per-wave shape (NRC_EXT_INFER_SHAPE=512, read per launch), 2^21 queries, outputs bit-identical.

    python tools/ab_ext_infer.py [--rounds 7] [--iters 10] [--wide]

--wide: the width-128 f16 and FP8 kernels instead (NRC_WIDE_SHAPE=512 selects their round-1 shape), 2^23 queries.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 21)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--wide", action="store_true")
    args = ap.parse_args()
    if args.wide:
        return wide(args)
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    q = torch.from_numpy(nrc.synthetic.cornell_queries(args.n, seed=9)).to(dev)
    res = {}
    for enc in (nrc.InputEncoding.Hash, nrc.InputEncoding.FrequencySH):
        net = nrc.Network()
        net.init(stream=st, encoding=enc)
        outs = {}
        shapes = {"queue": None, "round1": "512"}
        for k, env in shapes.items():
            os.environ.pop("NRC_EXT_INFER_SHAPE", None) if env is None else os.environ.__setitem__("NRC_EXT_INFER_SHAPE", env)
            o = torch.zeros((args.n, 3), device=dev)
            net.infer(q, o, args.n)
            torch.cuda.synchronize()
            outs[k] = o.cpu().numpy()
        times = {k: [] for k in shapes}
        o = torch.zeros((args.n, 3), device=dev)
        for _ in range(args.rounds):
            for k, env in shapes.items():
                os.environ.pop("NRC_EXT_INFER_SHAPE", None) if env is None else os.environ.__setitem__("NRC_EXT_INFER_SHAPE", env)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.iters):
                    net.infer(q, o, args.n)
                e1.record(st)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / args.iters * 1e3)
        os.environ.pop("NRC_EXT_INFER_SHAPE", None)
        net.destroy()
        res[enc.name] = {"bit_identical": bool(np.array_equal(outs["queue"], outs["round1"])),
                         "median_us": {k: float(np.median(v)) for k, v in times.items()}}
    print(json.dumps({"n": args.n, "results": res}, indent=1))


def wide(args) -> None:
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    n = 1 << 23
    q = torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=9)).to(dev)
    e = nrc.InputEncoding.Frequency
    net = nrc.Network()
    net.init(stream=st, encoding=e, config=nrc.default_config(e, width=128))
    res = {}
    shapes = {"queue": None, "round1": "512"}
    for prec, name in ((0, "f16"), (1, "fp8")):
        outs = {}
        for k, env in shapes.items():
            os.environ.pop("NRC_WIDE_SHAPE", None) if env is None else os.environ.__setitem__("NRC_WIDE_SHAPE", env)
            o = torch.zeros((n, 3), device=dev)
            net.infer_precision(prec, q, o, n)
            torch.cuda.synchronize()
            outs[k] = o.cpu().numpy()
        times = {k: [] for k in shapes}
        o = torch.zeros((n, 3), device=dev)
        for _ in range(args.rounds):
            for k, env in shapes.items():
                os.environ.pop("NRC_WIDE_SHAPE", None) if env is None else os.environ.__setitem__("NRC_WIDE_SHAPE", env)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.iters):
                    net.infer_precision(prec, q, o, n)
                e1.record(st)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / args.iters * 1e3)
        res[name] = {"bit_identical": bool(np.array_equal(outs["queue"], outs["round1"])),
                     "median_us": {k: float(np.median(v)) for k, v in times.items()}}
    os.environ.pop("NRC_WIDE_SHAPE", None)
    net.destroy()
    print(json.dumps({"n": n, "results": res}, indent=1))


if __name__ == "__main__":
    main()
