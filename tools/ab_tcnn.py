"""In-process A/B of the tcnn-numerics inference kernel's accumulator re-entry (knob tcnn_reentry: 0 two 32x32x16
identity MFMAs per block and chunk, 1 four 4x4x4 identity MFMAs), Frequency and Hash, against the default
f32-accumulate kernel; interleaved rounds, HIP events on one stream; outputs of the two forms compared bitwise.

    python tools/ab_tcnn.py [--n 2097152 --rounds 9 --iters 20] [--out f.json]
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
    ap.add_argument("--n", type=int, default=1 << 21)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    n = args.n
    q = torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=7)).to(dev)
    res = {}
    for enc_name in ("Frequency", "Hash"):
        enc = getattr(nrc.InputEncoding, enc_name)
        nets = {}
        for name, prec in (("default", None), ("tcnn", nrc.PRECISION_F16_ACC16)):
            cfg = nrc.default_config(enc) if prec is None else nrc.default_config(enc, infer_precision=prec)
            net = nrc.Network()
            net.init(stream=stream, encoding=enc, config=cfg)
            nets[name] = net
        nets["tcnn"].set_state(nrc.StateSlot.INFER, nets["default"].get_state(nrc.StateSlot.INFER))
        cases = {"default": ("default", -1), "reentry32": ("tcnn", 0), "reentry4x4": ("tcnn", 1)}
        outs = {c: torch.empty((n, 3), device=dev) for c in cases}

        def call(c):
            net, kv = cases[c]
            nrc._lib.set_knob("tcnn_reentry", kv)
            nets[net].infer(q, outs[c], n)

        for c in cases:
            call(c)
        torch.cuda.synchronize()
        same = bool(torch.equal(outs["reentry32"], outs["reentry4x4"]))
        times = {c: [] for c in cases}
        for _ in range(args.rounds):
            for c in cases:
                call(c)  # warm the variant's launch shape
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.iters):
                    nets[cases[c][0]].infer(q, outs[c], n)
                e1.record(stream)
                torch.cuda.synchronize()
                times[c].append(e0.elapsed_time(e1) / args.iters * 1e3)
        nrc._lib.set_knob("tcnn_reentry", -1)
        med = {c: float(np.median(v)) for c, v in times.items()}
        res[enc_name] = {"median_us": med, "min_us": {c: float(np.min(v)) for c, v in times.items()},
                         "slowdown_vs_default": {c: med[c] / med["default"] for c in ("reentry32", "reentry4x4")},
                         "reentry_forms_bitwise_equal": same}
        for net in nets.values():
            net.destroy()
    out = {"n": n, "rounds": args.rounds, "iters": args.iters, "encodings": res}
    print(json.dumps(out, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
