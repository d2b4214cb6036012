"""In-process A/B timing of width-128 inference kernel variants (interleaved rounds, one process, one device).
Variant codes are nrc_debug_infer_precision's: precision | (kernel variant << 4). Outputs of every code are
compared with the production kernel of the same precision (expected bit-identical).

    python tools/ab_wide.py [--n 8388608] [--rounds 7] [--iters 10] [--codes 0,16,1,17]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402

FLOP_Q = 2 * (66 * 128 + 4 * 128 * 128 + 128 * 3)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 23)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--codes", default="0,16,1,17")
    args = ap.parse_args()
    import numpy as np
    import torch

    nrc = nrc_loader.load()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = int(stream.cuda_stream)
    codes = [int(c) for c in args.codes.split(",")]
    net = nrc.Network()
    net.init(stream=stream, encoding=nrc.InputEncoding.Frequency,
             config=nrc.default_config(nrc.InputEncoding.Frequency, width=128))
    q = torch.from_numpy(nrc.synthetic.cornell_queries(args.n, seed=1)).to(dev)
    outs = {c: torch.empty((args.n, 3), device=dev) for c in codes}
    for c in codes:
        nrc._lib.check(L.nrc_debug_infer_precision(net._h, c, q.data_ptr(), outs[c].data_ptr(), args.n, sp))
    torch.cuda.synchronize()
    same = {}
    for c in codes:
        base = outs[c & 15] if (c & 15) in outs else None
        same[c] = None if base is None else bool(torch.equal(outs[c], base))
    times = {c: [] for c in codes}
    for _ in range(args.rounds):
        for c in codes:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                L.nrc_debug_infer_precision(net._h, c, q.data_ptr(), outs[c].data_ptr(), args.n, sp)
            e1.record(stream)
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / args.iters * 1e3)
    res = {}
    for c in codes:
        t = np.array(times[c])
        med = float(np.median(t))
        res[c] = {"median_us": round(med, 2), "min_us": round(float(t.min()), 2),
                  "tflops_alg": round(FLOP_Q * args.n / (med * 1e-6) / 1e12, 1), "identical_to_production": same[c]}
    net.destroy()
    print(json.dumps({"n": args.n, "codes": res}, indent=1))


if __name__ == "__main__":
    main()
