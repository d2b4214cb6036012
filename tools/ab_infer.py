"""In-process A/B timing of the inference kernel variants (interleaved rounds, one process, one device;
cdna_hip_programming.md §5.4 rule 24). Also checks every variant against the oracle on a sample.

    python tools/ab_infer.py [--n 2097152] [--rounds 7] [--iters 20] [--variants 0,1,2]
"""
from __future__ import annotations

import argparse
import ctypes
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="0,1,2")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    orc = nrc_loader.load_oracle()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = int(stream.cuda_stream)
    variants = [int(v) for v in args.variants.split(",")]

    q_np = nrc.synthetic.cornell_queries(args.n, seed=2)
    q = torch.from_numpy(q_np).to(dev)
    net = nrc.Network()
    net.init(stream=stream)
    params = orc.init_params(1337) * np.float32(1.6)
    net.set_state(nrc.StateSlot.INFER, params)
    outs = {v: torch.empty((args.n, 3), device=dev) for v in variants}
    idx = np.arange(0, args.n, 4099)
    y_ref = orc.forward(params, q_np[idx], orc.MIXED)
    check = {}
    for v in variants:
        nrc._lib.check(L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), outs[v].data_ptr(), args.n, sp))
        torch.cuda.synchronize()
        y = outs[v].cpu().numpy()[idx]
        check[v] = float(np.linalg.norm(y - y_ref) / np.linalg.norm(y_ref))
    times = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), outs[v].data_ptr(), args.n, sp)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters * 1e3)
    res = {}
    for v in variants:
        t = np.array(times[v])
        med = float(np.median(t))
        res[v] = {"median_us": med, "min_us": float(t.min()), "Gq_per_s": args.n / med / 1e3,
                  "tflops_alg": 41600 * args.n / (med * 1e-6) / 1e12, "rel_l2_vs_oracle": check[v]}
    net.destroy()
    print(json.dumps({"n": args.n, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
