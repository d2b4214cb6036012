"""In-process A/B of the fused inference + accumulate_render_radiance kernel (nrc_infer_accumulate):
the 1024-thread LDS-work-queue shape (default) against the round-1 512-thread shape (NRC_ACC_THREADS=512, read per
launch), on a 1080p frame's 2,073,600 render + 32,400 train-suffix queries. Checks that both give bit-identical
frame buffers and suffix radiance.

    python tools/ab_accumulate.py [--rounds 9] [--iters 20]
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
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    npx, ntiles = 1920 * 1080, 240 * 135
    n = npx + ntiles
    q = torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=5)).to(dev)
    thr = torch.rand((npx, 3), device=dev)
    net = nrc.Network()
    net.init(stream=st)
    shapes = {"q1024": None, "r512": "512"}
    outs = {}
    for k, env in shapes.items():
        if env:
            os.environ["NRC_ACC_THREADS"] = env
        else:
            os.environ.pop("NRC_ACC_THREADS", None)
        rgba = torch.zeros((npx, 4), device=dev)
        res = torch.zeros((n, 3), device=dev)
        nrc.frame.infer_accumulate(net, q, res, n, thr, rgba, npx, nrc.frame.RenderMode.Full, 3)
        torch.cuda.synchronize()
        outs[k] = (rgba.cpu().numpy(), res.cpu().numpy()[npx:])
    same = bool(np.array_equal(outs["q1024"][0], outs["r512"][0]) and np.array_equal(outs["q1024"][1], outs["r512"][1]))
    rgba = torch.zeros((npx, 4), device=dev)
    res = torch.zeros((n, 3), device=dev)
    times = {k: [] for k in shapes}
    for _ in range(args.rounds):
        for k, env in shapes.items():
            if env:
                os.environ["NRC_ACC_THREADS"] = env
            else:
                os.environ.pop("NRC_ACC_THREADS", None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                nrc.frame.infer_accumulate(net, q, res, n, thr, rgba, npx, nrc.frame.RenderMode.Full, 3)
            e1.record(st)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / args.iters * 1e3)
    os.environ.pop("NRC_ACC_THREADS", None)
    net.destroy()
    print(json.dumps({"queries": n, "bit_identical": same,
                      "median_us": {k: float(np.median(v)) for k, v in times.items()},
                      "min_us": {k: float(np.min(v)) for k, v in times.items()}}, indent=1))


if __name__ == "__main__":
    main()
