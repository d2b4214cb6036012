"""Time course of the headline inference kernel over a long run of back-to-back launches: event-timed chunks of
--chunk launches, on bench.py's weights (4 frames of self-training) and on more-trained weights, to separate the chip's
clock ramp from the effect of the weights' activation statistics on the power-limited clock.

    python tools/infer_trajectory.py [--variant 47] [--chunks 30] [--chunk 100]
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
    ap.add_argument("--variant", type=int, default=47)
    ap.add_argument("--chunks", type=int, default=30)
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--frames", default="4,26,100", help="self-training frames before each trajectory")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = int(stream.cuda_stream)
    seed = nrc.synthetic.SEED
    q = torch.from_numpy(nrc.synthetic.cornell_queries(args.n, seed=seed)).to(dev)
    out = torch.empty((args.n, 3), device=dev)
    net = nrc.Network()
    net.init(stream=stream)
    frames = []
    for f in range(4):
        tq, tt = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=seed * 31 + f)
        frames.append((torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)))
    done = 0
    res = {"n": args.n, "variant": args.variant, "chunk": args.chunk, "runs": []}
    for target in [int(x) for x in args.frames.split(",")]:
        while done < target:
            tq, tt = frames[done % 4]
            for b in range(4):
                net.train(tq[b * nrc.BATCH_SIZE:], tt[b * nrc.BATCH_SIZE:])
            done += 1
        torch.cuda.synchronize()
        us = []
        for _ in range(args.chunks):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.chunk):
                L.nrc_debug_infer_variant(net._h, args.variant, q.data_ptr(), out.data_ptr(), args.n, sp)
            e1.record(stream)
            torch.cuda.synchronize()
            us.append(e0.elapsed_time(e1) / args.chunk * 1e3)
        y = out.cpu().numpy()
        res["runs"].append({"train_frames": done, "us_per_launch_by_chunk": [round(u, 2) for u in us],
                            "zero_output_frac": float((y == 0).mean())})
        print(json.dumps(res["runs"][-1]), flush=True)
    net.destroy()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
