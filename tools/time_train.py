"""Median fused training step (µs) of one configuration, one line of output (cross-build A/B with
tools/ab_cmd_libs.sh).   python tools/time_train.py [--encoding Hash] [--width 64] [--rounds 9] [--iters 40]"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--encoding", default="Frequency")
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--knob", action="append", default=[], help="name=value A/B knob of the library (repeatable)")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    for kv in args.knob:
        k, v = kv.split("=")
        nrc._lib.set_knob(k, int(v))
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    e = getattr(nrc.InputEncoding, args.encoding)
    net = nrc.Network()
    net.init(stream=st, encoding=e, config=nrc.default_config(e, width=args.width))
    q, t = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=3)
    q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    for _ in range(5):
        net.train(q, t)
    ts = []
    for _ in range(args.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.iters):
            net.train(q, t)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / args.iters * 1e3)
    loss = net.train(q, t, loss=True)
    net.destroy()
    print(f"{args.encoding} w{args.width} {' '.join(args.knob)} step_us {np.median(ts):.2f} loss {loss:.6g}")


if __name__ == "__main__":
    main()
