"""Training-step time eager vs replayed from a HIP graph, to separate the GPU's work from the host's launch cost.

Eager: K calls through the Python mirror (ctypes -> C-ABI -> hipLaunchKernel per kernel), event-timed.
Graph: the same K calls captured once into a HIP graph (the handle's stream set to the capture stream, so the library's
launches -- and the world-1 RCCL all-reduce of nrc_train_dp -- are recorded), then replayed; per-step time = replay
time / K. The gap between the two is host overhead: Python + ctypes + one hipLaunchKernel (~3.5 us, MI355X_MICROARCH.md
graph-replay-floor) per kernel.

    python tools/step_graph_probe.py [--k 32] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="run only the cases whose name contains this")
    ap.add_argument("--knob", action="append", default=[], help="name=value A/B knob of the library (repeatable)")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    for kv in args.knob:
        k, v = kv.split("=")
        nrc._lib.set_knob(k, int(v))
    dev = torch.device("cuda:0")
    main_stream = torch.cuda.current_stream()
    B = nrc.BATCH_SIZE
    q, t = nrc.synthetic.cornell_batch(4 * B, seed=3)
    q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    net = nrc.Network()
    net.init(stream=main_stream)
    grad = torch.zeros(net.grad_floats, dtype=torch.float32, device=dev)
    comm = nrc.Communicator(nrc.Communicator.unique_id(), 1, 0)
    b8 = B // 8
    cases = {
        "train_16384": lambda i: net.train(q[(i % 4) * B:], t[(i % 4) * B:]),
        "train_batch_2048": lambda i: net.train_batch(q[(i % 4) * B:], t[(i % 4) * B:], b8),
        "train_grad_2048_of_16384": lambda i: net.train_grad(q[(i % 4) * B:], t[(i % 4) * B:], b8, B, grad),
        "train_apply": lambda i: net.train_apply(grad),
        "train_dp_2048_of_16384_world1": lambda i: net.train_dp(q[(i % 4) * B:], t[(i % 4) * B:], b8, B),
    }
    res = {"k": args.k, "reps": args.reps, "cases": {}}
    for name, fn in cases.items():
        if args.only not in name:
            continue
        if "dp" in name:
            net.set_comm(comm)
        for i in range(4):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_stream)
        for i in range(args.k * args.reps):
            fn(i)
        e1.record(main_stream)
        torch.cuda.synchronize()
        eager_us = e0.elapsed_time(e1) / (args.k * args.reps) * 1e3
        # capture K steps on a side stream that the handle launches on
        cs = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        net.set_stream(cs)
        with torch.cuda.graph(g, stream=cs):
            for i in range(args.k):
                fn(i)
        net.set_stream(main_stream)
        torch.cuda.synchronize()
        for _ in range(2):
            g.replay()
        torch.cuda.synchronize()
        e0.record(main_stream)
        for _ in range(args.reps):
            g.replay()
        e1.record(main_stream)
        torch.cuda.synchronize()
        graph_us = e0.elapsed_time(e1) / (args.k * args.reps) * 1e3
        if "dp" in name:
            net.set_comm(None)
        res["cases"][name] = {"eager_us_per_step": round(eager_us, 2), "graph_us_per_step": round(graph_us, 2)}
        print(name, res["cases"][name], flush=True)
    comm.destroy()
    net.destroy()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
