"""In-process A/B of the width-64 Frequency training step: one launch (launch_train16_fused, round 6) vs the two
launches it replaces (the default; knob train_fused = 1 at nrc_init selects the fused step), and the fused step's arrival by a per-block counter (knob
fuse_mode 1) instead of per-block flags. Interleaved rounds, HIP events on the handles' stream; eager calls (the
reference's per-call API) and the same calls replayed from a HIP graph (GPU time only; a captured step takes the two
launches, so the graph figures of the fused handles time that path).

    python tools/ab_train_fused.py [--rounds 7 --steps 200] [--out f.json]
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--b", type=int, default=16384)
    ap.add_argument("--out", default=None)
    ap.add_argument("--ablations", action="store_true")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    B = args.b
    nets, modes = {}, {}
    cases = [("fused", 1, 0), ("fused_counter", 1, 1), ("two_launch", -1, -1)]
    if args.ablations:  # timing only (wrong results): no reducers / reducers that only wait
        cases += [("abl_no_reducers", 1, 3), ("abl_wait_only", 1, 4)]
    for name, v, m in cases:
        nrc._lib.set_knob("train_fused", v)
        n = nrc.Network()
        n.init(stream=stream)
        nets[name] = n
        modes[name] = m
    nrc._lib.set_knob("train_fused", -1)

    def use(name):
        nrc._lib.set_knob("fuse_mode", modes[name])
    qb, tb = nrc.synthetic.cornell_batch(4 * B, seed=nrc.synthetic.SEED * 31)
    qd, td = torch.from_numpy(qb).to(dev), torch.from_numpy(tb).to(dev)
    views = [(qd[i * B:], td[i * B:]) for i in range(4)]

    def eager(n, k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(k):
            n.train_batch(*views[i & 3], B)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k * 1e3

    graphs = {}
    cs = torch.cuda.Stream()
    for name, n in nets.items():
        use(name)
        for _ in range(4):
            n.train_batch(*views[0], B)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        n.set_stream(cs)
        with torch.cuda.graph(g, stream=cs):
            for i in range(32):
                n.train_batch(*views[i & 3], B)
        n.set_stream(stream)
        graphs[name] = g

    def replay(name, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            graphs[name].replay()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / (32 * reps) * 1e3

    res = {name: {"eager_us": [], "graph_us": []} for name in nets}
    for name, n in nets.items():
        use(name)
        eager(n, 50)
    for _ in range(args.rounds):
        for name, n in nets.items():
            use(name)
            res[name]["eager_us"].append(eager(n, args.steps))
            res[name]["graph_us"].append(replay(name, max(1, args.steps // 32)))
    summary = {name: {k: float(np.median(v)) for k, v in r.items()} | {"all": r} for name, r in res.items()}
    summary["b"] = B
    print(json.dumps({k: ({kk: vv for kk, vv in v.items() if kk != "all"} if isinstance(v, dict) else v)
                      for k, v in summary.items()}, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(summary, indent=1))
    nrc._lib.set_knob("fuse_mode", -1)
    graphs.clear()
    for n in nets.values():
        n.destroy()


if __name__ == "__main__":
    main()
