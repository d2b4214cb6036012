"""Why bench.py's event-timed inference differs from tools/ab_infer.py: times the same default kernel through
Network.infer (the product path, as bench.py calls it) and through nrc_debug_infer_variant (as ab_infer.py calls it),
interleaved, in one process, with per-launch events on the launch stream and the host time per call.

    python tools/infer_timing_probe.py [--n 2097152] [--iters 200] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 21)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = int(stream.cuda_stream)
    seed = nrc.synthetic.SEED
    q = torch.from_numpy(nrc.synthetic.cornell_queries(args.n, seed=seed)).to(dev)
    out = torch.empty((args.n, 3), dtype=torch.float32, device=dev)
    net = nrc.Network()
    net.init(stream=stream, encoding=nrc.InputEncoding.Frequency)
    for f in range(4):
        tq, tt = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=seed * 31 + f)
        tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
        for b in range(4):
            net.train(tq[b * nrc.BATCH_SIZE:], tt[b * nrc.BATCH_SIZE:])
    torch.cuda.synchronize()
    qp, op = q.data_ptr(), out.data_ptr()

    def run(how: str) -> dict:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.iters):
            if how == "net.infer":
                net.infer(q, out, args.n)
            elif how == "nrc_infer(int ptrs)":
                L.nrc_infer(net._h, qp, op, args.n)
            else:
                L.nrc_debug_infer_variant(net._h, 47, qp, op, args.n, sp)
        t_host = time.perf_counter() - t0
        e1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return {"event_us": e0.elapsed_time(e1) / args.iters * 1e3, "host_enqueue_us": t_host / args.iters * 1e6,
                "wall_us": wall / args.iters * 1e6}

    hows = ["net.infer", "nrc_infer(int ptrs)", "debug variant 47"]
    res = {h: [] for h in hows}
    for _ in range(args.rounds):
        for h in hows:
            res[h].append(run(h))
    # per-launch events through the product path
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
    torch.cuda.synchronize()
    evs[0].record(stream)
    for i in range(args.iters):
        net.infer(q, out, args.n)
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    per = np.array([evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(args.iters)])
    summary = {h: {k: float(np.median([r[k] for r in res[h]])) for k in res[h][0]} for h in hows}
    summary["per_launch_us_p0_10_50_90_100"] = [float(np.percentile(per, p)) for p in (0, 10, 50, 90, 100)]
    summary["per_launch_us_first10"] = [round(float(x), 1) for x in per[:10]]
    summary["per_launch_us_last10"] = [round(float(x), 1) for x in per[-10:]]
    print(json.dumps(summary, indent=1))
    net.destroy()


if __name__ == "__main__":
    main()
