"""Is the headline inference kernel's time a property of the kernel or of the 256-MB last-level cache (MALL)?

A 2^21-query launch reads 126 MB of queries and writes 25 MB: the whole working set fits the MI355X's infinity cache, so
the same buffer launched back to back may be served from it. Timed here, interleaved in one process (production kernel,
bench weights, HIP events on the stream), per 2^21 queries:
  one      one 2^21-query buffer, K launches back to back (what bench.py's `value` times)
  rot2     two disjoint 2^21-query buffers alternating (302 MB working set)
  rot4     four disjoint buffers alternating (604 MB)
  big      one 2^22-query buffer (configs[3] at N = 1), time / 2
  flushed  one 2^21-query buffer, a 1-GiB buffer written between launches (each launch timed alone)

    python tools/mall_probe.py [--rounds 5 --iters 40]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    n = 1 << 21
    net = nrc.Network()
    net.init(stream=stream)
    seed = nrc.synthetic.SEED
    for f in range(4):
        tq, tt = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=seed * 31 + f)
        tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
        for b in range(4):
            net.train(tq[b * nrc.BATCH_SIZE:], tt[b * nrc.BATCH_SIZE:])
    big_np = nrc.synthetic.cornell_queries(2 * n, seed=seed)
    big = torch.from_numpy(big_np).to(dev)
    bufs = [big[:n], big[n:]] + [torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=seed + 7 + i)).to(dev)
                                 for i in range(2)]
    outs = [torch.empty((n, 3), device=dev) for _ in range(4)]
    out_big = torch.empty((2 * n, 3), device=dev)
    junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB

    def timed(fn, k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(k):
            fn(i)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k * 1e3

    def flushed(k):
        tot = 0.0
        for i in range(k):
            junk.fill_(float(i))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            net.infer(bufs[0], outs[0], n)
            e1.record(stream)
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
        return tot / k * 1e3

    cases = {
        "one": lambda k: timed(lambda i: net.infer(bufs[0], outs[0], n), k),
        "rot2": lambda k: timed(lambda i: net.infer(bufs[i & 1], outs[i & 1], n), k),
        "rot4": lambda k: timed(lambda i: net.infer(bufs[i & 3], outs[i & 3], n), k),
        "big": lambda k: timed(lambda i: net.infer(big, out_big, 2 * n), k // 2) / 2,
        "flushed": lambda k: flushed(max(5, k // 4)),
    }
    # clock settle (as bench.py): ~60 ms of launches
    timed(lambda i: net.infer(bufs[0], outs[0], n), 800)
    res = {c: [] for c in cases}
    for _ in range(args.rounds):
        for c, fn in cases.items():
            res[c].append(fn(args.iters))
    summary = {c: {"median_us_per_2^21": float(np.median(v)), "all": v} for c, v in res.items()}
    print(json.dumps(summary, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(summary, indent=1))
    net.destroy()


if __name__ == "__main__":
    main()
