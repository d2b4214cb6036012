"""In-process interleaved A/B of a knob on fused Hash training steps (default: scatter_part, the first grid level whose
scatter stores per-slice partial sums; 16 = every level through the atomic accumulator). One network per value, all
initialised alike and trained on the same batches; the parameters must stay bitwise equal across values (the grid sums
are exact integers whichever way they are accumulated). HIP events on the networks' stream.

    python tools/ab_hash_train.py [--knob scatter_part] [--values 16,0,2,4,6,8] [--rounds 7] [--iters 30]
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
    ap.add_argument("--knob", default="scatter_part")
    ap.add_argument("--values", default="16,0,2,4,6,8")
    ap.add_argument("--rounds", type=int, default=7)  # interleaved rounds per value
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--set", action="append", default=[], help="name=value knob held for the whole run")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    for kv in args.set:
        k, v = kv.split("=")
        nrc._lib.set_knob(k, int(v))
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    vals = list(dict.fromkeys(int(v) for v in args.values.split(",")))  # one network per distinct value
    nets = {}
    for v in vals:
        n = nrc.Network()
        n.init(stream=st, encoding=nrc.InputEncoding.Hash)
        nets[v] = n
    q, t = nrc.synthetic.cornell_batch(4 * nrc.BATCH_SIZE, seed=3)
    q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    B = nrc.BATCH_SIZE

    def steps(v: int, k: int, i0: int = 0) -> None:
        nrc._lib.set_knob(args.knob, v)
        for i in range(k):
            j = (i0 + i) % 4
            nets[v].train(q[j * B:(j + 1) * B], t[j * B:(j + 1) * B])

    for v in vals:
        steps(v, 8)
    torch.cuda.synchronize()
    p0 = nets[vals[0]].get_state(nrc.StateSlot.PARAMS)
    equal = {v: bool(np.array_equal(nets[v].get_state(nrc.StateSlot.PARAMS), p0)) for v in vals}
    times = {v: [] for v in vals}
    for _ in range(args.rounds):
        for v in vals:
            steps(v, 3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            steps(v, args.iters)
            e1.record(st)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters * 1e3)
    nrc._lib.set_knob(args.knob, -1)
    p1 = nets[vals[0]].get_state(nrc.StateSlot.PARAMS)  # every network ran the same steps on the same batches
    for v in vals:
        equal[v] = equal[v] and bool(np.array_equal(nets[v].get_state(nrc.StateSlot.PARAMS), p1))
    res = {v: {"median_us": float(np.median(times[v])), "min_us": float(np.min(times[v])),
               "params_bitwise_equal_to_first": equal[v]} for v in vals}
    print(json.dumps({"knob": args.knob, "held": args.set, "batch": B, "by_value": res}))
    for n in nets.values():
        n.destroy()


if __name__ == "__main__":
    main()
