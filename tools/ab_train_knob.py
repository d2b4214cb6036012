"""In-process interleaved A/B of a library knob that is read at every training launch (e.g. train_prio, debug library):
the 16,384-sample width-64 Frequency step, HIP events on the handle's stream, rounds of `iters` steps per value in turn;
the state after the same number of steps must be bitwise equal across the values (the knob changes scheduling only).

    NRC_LIB_PATH=.../libnrc_amd_debug.so python tools/ab_train_knob.py --knob train_prio --values=-1,1,2
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
    ap.add_argument("--knob", default="train_prio")
    ap.add_argument("--values", default="-1,1,2")
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--iters", type=int, default=100)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    vals = [int(v) for v in args.values.split(",")]
    B = nrc.BATCH_SIZE
    qb, tb = nrc.synthetic.cornell_batch(4 * B, seed=77)
    qd, td = torch.from_numpy(qb).to(dev), torch.from_numpy(tb).to(dev)
    nets = {}
    for v in vals:
        n = nrc.Network()
        n.init(stream=st)
        nets[v] = n
    p0 = nets[vals[0]].get_state(nrc.StateSlot.PARAMS)
    for n in nets.values():
        n.set_state(nrc.StateSlot.PARAMS, p0)
        n.set_state(nrc.StateSlot.INFER, p0)

    def run(v, k):
        nrc._lib.set_knob(args.knob, v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(k):
            nets[v].train(qd[(i % 4) * B:], td[(i % 4) * B:])
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k * 1e3

    times = {v: [] for v in vals}
    for v in vals:
        run(v, 20)
    for _ in range(args.rounds):
        for v in vals:
            times[v].append(run(v, args.iters))
    nrc._lib.set_knob(args.knob, -1)
    states = {v: nets[v].get_state(nrc.StateSlot.PARAMS) for v in vals}
    same = {v: bool(np.array_equal(states[v], states[vals[0]])) for v in vals}
    out = {"knob": args.knob, "b": B, "by_value": {str(v): {"median_us": float(np.median(times[v])),
                                                            "min_us": float(np.min(times[v])),
                                                            "state_bitwise_equal_to_first": same[v]} for v in vals}}
    print(json.dumps(out, indent=1))
    for n in nets.values():
        n.destroy()


if __name__ == "__main__":
    main()
