"""In-process A/B of the cache policy of the role-split t16 training kernel's slab stores (NRC_T16_SLAB_AUX, read
per launch): 2 = nt (default), 16 = sc1, 18 = nt sc1. Times the fused training step and checks that the gradients
are bitwise equal.

    python tools/ab_slab_aux.py [--rounds 15] [--iters 60]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--iters", type=int, default=60)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    net = nrc.Network()
    net.init(stream=st)
    B = nrc.BATCH_SIZE
    q_np, t_np = nrc.synthetic.cornell_batch(B, seed=3)
    q, t = torch.from_numpy(q_np).to(dev), torch.from_numpy(t_np).to(dev)
    auxes = ["2", "16", "18"]
    grads = {}
    for a in auxes:
        os.environ["NRC_T16_SLAB_AUX"] = a
        g = torch.zeros(nrc.GRAD_FLOATS, device=dev)
        net.train_grad(q, t, B, B, g)
        torch.cuda.synchronize()
        grads[a] = g.cpu().numpy()
    same = all(np.array_equal(grads["2"], grads[a]) for a in auxes)
    times = {a: [] for a in auxes}
    for _ in range(args.rounds):
        for a in auxes:
            os.environ["NRC_T16_SLAB_AUX"] = a
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                net.train(q, t)
            e1.record(st)
            torch.cuda.synchronize()
            times[a].append(e0.elapsed_time(e1) / args.iters * 1e3)
    os.environ.pop("NRC_T16_SLAB_AUX", None)
    net.destroy()
    print(json.dumps({"gradients_bit_identical": same,
                      "fused_step_us_median": {a: float(np.median(v)) for a, v in times.items()}}, indent=1))


if __name__ == "__main__":
    main()
