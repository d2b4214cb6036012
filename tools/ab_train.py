"""In-process A/B of the 64-wide Frequency training kernels: the t16 kernel (nrc_train16.hip, default) against the
round-1 train_kernel (NRC_TRAIN_KERNEL=32, read at nrc_init). Interleaved rounds of HIP-event timing of the fused
step, grad (fwd/bwd + reduce-only) and apply-only, plus the two kernels' gradients on the same batch compared with
each other and with the oracle (rel-L2).

    python tools/ab_train.py [--rounds 7] [--iters 40]
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=40)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    orc = nrc_loader.load_oracle()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    nets = {}
    # t16: the default; t16s: the role-split t16 kernel (NRC_T16_SPLIT=1); k32: the round-1 kernel
    for name, env, split in (("t16", None, "0"), ("t16s", None, "1"), ("k32", "32", "0")):
        if env:
            os.environ["NRC_TRAIN_KERNEL"] = env
        else:
            os.environ.pop("NRC_TRAIN_KERNEL", None)
        os.environ["NRC_T16_SPLIT"] = split
        n = nrc.Network()
        n.init(stream=st)
        nets[name] = n
    os.environ.pop("NRC_TRAIN_KERNEL", None)
    os.environ.pop("NRC_T16_SPLIT", None)
    B = nrc.BATCH_SIZE
    q_np, t_np = nrc.synthetic.cornell_batch(B, seed=3)
    q, t = torch.from_numpy(q_np).to(dev), torch.from_numpy(t_np).to(dev)
    grads = {k: torch.zeros(nrc.GRAD_FLOATS, device=dev) for k in nets}

    # gradients on the same (initial) weights
    for k, n in nets.items():
        n.train_grad(q, t, B, B, grads[k])
    torch.cuda.synchronize()
    params = nets["t16"].get_state(nrc.StateSlot.PARAMS)
    g_ref, loss_ref = orc.grad(params, q_np, t_np, mode=orc.MIXED)
    P = nrc.NUM_PARAMS
    rel = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))  # noqa: E731
    gk = {k: v.cpu().numpy() for k, v in grads.items()}
    check = {k: {"grad_rel_l2_vs_oracle": rel(gk[k][:P], g_ref),
                 "loss": float(gk[k][P]), "loss_oracle": float(loss_ref)} for k in nets}
    check["t16_vs_k32_rel_l2"] = rel(gk["t16"][:P], gk["k32"][:P])
    check["t16s_vs_t16_max_abs"] = float(np.abs(gk["t16s"] - gk["t16"]).max())

    def timeit(fn, iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3

    times = {k: {"fused_step_us": [], "grad_us": [], "apply_us": []} for k in nets}
    for k, n in nets.items():  # warm-up
        for _ in range(5):
            n.train(q, t)
    for _ in range(args.rounds):
        for k, n in nets.items():
            times[k]["fused_step_us"].append(timeit(lambda: n.train(q, t), args.iters))
            times[k]["grad_us"].append(timeit(lambda: n.train_grad(q, t, B, B, grads[k]), args.iters))
            times[k]["apply_us"].append(timeit(lambda: n.train_apply(grads[k]), args.iters))
    res = {k: {m: float(np.median(v)) for m, v in d.items()} for k, d in times.items()}
    for n in nets.values():
        n.destroy()
    print(json.dumps({"median_us": res, "check": check}, indent=1))


if __name__ == "__main__":
    main()
