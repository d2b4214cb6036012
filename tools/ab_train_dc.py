"""In-process A/B of the Frequency training kernels: round 2's role-split t16 kernel (train_kernel knob 1) against
the decoupled-chain kernel's shapes (train_shape knob 0..5), at the full 16,384-sample minibatch and at configs[3]'s
per-rank 2,048-sample slice (global batch 16,384). Interleaved rounds, HIP events on the handle's stream; reports the
fused step (nrc_train_batch: fwd/bwd/dW kernel + reduce/Adam/EMA) and the gradient pass (nrc_train_grad).

    python tools/ab_train_dc.py [rounds] [steps]   ->  gpurun_out/ab_train_dc.json
"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nrc_loader  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    nrc = nrc_loader.load()
    L = nrc._lib
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    B = nrc.BATCH_SIZE
    tq, tt = nrc.synthetic.cornell_batch(4 * B, seed=5)
    tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
    arms = [("split", 1, -1)] + [(f"dc{s}", -1, s) for s in range(8)]
    nets = {}
    for name, k, s in arms:
        L.set_knob("train_kernel", k)
        n = nrc.Network()
        n.init(stream=st)
        nets[name] = (n, s)
    L.set_knob("train_kernel", -1)
    grad = torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev)

    def timed(fn, k):
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(k):
            fn(i)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k * 1e3

    res = {}
    for r in range(rounds):
        for name, (n, s) in nets.items():
            L.set_knob("train_shape", s)
            for b in (B, B // 8):
                step_us = timed(lambda i: n.train_batch(tq[(i % 4) * B:], tt[(i % 4) * B:], b), steps)
                grad_us = timed(lambda i: n.train_grad(tq[(i % 4) * B:], tt[(i % 4) * B:], b, B, grad), steps)
                res.setdefault(f"{name}_b{b}", {"step_us": [], "grad_us": []})
                res[f"{name}_b{b}"]["step_us"].append(step_us)
                res[f"{name}_b{b}"]["grad_us"].append(grad_us)
        L.set_knob("train_shape", -1)
    summary = {k: {m: float(np.median(v[m])) for m in v} for k, v in res.items()}
    for k, v in summary.items():
        print(f"{k:14s} step {v['step_us']:7.2f} us   grad {v['grad_us']:7.2f} us", flush=True)
    for n, _ in nets.values():
        n.destroy()
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "gpurun_out", "ab_train_dc.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"median": summary, "raw": res, "rounds": rounds, "steps": steps}, f, indent=1)


if __name__ == "__main__":
    main()
