"""Times the training step's pieces with HIP events: fused step, grad (fwd/bwd + reduce-only), apply-only."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main():
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    net = nrc.Network()
    net.init(stream=st)
    B = nrc.BATCH_SIZE
    q_np, t_np = nrc.synthetic.cornell_batch(B, seed=3)
    q, t = torch.from_numpy(q_np).to(dev), torch.from_numpy(t_np).to(dev)
    grad = torch.zeros(nrc.GRAD_FLOATS, device=dev)

    def timeit(fn, iters=40):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3

    res = {"fused_step_us": timeit(lambda: net.train(q, t)),
           "grad_us": timeit(lambda: net.train_grad(q, t, B, B, grad)),
           "apply_us": timeit(lambda: net.train_apply(grad))}
    net.destroy()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
