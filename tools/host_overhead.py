"""Host cost per training call against the GPU time per step (16,384 samples): is the eager step host-bound?

    python tools/host_overhead.py [--iters 2000]

(a) the Python mirror (Network.train: argument checks + ctypes), (b) the bare ctypes call of nrc_train with
precomputed pointers, (c) the GPU's own step time (events around a burst, host far ahead), each as microseconds per
call; the host columns are wall time of the issuing loop only (the GPU queue absorbs the launches while it is behind).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    net = nrc.Network()
    net.init(stream=st)
    q, t = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=3)
    q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    L = nrc._lib.lib()
    pq, pt = q.data_ptr(), t.data_ptr()
    for _ in range(50):
        net.train(q, t)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("python_mirror", lambda: net.train(q, t)),
                     ("bare_ctypes", lambda: L.nrc_train(net._h, pq, pt, None))):
        # host issue rate with the GPU kept busy: the loop's wall time per call; then the GPU's own rate
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(st)
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        host = (time.perf_counter() - t0) / args.iters * 1e6
        e1.record(st)
        torch.cuda.synchronize()
        res[name] = {"host_us_per_call": host, "gpu_us_per_step": e0.elapsed_time(e1) / args.iters * 1e3}
    net.destroy()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
