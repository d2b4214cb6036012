"""Per-kernel and whole-frame timing of the post-trace NRC sequence at 1080p:
infer -> accumulate -> propagate -> shuffle -> 4 x train, on a synthetic Cornell frame resident in HBM.

    python tools/bench_frame.py [--iters 50] [--width 1920 --height 1080 --tile 8]

Each step is timed with HIP events on the stream it runs on (the network's stream = torch's current stream),
averaged over --iters launches. Algorithmic bytes per launch are stated next to each kernel.
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
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tile", type=int, default=8)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    F = nrc.frame
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    f = nrc.synthetic.cornell_frame(args.width, args.height, (args.tile, args.tile), seed=1)
    cap = F.NUM_TRAINING_RECORDS_PER_FRAME
    nrec = min(f.num_training_records, cap)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    pad = lambda a, w: np.concatenate([a[:nrec], np.zeros((cap - nrec, w), np.float32)])  # noqa: E731
    rec = np.zeros(cap, F.TRAINING_RECORD_DTYPE)
    rec[:nrec] = f.train_records[:nrec]
    S, T = f.screen_size, f.num_tiles
    fb = F.FrameBuffers(t(f.queries_inference), torch.zeros((S + T, 3), device=dev), t(f.last_render_throughput),
                        torch.zeros((S, 4), device=dev), F.records_to_device(f.end_vertices, dev),
                        F.records_to_device(rec, dev), [t(pad(f.train_queries, 15)), torch.zeros((cap, 15), device=dev)],
                        [t(pad(f.train_targets, 3)), torch.zeros((cap, 3), device=dev)])
    net = nrc.Network()
    net.init(stream=stream)

    def timed(fn, iters=args.iters):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3  # us

    out = {"frame": {"width": args.width, "height": args.height, "tile": args.tile, "screen": S, "tiles": T,
                     "train_records": f.num_training_records}}
    us = {}
    # render part: unfused (infer + accumulate) vs fused, interleaved rounds in one process (box clocks drift)
    ab = {"infer": lambda: net.infer(fb.queries_inference, fb.results_inference, S + T),
          "accumulate_full": lambda: F.accumulate_render_radiance(fb.results_inference, fb.last_render_throughput,
                                                                  fb.output_rgba, S, F.RenderMode.Full, 3),
          "infer_accumulate_fused": lambda: F.infer_accumulate(net, fb.queries_inference, fb.results_inference,
                                                               S + T, fb.last_render_throughput, fb.output_rgba, S,
                                                               F.RenderMode.Full, 3)}
    rounds = {k: [] for k in ab}
    for _ in range(7):
        for k, fn in ab.items():
            rounds[k].append(timed(fn, iters=max(args.iters // 5, 4)))
    for k in ab:
        us[k] = float(np.median(rounds[k]))
    us["propagate"] = timed(lambda: F.propagate_train_radiance(fb.end_vertices, fb.results_inference[S:], T,
                                                               fb.train_records, fb.train_targets[0], nrec))
    us["permute_feistel"] = timed(lambda: F.permute_train_data(fb.train_queries[0], fb.train_targets[0], None, 1, 0,
                                                               nrec, fb.train_queries[1], fb.train_targets[1]))
    us["train_step_async"] = timed(lambda: net.train(fb.train_queries[1], fb.train_targets[1]), iters=20)
    params = F.FrameParams(S, T, f.num_training_records, F.RenderMode.Full, 3, 0, 1)
    unfused = F.FrameParams(S, T, f.num_training_records, F.RenderMode.Full, 3, 0, 1, keep_render_results=True)
    us["process_frame_async"] = timed(lambda: F.process_frame(net, fb, params, loss=False), iters=20)
    us["process_frame_async_unfused"] = timed(lambda: F.process_frame(net, fb, unfused, loss=False), iters=20)
    # with the reference's per-minibatch loss read-back (host syncs, Device.cpp:1503-1509): wall clock
    F.process_frame(net, fb, params, loss=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        F.process_frame(net, fb, params, loss=True)
    torch.cuda.synchronize()
    us["process_frame_with_loss_wall"] = (time.perf_counter() - t0) / 20 * 1e6
    b = {"infer": 72 * (S + T), "accumulate_full": 56 * S, "infer_accumulate_fused": 60 * (S + T) + 12 * T + 44 * S,
         "propagate": 28 * T + 40 * nrec,  # end vertex+radiance per tile; record (16 B used) + target r/w per record
         "permute_feistel": 144 * cap}
    out["us"] = us
    out["algorithmic_bytes"] = b
    out["hbm_gbs_algorithmic"] = {k: b[k] / (us[k] * 1e-6) / 1e9 for k in b}
    net.destroy()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
