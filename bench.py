"""Benchmark of the NRC hot path on MI355X (BASELINE.json metric).

N = 1 — configs[1]: a step = one ``infer`` over 2^21 synthetic Cornell queries resident in HBM (the 1080p 1spp
batch); configs[2]: the per-frame self-training (4 x 16,384-sample steps) reported as ``train_step_ms``.

N > 1 — configs[3] (C4): the 2K frame's 2^22 queries sharded contiguously over the ranks
(2^19 per GPU at 8; strong scaling, no collective on the inference path), and every 16,384-sample minibatch split
into 16,384 / N per rank with the gradients combined INSIDE the library (nrc_train_dp: global batch 16,384, the
reference's per-step semantics) -- through the one-shot peer exchange inside the reduction when every rank could open it
and run a frame through it (``train_dp_path``), else over the RCCL communicator (nrc_set_comm); the all-reduce figure
is kept beside it (``train_step_allreduce_ms``). The weak-scaling figures (2^21 queries per GPU) are kept as the extra key
``weak``.

Launch: ``python bench.py [--gpus N --steps K --warmup W]``. N > 1 either under torch.distributed.run (WORLD_SIZE set) or
on its own: with WORLD_SIZE unset the process starts N fresh child processes of itself (one rank per GPU, RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in their environment) before it makes any GPU call, passes rank 0's
JSON line through and exits non-zero if any rank fails (``launch_ranks``).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402

FLOP_PER_QUERY = 2 * (66 * 64 + 4 * 64 * 64 + 64 * 3)  # 41,600 algorithmic
BYTES_PER_QUERY = 60 + 12
TRAIN_FLOP_PER_SAMPLE = 116_352
PEAK_F16_TFLOPS = 2500.0  # MI355X dense f16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0  # MI355X dense fp8 (MX-scaled) MFMA
FLOP_PER_QUERY_WIDE = 2 * (66 * 128 + 4 * 128 * 128 + 128 * 3)  # 148,736
PEAK_HBM_GBS = 8000.0
QUERIES_PER_GPU = 1 << 21
QUERIES_C4 = 1 << 22  # configs[3]: the 2K frame, sharded over the ranks
ROUND = "r06"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--queries", type=int, default=QUERIES_PER_GPU, help="queries per GPU per step")
    ap.add_argument("--train-frames", type=int, default=20, help="timed frames of 4 x 16384 training")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample duration")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-wide", action="store_true", help="skip the configs[4] width-128 f16/FP8 inference lines")
    ap.add_argument("--no-hash", action="store_true", help="skip the InputEncoding::Hash line")
    ap.add_argument("--no-c4", action="store_true", help="N = 1: skip the configs[3] per-rank measurement")
    ap.add_argument("--no-peer", action="store_true", help="N > 1: skip the one-shot peer-exchange training leg")
    ap.add_argument("--sustained", type=int, default=4000,
                    help="N = 1: sustained-inference launches timed after as many untimed ones (0: skip)")
    ap.add_argument("--settle-ms", type=float, default=60.0,
                    help="untimed inference launches before the warmup steps until this much GPU time has passed: the "
                         "chip's clock ramps up over the first ~30 ms of load (profiles/r03_infer/trajectory_v39.log)")
    ap.add_argument("--frame-iters", type=int, default=20, help="timed 1080p post-trace frames (0: skip)")
    ap.add_argument("--rehearse-comm", action="store_true",
                    help="N = 1 only: train through a world-1 RCCL communicator (nrc_train_dp), to rehearse the N > 1 "
                         "training path on one GPU")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only to rehearse several ranks on one "
                         "GPU, which is not a measurement)")
    return ap.parse_args()


def cpu_baseline(queries: np.ndarray, params: np.ndarray, target_s: float, train_batch, gpu_out=None) -> dict:
    """The naive C oracle (FP32, scalar loops) on the host cores, bounded sample of the workload. Its first pass over
    the frame doubles as the checker of the timed GPU inference (gpu_out: the bench's last output buffer)."""
    orc = nrc_loader.load_oracle()
    threads, cores_how = orc.host_cores()
    # configs[0] (C1): the FP32 forward of 4096 queries on every host core (best of 3 after one warm-up)
    n = 4096
    orc.forward(params, queries[:n], orc.FP32, threads)
    c1 = []
    for _ in range(3):
        t0 = time.perf_counter()
        orc.forward(params, queries[:n], orc.FP32, threads)
        c1.append(time.perf_counter() - t0)
    dt = min(c1)
    # whole passes over the frame while they fit the budget, then a partial pass to reach ~target_s
    want = int(max(n, n * target_s / max(dt, 1e-6)))
    total = 0
    first = None
    t0 = time.perf_counter()
    while total < want:
        m = min(len(queries), want - total)
        y = orc.forward(params, queries[:m], orc.FP32, threads)
        if first is None:
            first = y
        total += m
    dt = time.perf_counter() - t0
    parity = None
    if gpu_out is not None and first is not None:
        ref = first.astype(np.float64)
        got = gpu_out[:len(ref)].astype(np.float64)
        parity = {"rel_l2_vs_oracle_fp32": float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)),
                  "queries": int(len(ref)), "tolerance": 1e-3,
                  "what": "the timed inference's output buffer vs the FP32 oracle forward of the same queries"}
    # the same forward on one thread (bounded sample) and one 16,384-sample train step
    n1 = 8192
    t1 = time.perf_counter()
    orc.forward(params, queries[:n1], orc.FP32, 1)
    dt1 = time.perf_counter() - t1
    tq, tt = train_batch
    t2 = time.perf_counter()
    g, _ = orc.grad(params, tq, tt, mode=orc.FP32, threads=threads)
    orc.AdamEmaState(params).apply(g)
    dt2 = time.perf_counter() - t2
    return {"value": total / dt / 1e6, "unit": "M queries/s", "cores": threads, "kind": "port",
            "cpu_model": orc.cpu_model(), "cores_how": cores_how,
            "sample": f"{total} queries ({total / len(queries):.2f} passes over the {len(queries)}-query "
                      f"Cornell frame), oracle/nrc_oracle.c FP32 forward, "
                      f"{threads} pthreads on {orc.cpu_model()} "
                      f"({os.cpu_count()} logical CPUs on the host; {cores_how}), {dt:.1f} s",
            "c1_ms": min(c1) * 1e3,
            "c1_what": f"configs[0]: FP32 forward of 4096 Cornell queries, {threads} pthreads, best of 3",
            "value_1thread": n1 / dt1 / 1e6, "sample_1thread": f"{n1} queries on 1 thread, {dt1:.2f} s",
            "train_step_ms": dt2 * 1e3,
            "sample_train": f"one {len(tq)}-sample step: FP32 encode+fwd+loss+bwd ({threads} pthreads) + Adam/EMA",
            "parity": parity}


def frame_bench(nrc, net, dev, iters: int) -> dict:
    """Wall-clock ms of nrc_process_frame on a synthetic 1920x1080 Cornell frame (8x8 tiles) resident in HBM."""
    import torch
    F = nrc.frame
    f = nrc.synthetic.cornell_frame(1920, 1080, (8, 8), seed=1)
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
    state = [net.get_state(s) for s in (nrc.StateSlot.PARAMS, nrc.StateSlot.INFER)]

    def frames() -> float:
        for it in range(3):
            F.process_frame(net, fb, F.FrameParams(S, T, f.num_training_records, F.RenderMode.Full, it, it, 1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(iters):
            F.process_frame(net, fb, F.FrameParams(S, T, f.num_training_records, F.RenderMode.Full, it, it, 1))
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e3

    ms = frames()
    # the reference's shuffle contract (NRCUtil.cu:19-35, Device.cpp:1427-1469): the renderer's 65,536 random u32 keys,
    # stable-sorted with their indices -- nrc_sort_train_permutation inside the frame driver (shuffle_keys_d)
    keys = torch.randint(0, 1 << 31, (cap,), dtype=torch.int32, device=dev)
    fb.shuffle_keys = keys
    ms_keys = frames()
    fb.shuffle_keys = None
    perm = torch.empty(cap, dtype=torch.int32, device=dev)
    temp = torch.empty(max(1, F.sort_train_permutation_temp_bytes(cap)), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    for _ in range(3):
        F.sort_train_permutation(keys, perm, cap, temp=temp)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        F.sort_train_permutation(keys, perm, cap, temp=temp)
    e1.record(stream)
    torch.cuda.synchronize()
    sort_ms = e0.elapsed_time(e1) / iters
    for s, v in zip((nrc.StateSlot.PARAMS, nrc.StateSlot.INFER), state):  # leave the network as it was
        net.set_state(s, v)
    return {"frame_ms": ms, "key_sort_frame_ms": ms_keys, "key_sort_ms": sort_ms, "queries": S + T,
            "train_records": f.num_training_records, "iters": iters,
            "what": "nrc_process_frame: fused infer+accumulate, propagate, Feistel shuffle, 4 x 16384 train with "
                    "loss read-back; synthetic 1920x1080 Cornell frame, 8x8 tiles. key_sort_frame_ms: the same frame "
                    "shuffled by the reference's contract (65,536 caller keys, stable LSD radix sort, "
                    "nrc_sort_train_permutation); key_sort_ms: that sort alone (HIP events)"}


def hash_bench(nrc, dev, iters: int) -> dict:
    """the InputEncoding::Hash model (16-level HashGrid + OneBlob + Identity -> 64x5 MLP) on
    one GPU: 2^21-query inference and the 16,384-sample training step (encode -> fwd -> loss -> bwd -> grid scatter
    -> Adam), HIP events on the network's stream, after 8 warm-up steps (random-init weights)."""
    import torch

    stream = torch.cuda.current_stream()
    net = nrc.Network()
    net.init(stream=stream, encoding=nrc.InputEncoding.Hash)
    n = QUERIES_PER_GPU
    q = torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=nrc.synthetic.SEED + 2000)).to(dev)
    out = torch.empty((n, 3), dtype=torch.float32, device=dev)
    tq, tt = nrc.synthetic.cornell_batch(4 * nrc.BATCH_SIZE, seed=nrc.synthetic.SEED + 2001)
    tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
    B = nrc.BATCH_SIZE

    def timed(fn, k: int) -> float:
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(k):
            fn(i)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    for f in range(8):
        net.train(tq[(f % 4) * B:], tt[(f % 4) * B:])
    # clock settle as for the headline kernel (main(): the first few hundred back-to-back launches after idle run while
    # the clock ramps): ~60 ms of untimed launches first (round 5: 20 timed launches straight after the training steps
    # read 212-217 us where the same launches back to back for 1.5 s run 180 us, profiles/r05_end/power_paths.json)
    settled = 0.0
    while settled < 60.0:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(25):
            net.infer(q, out, n)
        e1.record(stream)
        torch.cuda.synchronize()
        settled += e0.elapsed_time(e1)
    infer_ms = timed(lambda i: net.infer(q, out, n), iters)
    train_ms = timed(lambda i: net.train(tq[(i % 4) * B:], tt[(i % 4) * B:]), 4 * iters)
    # tiny-cuda-nn's f16-accumulate numerics for the same queries (NRC_PRECISION_F16_ACC16, round 5): its price per launch,
    # as 3 interleaved rounds of both modes (the median round of each; as tcnn_numerics_bench)
    out_t = torch.empty_like(out)
    pair = {"default": [], "tcnn": []}
    for _ in range(3):
        pair["default"].append(timed(lambda i: net.infer(q, out, n), iters))
        pair["tcnn"].append(timed(lambda i: net.infer_precision(nrc.PRECISION_F16_ACC16, q, out_t, n), iters))
    tcnn_ms = statistics.median(pair["tcnn"])
    tcnn_vs = tcnn_ms / statistics.median(pair["default"])
    net.infer(q, out, n)  # the default kernel's output with the same (trained-since) weights
    torch.cuda.synchronize()
    d = float(torch.linalg.vector_norm(out_t - out) / torch.linalg.vector_norm(out))
    net.destroy()
    return {"workload": "SURVEY 8(f) row 3: InputEncoding::Hash, 2^21-query inference + 16384-sample train step",
            "M_queries_per_s": n / (infer_ms * 1e-3) / 1e6, "infer_kernel_ms": infer_ms, "train_step_ms": train_ms,
            "infer_f16_acc16_ms": tcnn_ms, "f16_acc16_slowdown_interleaved": tcnn_vs, "f16_acc16_vs_default_rel_l2": d,
            "bound": "feature pass (one level table per CU in LDS: random LDS gathers + VALU) + MLP pass, DESIGN.md section 10"}


def tcnn_numerics_bench(nrc, net, q, out, n: int, iters: int) -> dict:
    """The price of north_star's 1e-3-vs-tiny-cuda-nn tolerance on random weights: the 2^21-query launch with tcnn's
    f16-accumulate numerics (NRC_PRECISION_F16_ACC16: an f16 accumulator rounded after every 16-wide K chunk) next to the
    default f32-accumulate kernel, same weights and queries, HIP events on the network's stream: 5 interleaved rounds
    of `iters` launches per mode (after 3 untimed launches of that mode), the median round of each -- both kernels run at
    the package power limit, so a single burst right after the other mode's reads the other's clock state."""
    import torch

    stream = torch.cuda.current_stream()
    out_t = torch.empty_like(out)

    def timed(fn, k: int) -> float:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    rounds = {"default": [], "tcnn": []}
    for _ in range(5):
        rounds["default"].append(timed(lambda: net.infer(q, out, n), iters))
        rounds["tcnn"].append(timed(lambda: net.infer_precision(nrc.PRECISION_F16_ACC16, q, out_t, n), iters))
    default_ms, tcnn_ms = statistics.median(rounds["default"]), statistics.median(rounds["tcnn"])
    d = float(torch.linalg.vector_norm(out_t - out) / torch.linalg.vector_norm(out))
    return {"workload": "Frequency 64x5, 2^21 queries, bench weights", "default_ms": default_ms,
            "f16_acc16_ms": tcnn_ms, "slowdown": tcnn_ms / default_ms, "f16_acc16_vs_default_rel_l2": d,
            "iters": iters, "rounds": 5}


def wide_bench(nrc, dev, world: int, rank: int, steps: int, barrier) -> dict:
    """BASELINE configs[4] (C5): the width-128 network on the ~8M-query 4K frame, sharded over the ranks
    (2^23 / world queries per GPU, no collective), f16 and FP8 inference; HIP events on the launch stream and the
    max-over-ranks wall time."""
    import torch
    import torch.distributed as dist

    nq = (1 << 23) // world
    q = torch.from_numpy(nrc.synthetic.cornell_queries(nq, seed=nrc.synthetic.SEED + 1000 + rank)).to(dev)
    out = torch.empty((nq, 3), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()
    net = nrc.Network()
    net.init(stream=stream, encoding=nrc.InputEncoding.Frequency,
             config=nrc.default_config(nrc.InputEncoding.Frequency, width=128))
    res = {"workload": "configs[4]: 128-wide 5-hidden-layer MLP + Frequency encoding, 4K frame of 2^23 queries "
                       "sharded over the GPUs (xavier-init weights)", "queries_per_gpu": nq,
           "flop_per_query": FLOP_PER_QUERY_WIDE}
    for prec, name, peak in ((nrc.PRECISION_F16, "f16", PEAK_F16_TFLOPS), (nrc.PRECISION_FP8, "fp8", PEAK_FP8_TFLOPS)):
        # clock settle as for the headline kernel: >= 60 ms of untimed launches (the first ones run while the clock
        # ramps; a 1.5-s back-to-back run of the FP8 path takes 631.6 us per launch, profiles/r05_end/power_paths.json)
        settled = 0.0
        while settled < 60.0:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(5):
                net.infer_precision(prec, q, out, nq, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            settled += e0.elapsed_time(e1)
        barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(steps):
            net.infer_precision(prec, q, out, nq, stream=stream)
        ev1.record(stream)
        barrier()
        wall = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(wall, op=dist.ReduceOp.MAX)
        kms = ev0.elapsed_time(ev1) / steps
        tf = FLOP_PER_QUERY_WIDE * nq / (kms * 1e-3) / 1e12
        res[name] = {"M_queries_per_s": world * nq * steps / float(wall.item()) / 1e6, "kernel_ms": kms,
                     "achieved_tflops": tf, "peak_tflops": peak, "frac": tf / peak}
    if world == 1:
        # the width-128 training step (16,384 samples: encode -> fwd -> loss -> bwd -> dW -> Adam/EMA -> repack)
        B = nrc.BATCH_SIZE
        tq, tt = nrc.synthetic.cornell_batch(4 * B, seed=nrc.synthetic.SEED + 1001)
        tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
        for i in range(4):
            net.train(tq[i * B:], tt[i * B:])
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k = 4 * max(5, steps // 2)
        ev0.record(stream)
        for i in range(k):
            net.train(tq[(i % 4) * B:], tt[(i % 4) * B:])
        ev1.record(stream)
        torch.cuda.synchronize()
        res["train_step_ms"] = ev0.elapsed_time(ev1) / k
    net.destroy()
    return res


def graph_ms_per_call(net, stream, fn, k: int, reps: int) -> float:
    """k calls of fn captured into a HIP graph (the handle launches on the capture stream meanwhile), replayed reps
    times: event-timed ms per call on the GPU, host launch cost excluded."""
    import torch

    cs = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    net.set_stream(cs)
    try:
        with torch.cuda.graph(g, stream=cs):
            for i in range(k):
                fn(i)
    finally:
        net.set_stream(stream)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        g.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) / (k * reps)


def c4_frame_n1(nrc, net, dev, steps: int, warmup: int, barrier) -> dict:
    """configs[3]'s workload at N = 1: the 2K frame's 2^22 queries (the same seeded frame the N > 1 ranks shard,
    bench.main) through one GPU's inference, K timed steps between barriers; `value` comparable to the N > 1 line's."""
    import torch

    stream = torch.cuda.current_stream()
    n = QUERIES_C4
    q = torch.from_numpy(nrc.synthetic.cornell_queries(n, seed=nrc.synthetic.SEED)).to(dev)
    out = torch.empty((n, 3), dtype=torch.float32, device=dev)
    # clock settle as main()'s: making the frame leaves the GPU idle for seconds, and a first round's 20 + 50 launches
    # then ran inside the clock ramp (185 us per 2^22 launch against 156 settled; tools/mall_probe.py)
    settled = 0.0
    while settled < 60.0:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(25):
            net.infer(q, out, n)
        e1.record(stream)
        torch.cuda.synchronize()
        settled += e0.elapsed_time(e1)
    for _ in range(max(warmup, 5)):
        net.infer(q, out, n)
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        net.infer(q, out, n)
    ev1.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    kms = ev0.elapsed_time(ev1) / steps
    del q, out
    return {"workload": "configs[3] at N = 1: the 2K frame's 2^22 queries on one GPU (measured, not extrapolated)",
            "queries": n, "steps": steps, "value": n * steps / wall / 1e6, "unit": "M queries/s",
            "ms_per_step": wall / steps * 1e3, "kernel_ms": kms,
            "frac": FLOP_PER_QUERY * n / (kms * 1e-3) / 1e12 / PEAK_F16_TFLOPS}


def c4_per_rank_bench(nrc, net, dev, q, frames_q, frames_t, iters: int, t_full_ms: float, step16k_ms: float) -> dict:
    """configs[3] (C4) per-rank work, measured on ONE GPU: what each of the 8 ranks runs.
    Inference: its 2^19-query shard (no collective). Training: one 2,048-sample slice of a 16,384-sample global
    minibatch through nrc_train_dp over a world-1 peer exchange (gradient pass normalised by the global batch -> the
    reduction with the exchange and Adam/EMA fused) and over a world-1 RCCL communicator (gradient pass ->
    ncclAllReduce -> Adam/EMA), plus the gradient pass (nrc_train_grad) and the apply (nrc_train_apply) on their own.
    HIP events on the handle's stream. The 8-GPU prediction divides the 1-GPU work by the per-rank time; the
    all-reduce at 8 ranks is NOT measured here (a world-1 communicator moves no bytes) and is stated as an assumption."""
    import torch

    stream = torch.cuda.current_stream()
    n = QUERIES_C4 // 8
    out = torch.empty((n, 3), dtype=torch.float32, device=dev)
    B, b_local = nrc.BATCH_SIZE, nrc.BATCH_SIZE // 8

    def timed(fn, k: int) -> float:
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(k):
            fn(i)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    infer_ms = timed(lambda i: net.infer(q, out, n), iters)
    state = [net.get_state(s) for s in (nrc.StateSlot.PARAMS, nrc.StateSlot.INFER, nrc.StateSlot.EMA,
                                        nrc.StateSlot.ADAM_M, nrc.StateSlot.ADAM_V)]
    step0 = net.step
    tq, tt = frames_q[0], frames_t[0]
    k = 4 * iters
    # the production data-parallel path: the peer exchange fused into the reduction, at world 1. A rank keeps its own
    # partials in registers, so at world 1 nothing crosses memory: this is the per-rank gradient pass + reduction +
    # Adam of the N-rank step; the wait for the other ranks' words is the prediction's assumed xGMI term below.
    peer_ms = None
    try:
        net.peer_exchange_open(0, 1, net.peer_exchange_handle(1))
        peer_ms = timed(lambda i: net.train_dp(tq[(i % 4) * B:], tt[(i % 4) * B:], b_local, B), k)
    finally:
        net.peer_exchange_close()
    comm = nrc.Communicator(nrc.Communicator.unique_id(), 1, 0)
    net.set_comm(comm)
    dp_ms = timed(lambda i: net.train_dp(tq[(i % 4) * B:], tt[(i % 4) * B:], b_local, B), k)
    dp_graph_ms = graph_ms_per_call(net, stream, lambda i: net.train_dp(tq[(i % 4) * B:], tt[(i % 4) * B:], b_local, B),
                                    16, 10)
    net.set_comm(None)
    comm.destroy()
    grad = torch.zeros(net.grad_floats, dtype=torch.float32, device=dev)
    grad_ms = timed(lambda i: net.train_grad(tq[(i % 4) * B:], tt[(i % 4) * B:], b_local, B, grad), k)
    apply_ms = timed(lambda i: net.train_apply(grad), k)
    local_ms = timed(lambda i: net.train_batch(tq[(i % 4) * B:], tt[(i % 4) * B:], b_local), k)
    local_graph_ms = graph_ms_per_call(net, stream, lambda i: net.train_batch(tq[(i % 4) * B:], tt[(i % 4) * B:], b_local),
                                       16, 10)
    for s, v in zip((nrc.StateSlot.PARAMS, nrc.StateSlot.INFER, nrc.StateSlot.EMA, nrc.StateSlot.ADAM_M,
                     nrc.StateSlot.ADAM_V), state):
        net.set_state(s, v)
    net.step = step0
    allreduce_assumed_us = 25.0
    xgmi_assumed_us = 3.0
    dp_step = peer_ms if peer_ms is not None else dp_ms
    return {"workload": "configs[3] per-rank work on one GPU: 2^19-query inference shard; a 2048-sample slice of a "
                        "16384-sample global minibatch (nrc_train_dp: the peer exchange fused into the reduction at "
                        "world 1; beside it the same step over a world-1 RCCL communicator)",
            "infer_queries": n, "infer_kernel_ms": infer_ms, "infer_M_queries_per_s": n / (infer_ms * 1e-3) / 1e6,
            "train_b_local": b_local, "train_global_b": B,
            "train_dp_step_ms": dp_step, "train_dp_path": "peer exchange (world 1)" if peer_ms is not None else "rccl",
            "train_dp_rccl_step_ms": dp_ms, "train_grad_ms": grad_ms, "train_apply_ms": apply_ms,
            "train_local_fused_step_ms": local_ms,
            "graph_replayed": {"train_dp_rccl_step_ms": dp_graph_ms, "train_local_fused_step_ms": local_graph_ms,
                               "what": "the same calls replayed from a HIP graph: GPU time per step without the "
                                       "per-call host cost (Python, ctypes, one hipLaunchKernel per kernel)"},
            "prediction_8gpu": {
                "infer_speedup": (t_full_ms / infer_ms) if infer_ms > 0 else None,
                "infer_what": "measured 1-GPU kernel time of the whole 2^22-query frame (c4_n1) / per-rank "
                              "2^19-query kernel time (no collective on the inference path)",
                "xgmi_us_assumed": xgmi_assumed_us,
                "train_step_ms_8gpu": dp_step + xgmi_assumed_us * 1e-3,
                "train_speedup": step16k_ms / (dp_step + xgmi_assumed_us * 1e-3),
                "train_what": "1-GPU 16384-sample step / (per-rank world-1 peer-exchange step + an ASSUMED wait for "
                              "the other ranks' words over xGMI; unmeasured on 8 GPUs)",
                "allreduce_us_assumed": allreduce_assumed_us,
                "train_step_ms_8gpu_rccl": grad_ms + apply_ms + allreduce_assumed_us * 1e-3,
                "train_speedup_rccl": step16k_ms / (grad_ms + apply_ms + allreduce_assumed_us * 1e-3),
                "train_what_rccl": "1-GPU 16384-sample step / (per-rank gradient pass + apply + an ASSUMED 88-KiB "
                                   "RCCL all-reduce latency over 8 ranks; unmeasured)"}}


def dp_exchange_bench(nrc, net, dev, world: int, rank: int, frames_q, frames_t, b0: int, bn: int, frames: int,
                      barrier, max_over_ranks) -> dict:
    """N > 1: the same training frames through the library's one-shot peer exchange (nrc_peer_exchange_*: each rank's
    slab reduction stores its partials into every peer's receive buffer over xGMI and sums the world's in rank order
    before Adam) instead of
    the RCCL all-reduce -- per step for configs[3]'s split minibatch (b_local = 16,384 / N) and weak-scaled (16,384 per
    rank, global batch N x 16,384). A setup or exchange failure is recorded, not raised (the inference line stands)."""
    import torch
    import torch.distributed as dist

    B = nrc.BATCH_SIZE
    res = {"exchange": "peer exchange inside the slab reduction (IPC-mapped uncached receive buffers, xGMI stores of "
                       "tagged 8-byte words, rank-order sum + Adam in the same launch; the split form when ranks share "
                       "a device)"}
    ok = torch.ones(1, dtype=torch.int32, device=dev)
    try:
        nrc.dp.open_peer_exchange(net)
    except Exception as e:  # noqa: BLE001
        res["error"] = f"open: {e}"
        ok.zero_()
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not int(ok.item()):
        res.setdefault("error", "open failed on another rank")
        return res

    def run(split: bool) -> float:
        def frame(fi: int) -> None:
            tq, tt = frames_q[fi % 4], frames_t[fi % 4]
            for b in range(4):
                s = b * B
                if split:
                    net.train_dp(tq[s + b0:], tt[s + b0:], bn, B)
                else:
                    net.train_dp(tq[s:], tt[s:], B, B * world)
        frame(0)
        barrier()
        t0 = time.perf_counter()
        for f in range(frames):
            frame(f)
        barrier()
        return max_over_ranks(time.perf_counter() - t0) / frames / 4 * 1e3

    try:
        split_ms = run(True)
        weak_ms = run(False)
        res.update({"split_step_ms": split_ms, "split_samples_per_s": B / (split_ms * 1e-3),
                    "weak_step_ms": weak_ms, "weak_samples_per_s": world * B / (weak_ms * 1e-3),
                    "b_local_split": bn, "b_local_weak": B})
    except Exception as e:  # noqa: BLE001
        res["error"] = f"step: {e}"
    barrier()
    try:
        net.peer_exchange_close()
    except Exception as e:  # noqa: BLE001
        res.setdefault("error", f"close: {e}")
    return res


def open_peer_training(nrc, net, dev, warm_frame) -> bool:
    """N > 1: open the library's one-shot peer exchange on every rank and run one training frame through it
    (``warm_frame``: nrc_train_dp takes the exchange while it is open). True when every rank succeeded (agreed with a
    MIN all-reduce after each stage); otherwise the exchange is closed again, the reason is left in
    ``net._peer_training_error`` and the caller keeps the RCCL communicator."""
    import torch
    import torch.distributed as dist

    ok = torch.ones(1, dtype=torch.int32, device=dev if dist.get_backend() == "nccl" else "cpu")
    err = None
    try:
        nrc.dp.open_peer_exchange(net)
    except Exception as e:  # noqa: BLE001
        err = f"open: {e}"
        ok.zero_()
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()):
        try:
            warm_frame()
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            err = f"step: {e}"
            ok.zero_()
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()):
        return True
    net._peer_training_error = err or "failed on another rank"
    try:
        net.peer_exchange_close()
    except Exception:  # noqa: BLE001
        pass
    return False


PEAK_CLOCK_MHZ = 2400.0  # the clock the 2.5 PF dense f16 peak is quoted at (1,024 SIMDs x 1,024 FLOP per cycle)


def power_sampler(torch, dev):
    """tools/energy_ab.py's amdsmi sampler (read-only gpu_metrics: socket power, gfx clock) on this rank's device, or
    None where amdsmi is unavailable: the power figures are context for the roofline, never required."""
    try:
        sys.path.insert(0, str(ROOT / "tools"))
        from energy_ab import Sampler

        props = torch.cuda.get_device_properties(dev)
        smp = Sampler(f"{props.pci_bus_id:02x}:{props.pci_device_id:02x}", period=0.01)
        smp.start()
        return smp
    except Exception:  # noqa: BLE001
        return None


def power_window(smp, t0: float, t1: float, achieved_tflops: float) -> dict | None:
    """Mean socket power and gfx clock over [t0, t1] (the sustained launches), and the achieved MFMA rate against the
    dense f16 peak at the sampled clock: the package power limit sets the clock."""
    if smp is None:
        return None
    try:
        w = smp.window(t0, t1)
    finally:
        smp.stop()
    res = {"samples": w.get("samples"), "socket_w": w.get("power_w"), "gfx_mhz": w.get("gfx_mhz")}
    if w.get("gfx_mhz"):
        peak = PEAK_F16_TFLOPS * w["gfx_mhz"] / PEAK_CLOCK_MHZ
        res.update({"peak_at_clock_tflops": peak, "frac_at_clock": achieved_tflops / peak})
    return res


def pmc_traffic() -> float | None:
    """HBM bytes per headline launch from the newest committed PMC summary (this round's, else the latest before)."""
    files = sorted(p for p in (ROOT / "profiles").glob("pmc_infer_r*.json") if p.stem.split("_")[-1] <= ROUND)
    for f in reversed(files):
        try:
            return float(json.loads(f.read_text())["hbm_bytes_per_launch"])
        except Exception:
            continue
    return None


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def rank_env(base: dict, world: int, rank: int, port: int) -> dict:
    """The environment of rank `rank` of a self-launched world (the variables torch.distributed.run sets)."""
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_WORLD_SIZE": str(world),
                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "GROUP_RANK": "0"})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (the peer exchange's buffer export)
    return env


def launch_ranks(cmd: list[str], world: int, port: int | None = None, poll_s: float = 0.05,
                 timeout_s: float | None = None) -> int:
    """Run `cmd` as `world` child processes, one per rank, and wait for them. Children inherit stdout / stderr (only
    rank 0 prints the JSON line). The first child to fail takes the others down (a rank blocked in a barrier would
    otherwise wait forever): they are terminated by their own Popen handles, then killed. Returns 0 if every rank
    exited 0, else the first failing rank's exit code (a signal -> 128 + signal number), never 0."""
    port = port or free_port()
    procs = [subprocess.Popen(cmd, env=rank_env(os.environ, world, r, port)) for r in range(world)]
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                return 0
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.terminate()
        for p in live:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return 128 - rc if rc < 0 else rc


def self_launch(args) -> int | None:
    """--gpus N > 1 without a launcher (WORLD_SIZE unset): N fresh children of this script. Called before anything
    touches the GPU; torch.cuda.device_count() does not initialise HIP on this image. None: run in this process."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    if args.dist_backend == "nccl":
        import torch

        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} with the nccl (RCCL) backend needs {args.gpus} visible GPUs, "
                  f"found {have} (one rank per GPU; --dist-backend gloo rehearses ranks sharing a GPU)",
                  file=sys.stderr, flush=True)
            return 2
    return launch_ranks([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], args.gpus)


def main() -> None:
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        raise SystemExit(rc)
    import torch
    import torch.distributed as dist

    nrc = nrc_loader.load()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one rank per GPU; a rehearsal with more ranks than GPUs (gloo) shares them round-robin
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    distributed = world > 1
    if distributed:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    seed = nrc.synthetic.SEED + rank
    c4 = world > 1
    stream = torch.cuda.current_stream()
    # configs[3] for N > 1: this rank's contiguous shard of the 2^22-query frame; configs[1] (2^21) for N = 1
    nq_total = QUERIES_C4 if c4 else args.queries
    q0, nq = nrc.dp.shard_range(nq_total, rank, world) if c4 else (0, nq_total)
    q_np = nrc.synthetic.cornell_queries(nq_total, seed=nrc.synthetic.SEED)[q0:q0 + nq] if c4 else \
        nrc.synthetic.cornell_queries(nq, seed=seed)
    q = torch.from_numpy(np.ascontiguousarray(q_np)).to(dev)
    out = torch.empty((nq, 3), dtype=torch.float32, device=dev)
    frames_q, frames_t = [], []
    for f in range(4):
        # the same global minibatches on every rank (each trains on its slice of them)
        tq, tt = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=nrc.synthetic.SEED * 31 + f)
        frames_q.append(torch.from_numpy(tq).to(dev))
        frames_t.append(torch.from_numpy(tt).to(dev))

    net = nrc.Network()
    net.init(stream=stream, encoding=nrc.InputEncoding.Frequency)
    comm = None
    trainer = None
    b0, bn = nrc.dp.shard_range(nrc.BATCH_SIZE, rank, world)
    if distributed:
        if args.dist_backend == "nccl":
            # RCCL communicator inside the library: rank 0 makes the unique id, torch.distributed carries it
            uid = torch.zeros(nrc.Communicator.UNIQUE_ID_BYTES, dtype=torch.uint8, device=dev)
            if rank == 0:
                uid.copy_(torch.frombuffer(bytearray(nrc.Communicator.unique_id()), dtype=torch.uint8))
            dist.broadcast(uid, src=0)
            comm = nrc.Communicator(bytes(uid.cpu().numpy().tobytes()), world, rank)
            net.set_comm(comm)
        else:
            # rehearsal of several ranks on one GPU (gloo): the Python all-reduce (RCCL cannot share a device)
            trainer = nrc.dp.DataParallelTrainer(net, torch.zeros(nrc.GRAD_FLOATS, dtype=torch.float32, device=dev))
        nrc.dp.DataParallelTrainer(net, None).broadcast_state(net, dev)
    elif args.rehearse_comm:
        comm = nrc.Communicator(nrc.Communicator.unique_id(), 1, 0)
        net.set_comm(comm)

    # the minibatch views of every frame, made once (the reference's renderer passes pointer offsets, which cost
    # nothing; a torch slice per call costs host time that the eager step figure would otherwise include)
    mb_views = [[(frames_q[fi][b * nrc.BATCH_SIZE + b0:], frames_t[fi][b * nrc.BATCH_SIZE + b0:]) for b in range(4)]
                for fi in range(4)]

    peer = {"on": False}  # N > 1: the library's peer exchange is open (nrc_train_dp takes it)

    def train_frame(fi: int) -> None:
        for tqv, ttv in mb_views[fi % 4]:
            if comm is not None or peer["on"]:
                net.train_dp(tqv, ttv, bn, nrc.BATCH_SIZE)
            elif trainer is not None:
                trainer.step(tqv, ttv, bn, nrc.BATCH_SIZE)
            else:
                net.train(tqv, ttv)

    def barrier():
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        if distributed:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # a few frames of self-training first so inference runs on non-trivial (EMA) weights
    for f in range(4):
        train_frame(f)
    # clock settle: the first ~300 back-to-back launches after idle run 94 -> 79 us while the clock ramps (a renderer
    # runs frame after frame, so the settled clock is the operating point); untimed, before the W warmup steps
    settle = {"ms": 0.0, "launches": 0}
    if args.settle_ms > 0:
        es0, es1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        while settle["ms"] < args.settle_ms and settle["launches"] < 20000:
            es0.record(stream)
            for _ in range(50):
                net.infer(q, out, nq)
            es1.record(stream)
            torch.cuda.synchronize()
            settle["ms"] += es0.elapsed_time(es1)
            settle["launches"] += 50
        settle["last_chunk_us_per_launch"] = es0.elapsed_time(es1) / 50 * 1e3
    for _ in range(args.warmup):
        net.infer(q, out, nq)
    barrier()

    # ---- timed inference region: exactly K steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        net.infer(q, out, nq)
    ev1.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one kernel launch per step, same stream
    wall_max = max_over_ranks(wall)
    ms_per_step = wall_max / args.steps * 1e3
    value = nq_total * args.steps / wall_max / 1e6
    # the weights the timed inference used (training below moves them), for the CPU leg's parity check
    infer_params = net.get_state(nrc.StateSlot.INFER) if rank == 0 and world == 1 and not args.no_cpu else None
    out_np = out.cpu().numpy() if infer_params is not None else None

    weak = None
    if c4:
        # weak scaling (the r01 line): 2^21 queries per GPU
        nw = QUERIES_PER_GPU
        qw = torch.from_numpy(nrc.synthetic.cornell_queries(nw, seed=seed)).to(dev)
        ow = torch.empty((nw, 3), dtype=torch.float32, device=dev)
        for _ in range(args.warmup):
            net.infer(qw, ow, nw)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            net.infer(qw, ow, nw)
        barrier()
        ww = max_over_ranks(time.perf_counter() - t0)
        weak = {"queries_per_gpu": nw, "value": world * nw * args.steps / ww / 1e6, "unit": "M queries/s",
                "ms_per_step": ww / args.steps * 1e3, "scaling": "weak"}
        del qw, ow

    # ---- training: frames of 4 x 16384 (N > 1: each minibatch split over the ranks). N > 1 over RCCL: the library's
    # production data-parallel path first -- the one-shot peer exchange inside the reduction (nrc_train_dp takes it
    # while it is open) -- when every rank opened it and ran one frame through it; otherwise, and
    # beside it, the RCCL all-reduce path
    allreduce_path = "rccl" if comm is not None else "python all-reduce (gloo)"
    train_dp_path = "single" if not distributed else allreduce_path
    train_dp_error = None
    if distributed and not args.no_peer:
        # (a gloo rehearsal of several ranks on one GPU takes the same path: the exchange's split form for ranks that
        # share a device, the Python all-reduce as the fallback)
        peer["on"] = True
        if open_peer_training(nrc, net, dev, lambda: train_frame(0)):
            train_dp_path = "peer exchange"
        else:
            peer["on"] = False
            train_dp_error = getattr(net, "_peer_training_error", "failed")

    def time_train_frames() -> float:
        for f in range(2):
            train_frame(f)
        barrier()
        t0 = time.perf_counter()
        for f in range(args.train_frames):
            train_frame(f)
        barrier()
        return max_over_ranks(time.perf_counter() - t0) / args.train_frames * 1e3

    train_frame_ms = time_train_frames()
    train_step_ms = train_frame_ms / 4
    train_step_allreduce_ms = None
    if train_dp_path == "peer exchange":
        net.peer_exchange_close()  # the same frames over the all-reduce path (RCCL), for comparison
        peer["on"] = False
        barrier()
        train_step_allreduce_ms = time_train_frames() / 4
    elif distributed:
        train_step_allreduce_ms = train_step_ms
    train_step_rccl_ms = train_step_allreduce_ms if comm is not None else None
    # the same training frames replayed from a HIP graph (N = 1): the GPU's own step time, without the per-call host
    # cost (Python + ctypes + one hipLaunchKernel per kernel) that the eager figure above includes
    train_step_graph_ms = None
    if world == 1:
        train_step_graph_ms = graph_ms_per_call(net, stream, lambda i: net.train(frames_q[(i // 4) % 4][(i % 4) * nrc.BATCH_SIZE:],
                                                                                frames_t[(i // 4) % 4][(i % 4) * nrc.BATCH_SIZE:]), 16, 10)

    # ---- N > 1: the same training through the one-shot peer exchange (split and weak-scaled), beside RCCL's
    dp_exchange = None
    if distributed and not args.no_peer:
        dp_exchange = dp_exchange_bench(nrc, net, dev, world, rank, frames_q, frames_t, b0, bn, args.train_frames,
                                        barrier, max_over_ranks)
        dp_exchange["rccl_split_step_ms"] = train_step_rccl_ms

    # ---- sustained inference: the clock the chip holds under a long run of back-to-back
    # launches is lower than in a short burst; the average of the last `sustained` of 2 x `sustained` launches
    sustained = None
    if args.sustained > 0:
        sampler = power_sampler(torch, dev)
        for _ in range(args.sustained):
            net.infer(q, out, nq)
        ev2, ev3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev2.record(stream)
        for _ in range(args.sustained):
            net.infer(q, out, nq)
        ev3.record(stream)
        # the sampled window is the timed half: from the moment the GPU reaches ev2 to the end
        while not ev2.query():
            time.sleep(0.0005)
        t_s0 = time.perf_counter()
        torch.cuda.synchronize()
        t_s1 = time.perf_counter()
        s_ms = ev2.elapsed_time(ev3) / args.sustained
        s_tf = FLOP_PER_QUERY * nq / (s_ms * 1e-3) / 1e12
        sustained = {"launches": 2 * args.sustained, "timed": args.sustained, "infer_kernel_ms": s_ms,
                     "achieved": s_tf, "frac": s_tf / PEAK_F16_TFLOPS,
                     "M_queries_per_s": nq / (s_ms * 1e-3) / 1e6,
                     "power": power_window(sampler, t_s0, t_s1, s_tf)}

    # ---- configs[3] at N = 1, measured: the whole 2^22-query 2K frame on this one GPU, timed
    # exactly as the N > 1 line times its shards (K steps, barrier + synchronize on both sides, wall clock), so the
    # 1 -> N strong-scaling ratio is read on one workload; then the per-rank work of 8 GPUs on one GPU
    c4_n1 = None
    c4_per_rank = None
    if world == 1 and not args.no_c4:
        c4_n1 = c4_frame_n1(nrc, net, dev, args.steps, args.warmup, barrier)
        c4_per_rank = c4_per_rank_bench(nrc, net, dev, q, frames_q, frames_t, max(10, args.steps // 4),
                                         c4_n1["kernel_ms"], train_step_ms)

    # ---- one whole post-trace frame: fused infer+accumulate over the 1080p frame's
    # render + train-suffix queries, propagate, shuffle, 4 x train with the minibatch-loss read-back (1 GPU)
    frame = None
    if world == 1 and args.frame_iters > 0:
        frame = frame_bench(nrc, net, dev, args.frame_iters)

    wide = None if args.no_wide else wide_bench(nrc, dev, world, rank, max(10, args.steps // 4), barrier)
    hashgrid = hash_bench(nrc, dev, max(10, args.steps // 10)) if world == 1 and not args.no_hash else None
    tcnn_numerics = tcnn_numerics_bench(nrc, net, q, out, nq, max(10, args.steps // 10)) if world == 1 else None

    achieved = FLOP_PER_QUERY * nq / (kernel_ms * 1e-3) / 1e12
    if c4:
        workload = (f"configs[3]: 2K frame of 2^22 queries sharded over {world} GPUs ({nq_total // world} per GPU), "
                    f"fused encode+64x5 MLP inference (fp16 MFMA, f32 accumulate); train: every 16384-sample minibatch "
                    f"split into {world} x {nrc.BATCH_SIZE // world}, RCCL all-reduce of the gradient inside the library "
                    f"(nrc_train_dp)")
    else:
        workload = ("configs[1]: Cornell 1080p 1spp, 2^21-query fused encode+64x5 MLP inference per GPU "
                    "(fp16 MFMA, f32 accumulate); train: configs[2] 4 x 16384 per frame per GPU")
    result = {
        "metric": "M radiance queries/sec + train-step ms, 64x5 MLP @ 2M samples/frame",
        "value": value,
        "unit": "M queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if c4 else "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic (seeded Cornell-box RadianceQuery stream, SURVEY §8(d)); random-init weights "
                "after 4 frames of self-training",
        "config": {"workload": workload, "queries_total": nq_total, "queries_per_gpu": nq,
                   "train_batch_global": nrc.BATCH_SIZE, "train_batch_per_gpu": bn if distributed else nrc.BATCH_SIZE,
                   "parallelism": f"dp{world}" if world > 1 else "single"},
        "train_step_ms": train_step_ms,
        "train_step_graph_ms": train_step_graph_ms,
        "train_frame_ms": train_frame_ms,
        "train_dp_path": train_dp_path,
        "train_step_allreduce_ms": train_step_allreduce_ms,
        "train_allreduce_path": allreduce_path if distributed else None,
        "train_dp_error": train_dp_error,
        "infer_kernel_ms": kernel_ms,
        "weak": weak,
        "settle": settle,
        "c4_n1": c4_n1,
        "c4_per_rank": c4_per_rank,
        "dp_exchange": dp_exchange,
        "frame": frame,
        "wide_c5": wide,
        "hash": hashgrid,
        "tcnn_numerics": tcnn_numerics,
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_F16_TFLOPS, "traffic": pmc_traffic(),
                     "frac_burst": achieved / PEAK_F16_TFLOPS,
                     "frac_sustained": sustained["frac"] if sustained else None, "sustained": sustained,
                     "algorithmic_bytes_per_launch": BYTES_PER_QUERY * nq,
                     "hbm_gbs_algorithmic": BYTES_PER_QUERY * nq / (kernel_ms * 1e-3) / 1e9},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(q_np, infer_params, args.cpu_seconds,
                                              nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=seed * 31),
                                              gpu_out=out_np)
    if comm is not None:
        net.set_comm(None)
    net.destroy()
    if comm is not None:
        comm.destroy()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
