"""In-process A/B timing of the inference kernel variants (interleaved rounds, one process, one device;
cdna_hip_programming.md §5.4 rule 24). Also checks every variant against the oracle on a sample.

    NRC_LIB_PATH=neural-radiance-caching_amd/libnrc_amd_debug.so python tools/ab_infer.py [--variants 23,30,39]

The A/B variants other than the product's 39 live in the debug library (libnrc_amd_debug.so).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402

# variants that record the in-kernel clock (nrc_debug_read_infer_clock): 40 = 39 clocked, 42 = 41 (pooled) clocked.
# 50: the rejected 16x16x32 inference kernel (nrc_infer16.hip)
CLOCKED = {40, 42, 46, 48}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 21)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="23,30,39")
    ap.add_argument("--weights", default="scaled", choices=["scaled", "bench"],
                    help="scaled: 1.6 x the init weights; bench: bench.py's state (xavier init + 4 frames of "
                         "self-training on its synthetic batches) and its query stream")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    orc = nrc_loader.load_oracle()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = int(stream.cuda_stream)
    variants = [int(v) for v in args.variants.split(",")]

    net = nrc.Network()
    net.init(stream=stream)
    if args.weights == "bench":
        seed = nrc.synthetic.SEED
        q_np = nrc.synthetic.cornell_queries(args.n, seed=seed)
        for f in range(4):
            tq, tt = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=seed * 31 + f)
            tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
            for b in range(4):
                net.train(tq[b * nrc.BATCH_SIZE:], tt[b * nrc.BATCH_SIZE:])
        torch.cuda.synchronize()
        params = net.get_state(nrc.StateSlot.INFER)
    else:
        q_np = nrc.synthetic.cornell_queries(args.n, seed=2)
        params = orc.init_params(1337) * np.float32(1.6)
        net.set_state(nrc.StateSlot.INFER, params)
    q = torch.from_numpy(q_np).to(dev)
    outs = {v: torch.empty((args.n, 3), device=dev) for v in variants}
    idx = np.arange(0, args.n, 4099)
    y_ref = orc.forward(params, q_np[idx], orc.MIXED)
    check = {}
    for v in variants:
        nrc._lib.check(L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), outs[v].data_ptr(), args.n, sp))
        torch.cuda.synchronize()
        y = outs[v].cpu().numpy()[idx]
        check[v] = float(np.linalg.norm(y - y_ref) / np.linalg.norm(y_ref))
    times = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), outs[v].data_ptr(), args.n, sp)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters * 1e3)
    res = {}
    for v in variants:
        t = np.array(times[v])
        med = float(np.median(t))
        res[v] = {"median_us": med, "min_us": float(t.min()), "Gq_per_s": args.n / med / 1e3,
                  "tflops_alg": 41600 * args.n / (med * 1e-6) / 1e12, "rel_l2_vs_oracle": check[v]}
        if v in CLOCKED:
            # in-kernel clock of the variant's last launch (per wave: s_memtime cycles, 100 MHz s_memrealtime ticks)
            for _ in range(args.iters):
                L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), outs[v].data_ptr(), args.n, sp)
            torch.cuda.synchronize()
            buf = np.zeros(6 * 8192, np.uint64)
            w = ctypes.c_uint32()
            nrc._lib.check(L.nrc_debug_read_infer_clock(buf.ctypes.data, 8192, ctypes.byref(w)))
            c = buf[: 6 * w.value].reshape(-1, 6).astype(np.float64)
            ghz = c[:, 0] / ((c[:, 2] - c[:, 1]) * 10.0)
            tiles_per_wave = (args.n / 32) / w.value
            t0 = c[:, 3].min()
            start, lstart, end = (c[:, 3] - t0) / 100.0, (c[:, 1] - t0) / 100.0, (c[:, 2] - t0) / 100.0  # us
            pct = lambda a: [float(np.percentile(a, p)) for p in (0, 10, 50, 90, 100)]  # noqa: E731
            res[v].update({"clock_ghz_median": float(np.median(ghz)), "waves": int(w.value),
                           "cycles_per_tile_median": float(np.median(c[:, 0]) / tiles_per_wave),
                           "loop_us_median": float(np.median(end - lstart)),
                           "wave_start_us_p0_10_50_90_100": pct(start), "loop_start_us_p": pct(lstart),
                           "loop_end_us_p": pct(end)})
            # per XCD and per CU: when their waves finish (the kernel ends with the slowest CU)
            xcc = c[:, 5].astype(int) & 15
            cu = (c[:, 4].astype(np.int64) >> 8) & 15
            se = (c[:, 4].astype(np.int64) >> 13) & 7
            res[v]["end_us_by_xcd_mean_max"] = {int(x): [float(end[xcc == x].mean()), float(end[xcc == x].max())]
                                                for x in sorted(set(xcc.tolist()))}
            keys = xcc * 256 + se * 16 + cu
            per_cu = np.array([end[keys == k].max() for k in sorted(set(keys.tolist()))])
            res[v]["cu_last_end_us_p0_10_50_90_100"] = pct(per_cu)
            res[v]["cus_seen"] = int(len(per_cu))
    net.destroy()
    print(json.dumps({"n": args.n, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
