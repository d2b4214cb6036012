"""Socket power, gfx clock and energy per query of the product inference paths, in-process and interleaved: is each one
at the package power limit (the 64-wide kernel is) or limited by something else?

Paths: the 64-wide Frequency network (2^21 queries, the product launch), the width-128 network in f16 and FP8
(2^23 queries, BASELINE configs[4]), InputEncoding::Hash (2^21 queries: feature pass + MLP pass) and, with --paths
train, the 16,384-sample training step (eager calls; "queries" = samples). Each runs back to
back for --seconds after --settle of the same launches, event-timed per chunk, while tools/energy_ab.py's Sampler reads
the GPU's gpu_metrics through amdsmi (read-only). For the MFMA kernels the MFMA-pipe share of the issue cycles at the
sampled clock follows from their per-tile MFMA cycles (MI355X_MICROARCH.md cycle constants).

    python tools/power_paths.py > gpurun_out/power_paths.json
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
sys.path.insert(0, str(ROOT / "tools"))
import nrc_loader  # noqa: E402
from energy_ab import Sampler  # noqa: E402

# MFMA cycles per 32-query tile on one SIMD (32 cycles per 32x32x16 f16, 64 per block-scaled 32x32x64 f8)
MFMA_CYCLES = {
    # layer 0: 2 M-blocks x 5 k-steps, layers 1-4: 2 x 4 each, output: 8 x 4x4x4 (8 cycles each, an estimate)
    "f64": 32 * (10 + 4 * 8) + 8 * 8,
    # layer 0: 4 x 5, layers 1-4: 4 x 8 each, output: 1 x 8 (f16); FP8 layers 1-4: 4 x 2 each, output 1 x 2 (64 cycles)
    "wide_f16": 32 * (20 + 4 * 32 + 8),
    "wide_fp8": 32 * 20 + 64 * (4 * 8 + 2),
}
SIMDS = 1024


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=1.5)
    ap.add_argument("--settle", type=float, default=0.4)
    ap.add_argument("--paths", default="f64,wide_f16,wide_fp8,hash")
    ap.add_argument("--hash-knob", default=None,
                    help="name=v1,v2,...: one more Hash path per value of a knob (debug library for the ablations)")
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    seed = nrc.synthetic.SEED
    paths = args.paths.split(",")
    runners = {}
    nets = []
    n21, n23 = 1 << 21, 1 << 23
    q21 = torch.from_numpy(nrc.synthetic.cornell_queries(n21, seed=seed)).to(dev)
    o21 = torch.empty((n21, 3), device=dev)
    tq, tt = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=seed * 31)
    tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)

    def trained(net):
        for f in range(4):
            for b in range(4):
                net.train(tq[b * nrc.BATCH_SIZE:], tt[b * nrc.BATCH_SIZE:])
        nets.append(net)
        return net

    if "f64" in paths:
        net = nrc.Network()
        net.init(stream=stream)
        net = trained(net)
        runners["f64"] = (n21, lambda net=net: net.infer(q21, o21, n21))
    if "train" in paths:
        # the 16,384-sample training step (bench.py's minibatches), per step: queries = samples
        net = nrc.Network()
        net.init(stream=stream)
        net = trained(net)
        B = nrc.BATCH_SIZE
        ctr = [0]

        def step(net=net):
            b = ctr[0] % 4
            ctr[0] += 1
            net.train(tq[b * B:], tt[b * B:])
        runners["train"] = (B, step)
    if "hash" in paths:
        net = nrc.Network()
        net.init(stream=stream, encoding=nrc.InputEncoding.Hash)
        net = trained(net)
        runners["hash"] = (n21, lambda net=net: net.infer(q21, o21, n21))
        if args.hash_knob:
            kname, vals = args.hash_knob.split("=")
            for v in vals.split(","):
                runners[f"hash@{kname}={v}"] = (n21, lambda net=net: net.infer(q21, o21, n21), (kname, int(v)))
    if "wide_f16" in paths or "wide_fp8" in paths:
        q23 = torch.from_numpy(nrc.synthetic.cornell_queries(n23, seed=seed + 1000)).to(dev)
        o23 = torch.empty((n23, 3), device=dev)
        net = nrc.Network()
        net.init(stream=stream, encoding=nrc.InputEncoding.Frequency,
                 config=nrc.default_config(nrc.InputEncoding.Frequency, width=128))
        nets.append(net)
        for name, prec in (("wide_f16", nrc.PRECISION_F16), ("wide_fp8", nrc.PRECISION_FP8)):
            if name in paths:
                runners[name] = (n23, lambda net=net, prec=prec: net.infer_precision(prec, q23, o23, n23, stream=stream))
    torch.cuda.synchronize()
    props = torch.cuda.get_device_properties(0)
    smp = Sampler(f"{props.pci_bus_id:02x}:{props.pci_device_id:02x}")
    smp.start()
    time.sleep(0.3)
    idle = smp.window(time.perf_counter() - 0.3, time.perf_counter())
    rounds = {p: [] for p in runners}

    def run_for(fn, seconds, chunk):
        us, launches = [], 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(chunk):
                fn()
            e1.record(stream)
            e1.synchronize()
            us.append(e0.elapsed_time(e1) / chunk * 1e3)
            launches += chunk
        return launches, us, t0, time.perf_counter()

    for _ in range(args.rounds):
        for p, (n, fn, *knob) in runners.items():
            if args.hash_knob:
                kname = args.hash_knob.split("=")[0]
                nrc._lib.set_knob(kname, knob[0][1] if knob else -1)
            chunk = 50 if n == n21 else 200 if n == nrc.BATCH_SIZE else 12
            run_for(fn, args.settle, chunk)
            launches, us, t0, t1 = run_for(fn, args.seconds, chunk)
            w = smp.window(t0, t1)
            rec = {"launches": launches, "us_median": float(np.median(us)), **w}
            if "energy_j" in w:
                rec["nj_per_query"] = w["energy_j"] / (launches * n * w["energy_dt_s"] / (t1 - t0)) * 1e9
            elif "power_w" in w:
                rec["nj_per_query"] = w["power_w"] * float(np.sum(us)) * chunk * 1e-6 / (launches * n) * 1e9
            rounds[p].append(rec)
            print(f"{p}: {rec['us_median']:.1f} us, {rec.get('power_w')} W, {rec.get('gfx_mhz')} MHz", file=sys.stderr,
                  flush=True)
    smp.stop()
    res = {}
    for p, r in rounds.items():
        n = runners[p][0]
        d = {k: float(np.median([x.get(k, np.nan) for x in r])) for k in ("us_median", "power_w", "gfx_mhz", "nj_per_query")}
        if p in MFMA_CYCLES and d["gfx_mhz"] == d["gfx_mhz"]:
            busy = (n / 32) * MFMA_CYCLES[p] / SIMDS / (d["us_median"] * 1e-6) / (d["gfx_mhz"] * 1e6)
            d["mfma_cycles_per_tile"] = MFMA_CYCLES[p]
            d["mfma_pipe_share_at_sampled_clock"] = busy
        d["queries"] = n
        d["rounds"] = r
        res[p] = d
    for net in nets:
        net.destroy()
    print(json.dumps({"idle": idle, "paths": res}, indent=1))


if __name__ == "__main__":
    main()
