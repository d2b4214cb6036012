"""Energy per query of inference kernel variants, in-process and interleaved.

The headline kernel runs at the package power limit, so throughput there is set by energy
per query, and a variant is better only if it needs fewer joules per query. For each variant, in interleaved rounds:
back-to-back launches of n queries for --seconds (after a --settle of the same launches), event-timed per chunk, while a
sampler thread reads the GPU's own counters through amdsmi (read-only queries): the energy accumulator of
gpu_metrics when the device exposes it (J = delta x its 15.259 uJ unit), else socket power x time; plus the socket power
and the gfx clock. J/query = energy over the timed window / queries processed in it.

    NRC_LIB_PATH=neural-radiance-caching_amd/libnrc_amd_debug.so python tools/energy_ab.py --variants 47,52,53

Output: one JSON document on stdout (per variant: median us per launch, W, GHz, nJ/query, per round).
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402

ENERGY_UNIT_J = 15.259e-6  # gpu_metrics energy_accumulator unit (amdsmi documentation: 15.259 uJ per count)


class Sampler:
    """amdsmi readings of one device every `period` s: (t, energy counter or None, socket W, gfx MHz)."""

    def __init__(self, bdf: str | None, period: float = 0.02):
        import amdsmi

        self.amdsmi = amdsmi
        amdsmi.amdsmi_init()
        handles = amdsmi.amdsmi_get_processor_handles()
        self.h = handles[0]
        if bdf:
            for h in handles:
                try:
                    if amdsmi.amdsmi_get_gpu_device_bdf(h).lower().endswith(bdf.lower()):
                        self.h = h
                        break
                except Exception:
                    pass
        self.period = period
        self.samples: list[tuple[float, float | None, float | None, float | None]] = []
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True)

    def read(self):
        a = self.amdsmi
        e = w = mhz = None
        try:
            m = a.amdsmi_get_gpu_metrics_info(self.h)
            ea = m.get("energy_accumulator")
            e = float(ea) if isinstance(ea, (int, float)) else None
            for k in ("current_socket_power", "average_socket_power"):
                if isinstance(m.get(k), (int, float)) and m[k] not in (0xFFFF,):
                    w = float(m[k])
                    break
            for k in ("current_gfxclk", "average_gfxclk_frequency"):
                v = m.get(k)
                if isinstance(v, (list, tuple)):
                    v = [x for x in v if isinstance(x, (int, float)) and x not in (0xFFFF,)]
                    v = float(np.mean(v)) if v else None
                if isinstance(v, (int, float)):
                    mhz = float(v)
                    break
        except Exception:
            pass
        if w is None:
            try:
                p = a.amdsmi_get_power_info(self.h)
                for k in ("current_socket_power", "average_socket_power", "socket_power"):
                    if isinstance(p.get(k), (int, float)):
                        w = float(p[k])
                        break
            except Exception:
                pass
        return e, w, mhz

    def _run(self):
        while not self._stop.is_set():
            t = time.perf_counter()
            self.samples.append((t, *self.read()))
            time.sleep(self.period)

    def start(self):
        self._th.start()

    def stop(self):
        self._stop.set()
        self._th.join()
        try:
            self.amdsmi.amdsmi_shut_down()
        except Exception:
            pass

    def window(self, t0: float, t1: float) -> dict:
        s = [x for x in self.samples if t0 <= x[0] <= t1]
        out = {"samples": len(s)}
        es = [(x[0], x[1]) for x in s if x[1] is not None]
        if len(es) >= 2 and es[-1][1] > es[0][1]:
            out["energy_j"] = (es[-1][1] - es[0][1]) * ENERGY_UNIT_J
            out["energy_dt_s"] = es[-1][0] - es[0][0]
        ws = [x[2] for x in s if x[2] is not None]
        if ws:
            out["power_w"] = float(np.mean(ws))
        cs = [x[3] for x in s if x[3] is not None]
        if cs:
            out["gfx_mhz"] = float(np.mean(cs))
        return out


def bench_weights(nrc, net, torch, dev, n):
    """bench.py's state: init + 4 frames of self-training on its synthetic batches, and its query stream."""
    seed = nrc.synthetic.SEED
    q_np = nrc.synthetic.cornell_queries(n, seed=seed)
    for f in range(4):
        tq, tt = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE * 4, seed=seed * 31 + f)
        tq, tt = torch.from_numpy(tq).to(dev), torch.from_numpy(tt).to(dev)
        for b in range(4):
            net.train(tq[b * nrc.BATCH_SIZE:], tt[b * nrc.BATCH_SIZE:])
    torch.cuda.synchronize()
    return q_np


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 21)
    ap.add_argument("--variants", default="47,52,53")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=1.5)
    ap.add_argument("--settle", type=float, default=0.4)
    ap.add_argument("--chunk", type=int, default=50)
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
    q_np = bench_weights(nrc, net, torch, dev, args.n)
    params = net.get_state(nrc.StateSlot.INFER)
    q = torch.from_numpy(q_np).to(dev)
    out = torch.empty((args.n, 3), device=dev)
    idx = np.arange(0, args.n, 4099)
    y_ref = orc.forward(params, q_np[idx], orc.MIXED)
    check = {}
    for v in variants:
        nrc._lib.check(L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), out.data_ptr(), args.n, sp))
        torch.cuda.synchronize()
        y = out.cpu().numpy()[idx]
        check[v] = float(np.linalg.norm(y - y_ref) / np.linalg.norm(y_ref))
    props = torch.cuda.get_device_properties(0)
    bdf = f"{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
    smp = Sampler(bdf)
    smp.start()
    time.sleep(0.3)
    idle = smp.window(time.perf_counter() - 0.3, time.perf_counter())
    rounds = {v: [] for v in variants}

    def run_for(v, seconds):
        """back-to-back chunks of launches for `seconds`; returns (launches, per-launch us list, t0, t1)"""
        us, launches = [], 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.chunk):
                L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), out.data_ptr(), args.n, sp)
            e1.record(stream)
            e1.synchronize()
            us.append(e0.elapsed_time(e1) / args.chunk * 1e3)
            launches += args.chunk
        return launches, us, t0, time.perf_counter()

    for _ in range(args.rounds):
        for v in variants:
            run_for(v, args.settle)
            launches, us, t0, t1 = run_for(v, args.seconds)
            w = smp.window(t0, t1)
            rec = {"launches": launches, "us_median": float(np.median(us)), "wall_s": t1 - t0, **w}
            queries = launches * args.n
            if "energy_j" in w:
                # energy over the sampled sub-window, scaled to the launches inside it by time
                rec["nj_per_query"] = w["energy_j"] / (queries * w["energy_dt_s"] / (t1 - t0)) * 1e9
            elif "power_w" in w:
                rec["nj_per_query"] = w["power_w"] * float(np.sum(us)) * args.chunk * 1e-6 / queries * 1e9
            rounds[v].append(rec)
    smp.stop()
    res = {}
    for v in variants:
        r = rounds[v]
        res[v] = {"us_median": float(np.median([x["us_median"] for x in r])),
                  "power_w": float(np.median([x.get("power_w", np.nan) for x in r])),
                  "gfx_mhz": float(np.median([x.get("gfx_mhz", np.nan) for x in r])),
                  "nj_per_query": float(np.median([x.get("nj_per_query", np.nan) for x in r])),
                  "rel_l2_vs_oracle": check[v], "rounds": r}
    net.destroy()
    print(json.dumps({"n": args.n, "idle": idle, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
