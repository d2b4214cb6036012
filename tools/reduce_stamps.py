"""Per-block timeline of reduce_adam_kernel (debug library: s_memrealtime stamps of each block's thread 0 at entry,
slab sums done, after the combine barrier, Adam issued), after a training step of --b samples; 100 MHz ticks -> us
relative to the first block's entry. With --events, also the step's event-timed kernel pair.

    NRC_LIB_PATH=neural-radiance-caching_amd/libnrc_amd_debug.so python tools/reduce_stamps.py [--b 16384]
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    q, t = nrc.synthetic.cornell_batch(nrc.BATCH_SIZE, seed=3)
    q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    pct = lambda a: [round(float(np.percentile(a, p)), 3) for p in (0, 10, 50, 90, 100)]  # noqa: E731
    runs = []
    for rep in range(args.reps + 3):
        for _ in range(8):
            net.train_batch(q, t, args.b)
        torch.cuda.synchronize()
        buf = np.zeros(6 * 8192, np.uint64)
        w = ctypes.c_uint32()
        nrc._lib.check(L.nrc_debug_read_infer_clock(buf.ctypes.data, 8192, ctypes.byref(w)))
        c = buf[: 6 * w.value].reshape(-1, 6).astype(np.float64)
        t0 = c[:, 0].min()
        rel = (c[:, :4] - t0) / 100.0  # us
        if rep < 3:
            continue
        runs.append({"blocks": int(w.value), "entry_us": pct(rel[:, 0]), "sums_done_us": pct(rel[:, 1]),
                     "after_barrier_us": pct(rel[:, 2]), "adam_issued_us": pct(rel[:, 3]),
                     "span_us": round(float(rel[:, 3].max()), 3)})
    net.destroy()
    print(json.dumps({"b": args.b, "runs": runs}, indent=1))


if __name__ == "__main__":
    main()
