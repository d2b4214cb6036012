"""Per-phase cycle shares of the default inference kernel from its diagnostic stamp build (nrc_debug_infer_stamps):
s_memtime around the encoder + prefetch, each of the 5 hidden layers (LDS weight reads, MFMAs, ReLU/f16 packing),
the output layer and the epilogue, summed per wave over its tiles. Shares, not durations, are the result: the
stamps' scheduling fences forbid overlaps the product kernel has (cdna_hip_programming.md §7 In-kernel stamps).

    python tools/infer_stamps.py [--n 2097152] [--iters 20]
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

PHASES = ["encode+prefetch", "L0", "L1", "L2", "L3", "L4", "L5(out)", "epilogue"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 21)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    q = torch.from_numpy(nrc.synthetic.cornell_queries(args.n, seed=2)).to(dev)
    out = torch.empty((args.n, 3), device=dev)
    st = torch.zeros(8 * 8192, dtype=torch.int64, device=dev)
    waves = ctypes.c_uint64()
    for _ in range(args.iters):  # back-to-back launches so the clock settles; the last one is read
        nrc._lib.check(L.nrc_debug_infer_stamps(net._h, q.data_ptr(), out.data_ptr(), args.n, st.data_ptr(),
                                                ctypes.byref(waves)))
    torch.cuda.synchronize()
    w = int(waves.value)
    a = st.cpu().numpy()[: 8 * w].reshape(w, 8).astype(np.float64)
    tiles_per_wave = (args.n + 31) // 32 / w
    tot = a.sum(axis=1)
    share = a / tot[:, None]
    res = {"waves": w, "tiles_per_wave": tiles_per_wave,
           "cycles_per_tile_median": float(np.median(tot) / tiles_per_wave),
           "share_median": {p: round(float(np.median(share[:, i])), 4) for i, p in enumerate(PHASES)},
           "cycles_per_tile_by_phase": {p: round(float(np.median(a[:, i]) / tiles_per_wave), 1)
                                        for i, p in enumerate(PHASES)}}
    net.destroy()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
