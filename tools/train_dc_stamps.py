"""Per-phase in-kernel clock of the decoupled-chain training kernel (diagnostic build via nrc_debug_train_stamps; run
with NRC_LIB_PATH=neural-radiance-caching_amd/libnrc_amd_debug.so, the stamped builds live in the debug library).

Chain wave (wave 0 of each block), s_memtime cycles between stamps: 0->1 sample loads + encode, 1->2 layer 0,
2->3 .. 6->7 layers 1..5 (with the next layers' fragment loads), 7->8 loss + delta_5, 8->9 backward step 5,
9->10 .. 12->13 steps 4..1. dW wave (first dW wave): wait for step L and compute/publish/store it, L = 5..0.
s_memrealtime (100 MHz) at every wave's start and end gives the launch spread and the kernel span.

    python tools/train_dc_stamps.py  ->  gpurun_out/train_dc_stamps.json
"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nrc_loader  # noqa: E402

WAVES = {0: (2, 1), 1: (2, 1), 2: (4, 2), 3: (8, 4), 4: (8, 4), 5: (4, 2), 6: (3, 1), 7: (6, 2)}  # (waves, chain)
SPB = {0: 16, 1: 32, 2: 64, 3: 128, 4: 64, 5: 32, 6: 16, 7: 32}


def main():
    nrc = nrc_loader.load()
    L = nrc._lib
    lib = L.lib()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    B = nrc.BATCH_SIZE
    q, t = nrc.synthetic.cornell_batch(B, seed=3)
    q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    net = nrc.Network()
    net.init(stream=st)
    for i in range(4):
        net.train(q, t)
    out = {}
    for shape in (0, 6, 7, 3, 4):
        for b in (2048, 16384):
            L.set_knob("train_shape", shape)
            nw, cw = WAVES[shape]
            blocks = (b + SPB[shape] - 1) // SPB[shape]
            stamps = torch.zeros(blocks * nw * 16, dtype=torch.int64, device=dev)
            for rep in range(3):  # warm caches / clocks, keep the last
                L.check(lib.nrc_debug_train_stamps(net._h, q.data_ptr(), t.data_ptr(), b, stamps.data_ptr()))
                torch.cuda.synchronize()
            s = stamps.cpu().numpy().reshape(blocks, nw, 16).astype(np.int64)
            chain = np.diff(s[:, 0, :14], axis=1)
            dw = s[:, cw, :13]
            dwd = np.diff(dw, axis=1)
            rs, re = s[:, :, 14].min(axis=1), s[:, :, 15].max(axis=1)
            key = f"shape{shape}_b{b}"
            out[key] = {
                "blocks": blocks,
                "chain_phase_cycles_median": np.median(chain, axis=0).tolist(),
                "chain_total_cycles_median": float(np.median(s[:, 0, 13] - s[:, 0, 0])),
                "chain_total_cycles_max": float(np.max(s[:, 0, 13] - s[:, 0, 0])),
                "dw_phase_cycles_median": np.median(dwd, axis=0).tolist(),
                "dw_total_cycles_median": float(np.median(dw[:, 12] - dw[:, 0])),
                "block_start_spread_us": float((rs.max() - rs.min()) / 100.0),
                "kernel_span_us": float((re.max() - rs.min()) / 100.0),
                "block_span_us_median": float(np.median(re - rs) / 100.0),
                "clock_ghz": float(np.median((s[:, 0, 13] - s[:, 0, 0]) / np.maximum(1, (s[:, 0, 15] - s[:, 0, 14])) * 0.1)),
            }
            print(key, json.dumps({k: (np.round(v, 1).tolist() if isinstance(v, list) else v) for k, v in out[key].items()}),
                  flush=True)
    L.set_knob("train_shape", -1)
    net.destroy()
    p = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "gpurun_out", "train_dc_stamps.json")
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
