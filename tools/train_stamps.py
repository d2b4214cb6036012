"""Phase timing of the training kernel from the diagnostic s_memtime build (nrc_debug_train_stamps)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402

PHASES32 = ["start", "sample loads", "encode", "weights", "forward", "loss+img5", "L5", "L4", "L3", "L2", "L1", "L0"]
# nrc_train16.hip, per wave: encode (sample loads, forward-image DMA issue, encoder), weights (DMA wait + barrier),
# forward layers, loss (backward-image LDS stores, loss, layer-5 images, barrier), backward steps
PHASES16 = ["start", "encode", "weights", "fwd0", "fwd1", "fwd2", "fwd3", "fwd4", "fwd5", "loss+img5", "L5", "L4", "L3",
            "L2", "L1", "L0"]


def main():
    import os
    import torch

    k32 = os.environ.get("NRC_TRAIN_KERNEL") == "32"
    PHASES = PHASES32 if k32 else PHASES16
    W = 1 if k32 else 4  # stamped waves per block

    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=0, help="samples per launch (default: BATCH_SIZE)")
    args = ap.parse_args()
    nrc = nrc_loader.load()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    B = args.b or nrc.BATCH_SIZE
    q_np, t_np = nrc.synthetic.cornell_batch(B, seed=3)
    q, t = torch.from_numpy(q_np).to(dev), torch.from_numpy(t_np).to(dev)
    nb = (B + 127) // 128
    st = torch.zeros(nb * W * 16, dtype=torch.int64, device=dev)
    res = []
    for it in range(5):
        # steady state: the stamped launch follows a regular step, whose optimizer kernel just wrote the images
        net.train_batch(q, t, B)
        nrc._lib.check(L.nrc_debug_train_stamps(net._h, q.data_ptr(), t.data_ptr(), B, st.data_ptr()))
        torch.cuda.synchronize()
        a = st.cpu().numpy().reshape(nb, W, 16)[:, :, :len(PHASES)].astype(np.int64)
        if it == 0:
            continue
        a = a - a[:, :, :1].min(axis=1, keepdims=True)  # per block, from its first wave's start (s_memtime is per XCD)
        d = np.diff(a, axis=2)
        crit = np.diff(np.concatenate([np.zeros((nb, 1)), a.max(axis=1)[:, 1:]], axis=1), axis=1)
        res.append({"block_end_median": float(np.median(a[:, :, -1].max(axis=1))),
                    "phase_median_per_wave": {PHASES[i]: float(np.median(d[:, :, i - 1])) for i in range(1, len(PHASES))},
                    # phase end of the block's last wave minus the previous phase end of its last wave
                    "phase_median_last_wave": {PHASES[i]: float(np.median(crit[:, i - 1])) for i in range(1, len(PHASES))},
                    "wave_end_spread_median": {PHASES[i]: float(np.median(a[:, :, i].max(axis=1) - a[:, :, i].min(axis=1)))
                                               for i in range(1, len(PHASES))}})
    net.destroy()
    print(json.dumps(res[-1], indent=1))


if __name__ == "__main__":
    main()
