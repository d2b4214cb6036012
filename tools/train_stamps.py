"""Phase timing of the training kernel from the diagnostic s_memtime build (nrc_debug_train_stamps)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402

PHASES = ["start", "sample loads", "encode", "weights", "forward", "loss+img5", "L5", "L4", "L3", "L2", "L1", "L0"]


def main():
    import torch

    nrc = nrc_loader.load()
    L = nrc._lib.lib()
    dev = torch.device("cuda:0")
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    B = nrc.BATCH_SIZE
    q_np, t_np = nrc.synthetic.cornell_batch(B, seed=3)
    q, t = torch.from_numpy(q_np).to(dev), torch.from_numpy(t_np).to(dev)
    nb = (B + 127) // 128
    st = torch.zeros(nb * 16, dtype=torch.int64, device=dev)
    res = []
    for it in range(5):
        # steady state: the stamped launch follows a regular step, whose optimizer kernel just wrote the images
        net.train(q, t)
        nrc._lib.check(L.nrc_debug_train_stamps(net._h, q.data_ptr(), t.data_ptr(), B, st.data_ptr()))
        torch.cuda.synchronize()
        a = st.cpu().numpy().reshape(nb, 16)[:, :len(PHASES)].astype(np.int64)
        if it == 0:
            continue
        rel = a - a[:, :1].min()
        res.append({"block_start_spread": int(a[:, 0].max() - a[:, 0].min()),
                    "end_max": int(rel[:, -1].max()),
                    "phase_median": {PHASES[i]: float(np.median(a[:, i] - a[:, i - 1])) for i in range(1, len(PHASES))}})
    net.destroy()
    print(json.dumps(res[-1], indent=1))


if __name__ == "__main__":
    main()
