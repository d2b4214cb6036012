"""Debug check of the 16x16x32 inference kernel (variants 50 / 51) against the oracle."""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402
import torch

nrc = nrc_loader.load(); orc = nrc_loader.load_oracle(); L = nrc._lib.lib()
dev = torch.device("cuda:0"); st = torch.cuda.current_stream(); sp = int(st.cuda_stream)
import os
os.environ.setdefault("NRC_DEBUG_INFER16", "1")
n = 4096
q_np = nrc.synthetic.cornell_queries(n, seed=2)
q = torch.from_numpy(q_np).to(dev)
net = nrc.Network(); net.init(stream=st)
p = orc.init_params(1337)
net.set_state(nrc.StateSlot.PARAMS, p)
net.set_state(nrc.StateSlot.INFER, p * np.float32(1.6))
ref_p = orc.forward(p, q_np, orc.MIXED); ref_i = orc.forward(p * np.float32(1.6), q_np, orc.MIXED)
for v in (39, 50, 51):
    out = torch.zeros((n, 3), device=dev)
    nrc._lib.check(L.nrc_debug_infer_variant(net._h, v, q.data_ptr(), out.data_ptr(), n, sp))
    torch.cuda.synchronize()
    y = out.cpu().numpy()
    for name, r in (("params", ref_p), ("infer", ref_i)):
        print(v, name, float(np.linalg.norm(y - r) / np.linalg.norm(r)))
    print(v, y[:3].tolist(), y[16:18].tolist())
print("ref", ref_i[:3].tolist(), ref_i[16:18].tolist())
