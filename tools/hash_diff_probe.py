import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import nrc_loader
nrc = nrc_loader.load(); orc = nrc_loader.load_oracle()
dev = torch.device("cuda:0"); st = torch.cuda.current_stream()
n = 1 << 21
qn = nrc.synthetic.cornell_queries(n, seed=9)
q = torch.from_numpy(qn).to(dev)
net = nrc.Network(); net.init(stream=st, encoding=nrc.InputEncoding.Hash)
outs = {}
for k, env in (("queue", None), ("queue2", None), ("round1", "512"), ("round1b", "512")):
    if env: os.environ["NRC_EXT_INFER_SHAPE"] = env
    else: os.environ.pop("NRC_EXT_INFER_SHAPE", None)
    o = torch.zeros((n, 3), device=dev); net.infer(q, o, n); torch.cuda.synchronize(); outs[k] = o.cpu().numpy()
for a, b in (("queue", "queue2"), ("round1", "round1b"), ("queue", "round1")):
    d = np.abs(outs[a] - outs[b]).max(axis=1)
    idx = np.nonzero(d)[0]
    print(a, b, "rows differ:", idx.size, "max", float(d.max()) if idx.size else 0, "first", idx[:10].tolist())
params = net.get_state(nrc.StateSlot.INFER)
idx = np.nonzero(np.abs(outs["queue"] - outs["round1"]).max(axis=1))[0][:64]
if idx.size:
    ref = orc.hash_forward(params, qn[idx]) if hasattr(orc, "hash_forward") else None
    print("queue", outs["queue"][idx[:4]].tolist()); print("round1", outs["round1"][idx[:4]].tolist())
    if ref is not None: print("oracle", ref[:4].tolist())
    print("tile ids", sorted(set((idx // 32).tolist()))[:20])
net.destroy()
