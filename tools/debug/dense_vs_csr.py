"""Debug: per-parameter gradient error of the dense and CSR backward vs torch autograd (oracle)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eco-dqn_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from oracle import mpnn_oracle as mo
from test_dense_gpu import _inputs, _run
from test_dqn_gpu import _flat_to_dict
from eco_hip.networks.mpnn import MPNN
n, B = int(sys.argv[1]), int(sys.argv[2])
w, store, x, dq = _inputs(n, B, seed=n + B)
store.gs.adjbits = None
net = MPNN(device="cuda"); net.load_state_dict(w)
_, qd, gd = _run(net, store, x, dq, 1, True)
_, qc, gc = _run(net, store, x, dq, 1, False)
obs = torch.from_numpy(np.stack([np.vstack([x[b, :, :7].cpu().numpy().T.astype(np.float64), store.dense(b)]) for b in range(B)])).float()
wg = {k: v.clone().requires_grad_(True) for k, v in w.items()}
qr = mo.forward(wg, obs); (qr * dq.cpu()).sum().backward()
dd, dc = _flat_to_dict(gd), _flat_to_dict(gc)
print("q err dense", float((qd - qr.detach()).abs().max()), "csr", float((qc - qr.detach()).abs().max()))
for k in mo.KEYS:
    r = wg[k].grad
    ed = float((dd[k] - r).norm() / r.norm()); ec = float((dc[k] - r).norm() / r.norm())
    print(f"{k:55s} dense {ed:.2e} csr {ec:.2e}")
    if k.startswith("edge_embedding_layer.edge_embedding_NN"):
        print("  col0 (w_a) dense", float((dd[k][:, 0] - r[:, 0]).norm() / r[:, 0].norm()), "csr", float((dc[k][:, 0] - r[:, 0]).norm() / r[:, 0].norm()))
        print("  cols1: dense", float((dd[k][:, 1:] - r[:, 1:]).norm() / r[:, 1:].norm()), "csr", float((dc[k][:, 1:] - r[:, 1:]).norm() / r[:, 1:].norm()))
