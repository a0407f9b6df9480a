"""Debug: dense / CSR / fp32-oracle weight gradients against float64 autograd (test_dense_gpu inputs)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, "."); sys.path.insert(0, "eco-dqn_amd")
from test_dense_gpu import _inputs, _run
from test_dqn_gpu import _flat_to_dict
from oracle import mpnn_oracle as mo
from eco_hip.networks.mpnn import MPNN
from eco_hip._lib import ECO_NORM_PER_GRAPH


def rel(a, b):
    return float((a.double() - b).norm() / max(float(b.norm()), 1e-30))


for n, B in ((20, 64), (64, 19)):
    w, store, x, dq = _inputs(n, B, seed=n + B)
    store.gs.adjbits = None
    net = MPNN(device="cuda"); net.load_state_dict(w)
    qd, qsd, gd = _run(net, store, x, dq, ECO_NORM_PER_GRAPH, dense=True)
    qc, qsc, gc = _run(net, store, x, dq, ECO_NORM_PER_GRAPH, dense=False)
    dd, dc = _flat_to_dict(gd), _flat_to_dict(gc)
    obs = torch.from_numpy(np.stack([np.vstack([x[b, :, :7].cpu().numpy().T.astype(np.float64), store.dense(b)])
                                     for b in range(B)]))
    w32 = {k: v.clone().requires_grad_(True) for k, v in w.items()}
    (mo.forward(w32, obs.float()) * dq.cpu()).sum().backward()
    w64 = {k: v.double().clone().requires_grad_(True) for k, v in w.items()}
    (mo.forward(w64, obs) * dq.cpu().double()).sum().backward()
    for k in mo.KEYS:
        print(n, B, k[:40], "dense %.2e csr %.2e fp32-oracle %.2e" % (rel(dd[k], w64[k].grad), rel(dc[k], w64[k].grad),
                                                                   rel(w32[k].grad, w64[k].grad)))
