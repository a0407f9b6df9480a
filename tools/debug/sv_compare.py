"""Debug: saved activations and gradient-workspace tensors of the dense vs CSR MPNN paths."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eco-dqn_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from test_dense_gpu import _inputs
from eco_hip import _lib
from eco_hip.networks.mpnn import MPNN
n, B = int(sys.argv[1]), int(sys.argv[2])
w, store, x, dq = _inputs(n, B, seed=n + B)
store.gs.adjbits = None
net = MPNN(device="cuda"); net.load_state_dict(w)
gids = torch.arange(B, dtype=torch.int32, device="cuda")
out = {}
for dense in (True, False):
    if dense: os.environ.pop("ECO_MPNN_NO_DENSE", None)
    else: os.environ["ECO_MPNN_NO_DENSE"] = "1"
    saved = torch.zeros(MPNN.saved_bytes(n, B), dtype=torch.uint8, device="cuda")
    net.forward_graphs(x, store, gids, norm_scope=1, saved=saved)
    ws = torch.zeros(_lib.lib.eco_mpnn_backward_workspace_bytes(n, B), dtype=torch.uint8, device="cuda")
    grad = torch.zeros_like(net.flat)
    net.backward_graphs(x, store, gids, saved, dq, grad, workspace=ws)
    torch.cuda.synchronize()
    out[dense] = (saved.view(torch.float32).cpu(), ws.view(torch.float32).cpu())
R = B * n * 64
names_sv = ["H0", "H1", "H2", "H3", "E", "EAGG", "M0", "M1", "M2", "AGG0", "AGG1", "AGG2"]
for i, nm in enumerate(names_sv):
    a, b = out[True][0][i * R:(i + 1) * R].view(B * n, 64), out[False][0][i * R:(i + 1) * R].view(B * n, 64)
    d = (a - b).abs().max(1).values
    print("sv", nm, float(d.max()), "rows>1e-4:", int((d > 1e-4).sum()), "first bad row", int(torch.nonzero(d > 1e-4)[0]) if (d > 1e-4).any() else -1)
names_gr = ["DUU0", "DUU1", "DUU2", "DUM0", "DUM1", "DUM2", "DUE", "DU0", "DZ"]
for i, nm in enumerate(names_gr):
    a, b = out[True][1][i * R:(i + 1) * R].view(B * n, 64), out[False][1][i * R:(i + 1) * R].view(B * n, 64)
    d = (a - b).abs().max(1).values / (1e-6 + b.abs().max())
    print("gr", nm, float(d.max()), "rows>1e-3:", int((d > 1e-3).sum()), "first bad row", int(torch.nonzero(d > 1e-3)[0]) if (d > 1e-3).any() else -1)
i = names_gr.index("DUE")
a, b = out[True][1][i * R:(i + 1) * R].view(B * n, 64), out[False][1][i * R:(i + 1) * R].view(B * n, 64)
print("dense row219", a[219, :8].numpy()); print("csr   row219", b[219, :8].numpy())
dif = (a[219] - b[219]).abs()
print("diff features", torch.nonzero(dif > 1e-5).flatten().tolist())
# does the csr row match any dense row?
m = ((a - b[219]).abs().max(1).values < 1e-6).nonzero().flatten().tolist()
print("csr row 219 equals dense rows", m)
deg = np.diff(store.row_ptr.cpu().numpy()[10])
print("graph 10 degrees", deg.tolist())
