"""Every bit of the MPNN kernel-path policy (eco_set_kernel_paths, include/eco_hip.h) routes a call to
another product kernel family; each routed call must give the default path's results within the fp32
bars of the other MPNN tests (the same forward of mpnn.py:40-159 in a different summation order):
  Q: |q - q_default| <= 5e-7 (1 + |q_default|) (measured <= 6.2e-8);  gradients: relative L2 difference < 5e-6 per tensor.
NO_DENSE is covered against the dense kernels in test_dense_gpu.py; here NO_DL (BA one-graph blocks of
224 < N <= 512 on the CSR-gather kernels), NO_SHARED (one shared graph of N > 512 on the per-episode
global-memory kernel) and NO_PAIR / NO_DENSE on the double-DQN pair (two eco_mpnn_forward calls, bitwise
equal to the one-launch pair)."""
import numpy as np
import pytest
import torch

from oracle import graphs as og
from oracle import mpnn_oracle as mo

pytestmark = pytest.mark.gpu


def _net(seed):
    from eco_hip.networks.mpnn import MPNN
    w = mo.init_weights(torch.Generator().manual_seed(seed), std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    return net


def _x(B, n, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    return x.cuda(), torch.randn(B, n, generator=g).cuda()


def _scaled(a, b):
    e = float(((a - b).abs() / (1 + b.abs())).max())
    print(f"scaled err {e:.3e}")
    return e


def _rel(a, b):
    e = float((a - b).norm() / b.norm().clamp_min(1e-30))
    print(f"rel L2 {e:.3e}")
    return e


def test_no_dl_matches_dense_large_kernels():
    """BA(300, 4) +-1: one graph of 224 < N <= 512 per workgroup (eco_mpnn_dl.h) by default, the CSR-gather
    kernels under ECO_PATH_NO_DL; inference forward, training forward and backward (weight gradients)."""
    from eco_hip import _lib
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    n, B = 300, 12
    store = GraphStore.random("BA", B, n, 4, seed=300)
    net = _net(3)
    x, dq = _x(B, n, 4)
    gids = torch.arange(B, dtype=torch.int32, device="cuda")
    out = {}
    for mask in (0, _lib.ECO_PATH_NO_DL):
        with _lib.kernel_paths(mask):
            q = net.forward_graphs(x, store, gids, norm_scope=_lib.ECO_NORM_PER_GRAPH).clone()
            saved = torch.empty(MPNN.saved_bytes(n, B), dtype=torch.uint8, device="cuda")
            qs = net.forward_graphs(x, store, gids, norm_scope=_lib.ECO_NORM_PER_CALL, saved=saved).clone()
            grad = torch.zeros_like(net.flat)
            net.backward_graphs(x, store, gids, saved, dq, grad)
            torch.cuda.synchronize()
            out[mask] = (q, qs, grad.clone())
    (q0, qs0, g0), (q1, qs1, g1) = out[0], out[_lib.ECO_PATH_NO_DL]
    assert _scaled(q1, q0) <= 5e-7
    assert _scaled(qs1, qs0) <= 5e-7
    from eco_hip.networks.mpnn import param_layout
    off = 0
    for name, shape in param_layout():
        k = int(np.prod(shape))
        assert _rel(g1[off:off + k], g0[off:off + k]) < 5e-6, name
        off += k


def test_no_shared_matches_shared_graph_kernels():
    """One ER(600, 0.02) +-1 graph shared by 20 episodes: the shared-graph kernels (eco_mpnn_shared.h) by
    default, the per-episode global-memory kernel under ECO_PATH_NO_SHARED; Q and fused greedy actions."""
    from eco_hip import _lib
    from eco_hip.graphs import GraphStore
    n, B = 600, 20
    J = og.er_graph(n, 0.02, np.random.default_rng(601), weights="discrete")
    one = GraphStore.from_dense([J])
    net = _net(6)
    x, _ = _x(B, n, 7)
    gz = torch.zeros(B, dtype=torch.int32, device="cuda")
    res = {}
    for mask in (0, _lib.ECO_PATH_NO_SHARED):
        with _lib.kernel_paths(mask):
            q = torch.empty(B, n, device="cuda")
            a = torch.empty(B, dtype=torch.int32, device="cuda")
            net.forward_graphs(x, one, gz, norm_scope=_lib.ECO_NORM_PER_CALL, q_out=q,
                               act=_lib.ActConfig(0.0, 1, 0.0, 1, 0), actions_out=a)
            torch.cuda.synchronize()
            res[mask] = (q, a)
    (q0, a0), (q1, a1) = res[0], res[_lib.ECO_PATH_NO_SHARED]
    assert _scaled(q1, q0) <= 5e-7
    assert torch.equal(a0.long(), q0.argmax(1)) and torch.equal(a1.long(), q1.argmax(1))


@pytest.mark.parametrize("bit", ["NO_PAIR", "NO_DENSE"])
def test_pair_paths(bit):
    """eco_mpnn_forward_pair on ER-200 one-graph blocks: one launch by default; two eco_mpnn_forward calls
    under NO_PAIR (bitwise equal), or two CSR-kernel forwards under NO_DENSE (within the fp32 bar)."""
    from eco_hip import _lib
    from eco_hip.graphs import GraphStore
    n, B = 200, 64
    store = GraphStore.random("ER", B, n, 0.15, seed=200)
    net, tgt = _net(8), _net(9)
    x, _ = _x(B, n, 10)
    gids = torch.arange(B, dtype=torch.int32, device="cuda")
    greedy = _lib.ActConfig(0.0, 1, 0.0, 0, 0)
    res = {}
    mask = getattr(_lib, "ECO_PATH_" + bit)
    for m in (0, mask):
        with _lib.kernel_paths(m):
            a = torch.empty(B, dtype=torch.int32, device="cuda")
            qb = torch.empty(B, n, device="cuda")
            net.forward_pair_graphs(tgt, x, store, gids, norm_scope=_lib.ECO_NORM_PER_CALL, act=greedy,
                                    actions_out=a, q_out_other=qb)
            torch.cuda.synchronize()
            res[m] = (a.clone(), qb.clone())
    (a0, q0), (a1, q1) = res[0], res[mask]
    if bit == "NO_PAIR":
        assert torch.equal(a0, a1) and torch.equal(q0, q1)
    else:
        assert _scaled(q1, q0) <= 5e-7
        qa = net.forward_graphs(x, store, gids, norm_scope=_lib.ECO_NORM_PER_CALL)
        assert torch.equal(a0.long(), qa.argmax(1))

