"""The dense-aggregation MPNN kernels (eco_mpnn_dense.h: blocks of <= 224 rows, +-1 weights) against
the CSR-gather kernels (eco_mpnn.hip) on the same inputs, and against the fp32 torch oracle.

The CSR path is selected per call with the ECO_PATH_NO_DENSE kernel-path bit (eco_set_kernel_paths).  Both compute the reference's fp32
arithmetic in a different summation order (dense: exact bf16x3 splits, fp32 accumulation), so the bars
are the oracle tolerances of test_mpnn_gpu / test_dqn_gpu:
  Q: |q - q_ref| <= 5e-7 (1 + |q_ref|) (measured <= 6.3e-8, profiles/r06/numerics_errors.log);  gradients: relative L2 error < 1e-5 (measured <= 1.3e-6) per parameter tensor against
  float64 autograd of the oracle.
Covers one graph per block with the prepared bitmask (N = 150, 200, 224), one graph per block built
in-kernel (adjbits dropped), several graphs per block (N = 20, 64), padding rows, and the fallback for
non-unit weights; and the dense kernels for one graph of 224 < N <= 512 per workgroup (eco_mpnn_dl.h: BA-500,
N = 512 without padding, 497 with a padded last tile, 300 / 225 with waves of unequal tile counts), whose
gradients are checked against float64 autograd of the oracle on the GPU."""

import numpy as np
import pytest
import torch

from oracle import mpnn_oracle as mo

pytestmark = pytest.mark.gpu


def _inputs(n, B, seed, kind="ER", param=0.15):
    from eco_hip.graphs import GraphStore
    g = torch.Generator().manual_seed(seed)
    w = mo.init_weights(g, std=0.1)
    store = GraphStore.random(kind, B, n, param, seed=seed)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    dq = torch.randn(B, n, generator=g)
    return w, store, x.cuda(), dq.cuda()


def _run(net, store, x, dq, scope, dense):
    from eco_hip.networks.mpnn import MPNN
    B, n = x.shape[0], x.shape[1]
    from eco_hip import _lib
    with _lib.kernel_paths(0 if dense else _lib.ECO_PATH_NO_DENSE):
        gids = torch.arange(B, dtype=torch.int32, device="cuda")
        q = net.forward_graphs(x, store, gids, norm_scope=scope).clone()
        saved = torch.empty(MPNN.saved_bytes(n, B), dtype=torch.uint8, device="cuda")
        qs = net.forward_graphs(x, store, gids, norm_scope=1, saved=saved).clone()
        grad = torch.zeros_like(net.flat)
        net.backward_graphs(x, store, gids, saved, dq, grad)
        torch.cuda.synchronize()
        return q.cpu(), qs.cpu(), grad.cpu()


def _scaled_err(a, b):
    e = float(((a - b).abs() / (1 + b.abs())).max())
    print(f"scaled err {e:.3e}")
    return e


@pytest.mark.parametrize("n,B,prepared", [(200, 24, True), (224, 9, True), (150, 16, True), (200, 10, False),
                                          (20, 64, False), (64, 19, False)])
def test_dense_matches_csr_and_oracle(n, B, prepared):
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_GRAPH
    from test_dqn_gpu import _flat_to_dict
    w, store, x, dq = _inputs(n, B, seed=n + B)
    assert store.unit_weights
    assert (store.adjbits is not None) == (104 < n <= 224)
    if not prepared:  # force the in-kernel bitmask build
        store.gs.adjbits = None
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    qd, qsd, gd = _run(net, store, x, dq, ECO_NORM_PER_GRAPH, dense=True)
    qc, qsc, gc = _run(net, store, x, dq, ECO_NORM_PER_GRAPH, dense=False)
    assert torch.isfinite(qd).all() and torch.isfinite(gd).all()
    assert _scaled_err(qd, qc) <= 5e-7 and _scaled_err(qsd, qsc) <= 5e-7
    for b in [0, B // 2, B - 1]:  # oracle, per-graph norm scope (B=1 semantics)
        obs = torch.from_numpy(np.vstack([x[b, :, :7].cpu().numpy().T.astype(np.float64), store.dense(b)])).float()
        assert _scaled_err(qd[b], mo.forward(w, obs)) <= 5e-7
    # gradients: dense vs torch autograd of the oracle (norm.max over the batch, as train_step) evaluated in
    # float64.  The fp32 oracle is not the judge here: a ReLU input within fp32 rounding of 0 takes either
    # side depending on the summation order, and at N=20 the fp32 oracle's own edge-embedding gradients sit
    # 8e-3 from float64 for exactly that reason (seen), while both HIP paths are within 1e-6.
    obs = torch.from_numpy(np.stack([np.vstack([x[b, :, :7].cpu().numpy().T.astype(np.float64), store.dense(b)])
                                     for b in range(B)]))
    w64 = {k: v.double().clone().requires_grad_(True) for k, v in w.items()}
    (mo.forward(w64, obs) * dq.cpu().double()).sum().backward()
    dd, dc = _flat_to_dict(gd), _flat_to_dict(gc)
    for k in mo.KEYS:
        ref = w64[k].grad
        err = float((dd[k].double() - ref).norm() / max(float(ref.norm()), 1e-12))
        print(f"grad {k} rel L2 vs float64 {err:.3e}")
        assert err < 1e-5, (k, err)
        # CSR path: same math, other summation order (a ReLU input within rounding of 0 may take the other
        # side), so this cross-check only catches gross errors
        err_c = float((dd[k] - dc[k]).norm() / max(float(dc[k].norm()), 1e-12))
        assert err_c < 2e-2, (k, err_c)


def test_non_unit_weights_use_the_csr_path():
    """Weights of +-2 are outside the dense kernels' {0, +-1} operand: the store says so and the forward
    still matches the oracle (CSR gather)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    rng = np.random.default_rng(0)
    n, B = 40, 6
    mats = []
    for _ in range(B):
        a = np.triu((rng.random((n, n)) < 0.2) * rng.choice([-2.0, 1.0, 2.0], (n, n)), 1)
        mats.append(a + a.T)
    store = GraphStore.from_dense(mats)
    assert not store.unit_weights and store.adjbits is None
    g = torch.Generator().manual_seed(5)
    w = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g)
    gids = torch.arange(B, dtype=torch.int32, device="cuda")
    q = net.forward_graphs(x.cuda(), store, gids).cpu()
    for b in range(B):
        obs = torch.from_numpy(np.vstack([x[b, :, :7].numpy().T.astype(np.float64), mats[b]])).float()
        assert _scaled_err(q[b], mo.forward(w, obs)) <= 5e-7


@pytest.mark.parametrize("n,B,kind,param", [(500, 6, "BA", 4), (512, 3, "BA", 4), (497, 3, "BA", 4),
                                            (300, 5, "ER", 0.05), (225, 4, "ER", 0.15)])
def test_dense_large_matches_csr_and_oracle(n, B, kind, param):
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ActConfig, ECO_NORM_PER_CALL, ECO_NORM_PER_GRAPH
    from test_dqn_gpu import _flat_to_dict
    w, store, x, dq = _inputs(n, B, seed=n + B, kind=kind, param=param)
    assert store.unit_weights and store.adjbits is not None
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    qd, qsd, gd = _run(net, store, x, dq, ECO_NORM_PER_GRAPH, dense=True)
    qc, qsc, gc = _run(net, store, x, dq, ECO_NORM_PER_GRAPH, dense=False)
    assert torch.isfinite(qd).all() and torch.isfinite(gd).all()
    assert not torch.equal(qd, qc)  # two different kernels ran
    assert _scaled_err(qd, qc) <= 5e-7 and _scaled_err(qsd, qsc) <= 5e-7
    wc = {k: v.cuda() for k, v in w.items()}
    obs = torch.stack([torch.from_numpy(np.vstack([x[b, :, :7].cpu().numpy().T.astype(np.float64), store.dense(b)]))
                       for b in range(B)]).cuda()
    with torch.no_grad():
        for b in range(B):
            assert _scaled_err(qd[b], mo.forward(wc, obs[b].float()).cpu()) <= 5e-7, b
    w64 = {k: v.cuda().double().clone().requires_grad_(True) for k, v in w.items()}
    (mo.forward(w64, obs) * dq.double()).sum().backward()
    dd, dc = _flat_to_dict(gd), _flat_to_dict(gc)
    for k in mo.KEYS:
        ref = w64[k].grad.cpu()
        err = float((dd[k].double() - ref).norm() / max(float(ref.norm()), 1e-12))
        print(f"grad {k} rel L2 vs float64 {err:.3e}")
        assert err < 1e-5, (k, err)
        err_c = float((dd[k] - dc[k]).norm() / max(float(dc[k].norm()), 1e-12))
        assert err_c < 2e-2, (k, err_c)
    # fused greedy act on the dense kernel (per-call norm scope)
    gids = torch.arange(B, dtype=torch.int32, device="cuda")
    q = torch.empty(B, n, device="cuda")
    acts = torch.empty(B, dtype=torch.int32, device="cuda")
    net.forward_graphs(x, store, gids, norm_scope=ECO_NORM_PER_CALL, q_out=q, act=ActConfig(0.0, 1, 0.0, 7, 0),
                       actions_out=acts)
    assert torch.equal(acts.long(), q.argmax(1))


@pytest.mark.parametrize("n,B,p", [(200, 300, 0.15), (20, 64, 0.3)])
def test_forward_pair_matches_two_forwards(n, B, p):
    """eco_mpnn_forward_pair (the double-DQN s' pair of dqn.py:416-428: online greedy argmax + target Q) against
    two separate forwards on the same inputs: ER-200 runs the one-launch two-network dense kernel (one graph per
    block), ER-20 the fallback of two launches.  Bitwise equal Q and actions (the same operations per network)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ActConfig, ECO_NORM_PER_CALL
    store = GraphStore.random("ER", B, n, p, seed=5)
    g = torch.Generator().manual_seed(55)
    wa, wb = mo.init_weights(g, std=0.1), mo.init_weights(g, std=0.1)
    na, nb = MPNN(device="cuda"), MPNN(device="cuda")
    na.load_state_dict(wa)
    nb.load_state_dict(wb)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    xc = x.cuda()
    gids = torch.randperm(B, generator=g).to(torch.int32).cuda()
    greedy = ActConfig(0.0, 1, 0.0, 0, 0)
    a1 = torch.empty(B, dtype=torch.int32, device="cuda")
    q1 = torch.empty(B, n, device="cuda")
    qb1 = torch.empty(B, n, device="cuda")
    na.forward_pair_graphs(nb, xc, store, gids, norm_scope=ECO_NORM_PER_CALL, q_out=q1, act=greedy, actions_out=a1,
                           q_out_other=qb1)
    a2 = torch.empty(B, dtype=torch.int32, device="cuda")
    q2 = torch.empty(B, n, device="cuda")
    na.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL, q_out=q2, act=greedy, actions_out=a2)
    qb2 = nb.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL)
    assert torch.equal(q1, q2)
    assert torch.equal(a1, a2)
    assert torch.equal(qb1, qb2)
    assert torch.equal(a1.long(), q1.argmax(1))


@pytest.mark.parametrize("n,B,p", [(200, 96, 0.15), (20, 64, 0.3), (500, 8, 0.02)])
def test_norm_per_call_reuse(n, B, p):
    """ECO_NORM_PER_CALL_REUSE (train_step's online(s) forward after the s' pair on the same graph ids) takes the
    per-call max degree the previous PER_CALL forward left in the workspace: bitwise the PER_CALL result, with and
    without saved activations, on the dense, the small-graph and the BA-500-size paths.  After a forward on other
    graph ids the workspace holds THEIR maximum, which is the documented contract (the reuse is the caller's
    promise), so the test only checks the same-ids case and that a fresh PER_CALL call restores it."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL, ECO_NORM_PER_CALL_REUSE
    store = GraphStore.random("ER", B, n, p, seed=7)
    g = torch.Generator().manual_seed(77)
    net = MPNN(device="cuda")
    net.load_state_dict(mo.init_weights(g, std=0.1))
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    xc = x.cuda()
    gids = torch.randperm(B, generator=g).to(torch.int32).cuda()
    q_ref = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL).clone()
    q_re = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL_REUSE).clone()
    assert torch.equal(q_ref, q_re)
    saved = torch.empty(net.saved_bytes(n, B), dtype=torch.uint8, device="cuda")
    q_sv = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL_REUSE, saved=saved).clone()
    assert torch.equal(q_ref, q_sv)
    # a different subset of graphs (smaller max degree possible), then the full set again with PER_CALL
    sub = gids[: max(1, B // 4)].contiguous()
    net.forward_graphs(xc[: sub.numel()].contiguous(), store, sub, norm_scope=ECO_NORM_PER_CALL)
    q_again = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL)
    assert torch.equal(q_ref, q_again)


@pytest.mark.parametrize("n,B,p,prepared", [(200, 300, 0.15, True), (224, 9, 0.15, True), (150, 16, 0.3, True),
                                            (200, 10, 0.15, False), (20, 4101, 0.15, False), (64, 19, 0.2, False),
                                            (104, 33, 0.1, False)])
def test_dense3_matches_dense2_bitwise(n, B, p, prepared):
    """The two-tiles-per-wave forward (eco_mpnn_dense3.h, 8 waves) against the one-tile-per-wave forward
    (eco_mpnn_dense2.h, 16 waves, ECO_PATH_DENSE2_FWD): the same MFMAs per accumulator in the same order, so Q,
    the fused epsilon-greedy actions, every saved activation and ReLU mask, the backward's gradients and the paired
    s' forward are bitwise equal -- one graph per block (prepared bitmask or built in-kernel, 13 / 14 tiles, a padded
    last tile) and several graphs per block (ER-20 x 4101: 10-graph blocks and a 1-graph tail)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip import _lib
    from eco_hip._lib import ActConfig, ECO_NORM_PER_CALL, ECO_NORM_PER_GRAPH
    store = GraphStore.random("ER", B, n, p, seed=n + B)
    if not prepared:
        store.gs.adjbits = None
    g = torch.Generator().manual_seed(3 * n + B)
    na, nb = MPNN(device="cuda"), MPNN(device="cuda")
    na.load_state_dict(mo.init_weights(g, std=0.1))
    nb.load_state_dict(mo.init_weights(g, std=0.1))
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    xc = x.cuda()
    gids = torch.randperm(B, generator=g).to(torch.int32).cuda()
    dq = torch.randn(B, n, generator=g).cuda()

    def run(mask):
        with _lib.kernel_paths(mask):
            out = {}
            acts = torch.empty(B, dtype=torch.int32, device="cuda")
            out["q"] = na.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_GRAPH,
                                         act=ActConfig(0.3, 1, 0.0, 11, 5), actions_out=acts,
                                         q_out=torch.empty(B, n, device="cuda")).clone()
            out["acts"] = acts.clone()
            saved = torch.zeros(MPNN.saved_bytes(n, B), dtype=torch.uint8, device="cuda")
            out["qs"] = na.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL, saved=saved).clone()
            out["saved"] = saved
            grad = torch.zeros_like(na.flat)
            na.backward_graphs(xc, store, gids, saved, dq, grad)
            out["grad"] = grad
            a_star = torch.empty(B, dtype=torch.int32, device="cuda")
            qa, qb = torch.empty(B, n, device="cuda"), torch.empty(B, n, device="cuda")
            na.forward_pair_graphs(nb, xc, store, gids, norm_scope=ECO_NORM_PER_CALL, q_out=qa,
                                   act=ActConfig(0.0, 1, 0.0, 0, 0), actions_out=a_star, q_out_other=qb)
            out["pair"] = (qa, qb, a_star)
            torch.cuda.synchronize()
            return out

    old = run(_lib.ECO_PATH_DENSE2_FWD)
    new = run(0)
    assert torch.isfinite(new["q"]).all()
    for k in ("q", "acts", "qs", "saved", "grad"):
        assert torch.equal(new[k], old[k]), k
    for u, v in zip(new["pair"], old["pair"]):
        assert torch.equal(u, v)
