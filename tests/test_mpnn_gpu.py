"""Parity of the HIP MPNN forward + fused act with the reference MPNN outputs
(tests/golden/mpnn_fwd.npz, produced by the reference itself) and with the fp32
torch oracle (oracle/mpnn_oracle.py) at batch scale.

Tolerance (floating point, fp32): |q - q_ref| <= 5e-7 * (1 + |q_ref|).  The kernels compute with 22-bit
fp16x2 operand splits and f32 accumulation in another summation order than torch CPU; measured round 6
(profiles/r06/numerics_errors.log): at most 6.7e-8, i.e. fp32 rounding level, so the bar leaves ~7x headroom
(it was 2e-5 / 5e-5 before round 6).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import mpnn_oracle as mo

pytestmark = pytest.mark.gpu
RTOL = 5e-7


def _close(q, ref, tol=RTOL):
    q = np.asarray(q, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    err = np.abs(q - ref) / (1.0 + np.abs(ref))
    print(f"max scaled err {err.max():.3e} (bar {tol:.0e})")
    assert err.max() <= tol, f"max scaled err {err.max():.3e}"


def _net(f, prefix):
    from eco_hip.networks.mpnn import MPNN
    net = MPNN(n_obs_in=7, device="cuda")
    net.load_state_dict({k: torch.from_numpy(f[prefix + k]) for k in mo.KEYS})
    return net


def _split(obs, n_obs=7):
    """reference observation [B, n_obs+N, N] -> (node features [B,N,8] fp32, adjacencies)."""
    obs = np.asarray(obs)
    x = np.zeros((obs.shape[0], obs.shape[2], 8), np.float32)
    x[:, :, :n_obs] = obs[:, :n_obs, :].transpose(0, 2, 1).astype(np.float32)
    return torch.from_numpy(x).cuda(), [a for a in obs[:, n_obs:, :]]


def test_forward_matches_reference_pretrained_er200():
    from eco_hip.graphs import GraphStore
    from eco_hip._lib import ECO_NORM_PER_GRAPH, ECO_NORM_PER_CALL
    f = np.load(os.path.join(GOLDEN, "mpnn_fwd.npz"))
    net = _net(f, "er200/")
    x, adj = _split(f["er200/obs"])
    store = GraphStore.from_dense(adj)
    gids = torch.arange(2, dtype=torch.int32, device="cuda")
    q1 = net.forward_graphs(x, store, gids, norm_scope=ECO_NORM_PER_GRAPH).cpu().numpy()
    _close(q1, f["er200/q_b1"])
    q2 = net.forward_graphs(x, store, gids, norm_scope=ECO_NORM_PER_CALL).cpu().numpy()
    _close(q2, f["er200/q_b2"])
    xb, adjb = _split(f["er200/obs_binary"][None])
    qb = net.forward_graphs(xb, GraphStore.from_dense(adjb), gids[:1]).cpu().numpy()
    _close(qb[0], f["er200/q_binary"])


def test_forward_matches_reference_er20_batch_and_quirks():
    from eco_hip._lib import ECO_NORM_PER_CALL
    from eco_hip.graphs import GraphStore
    f = np.load(os.path.join(GOLDEN, "mpnn_fwd.npz"))
    net = _net(f, "er20/")
    x, adj = _split(f["er20/obs"])
    store = GraphStore.from_dense(adj)
    gids = torch.arange(8, dtype=torch.int32, device="cuda")
    q8 = net.forward_graphs(x, store, gids, norm_scope=ECO_NORM_PER_CALL).cpu().numpy()
    _close(q8, f["er20/q_b8"])
    # reference-format drop-in forward, incl. the in-place transpose_ (mpnn.py:44)
    t = torch.from_numpy(f["er20/obs"]).float().cuda()
    q = net(t).cpu().numpy()
    _close(q, f["er20/q_b8"])
    np.testing.assert_array_equal(t.cpu().numpy(), f["er20/input_after_forward"])
    q1 = net(torch.from_numpy(f["er20/obs"][3]).float().cuda()).cpu().numpy()
    _close(q1, f["er20/q_b1"][3])


@pytest.mark.parametrize("n,B", [(20, 512), (200, 96), (500, 8)])
def test_forward_matches_oracle_at_scale(n, B):
    """Seeded random features and weights; BA graphs at N=500 (hubs), ER elsewhere."""
    from eco_hip.graphs import GraphStore
    from eco_hip._lib import ECO_NORM_PER_GRAPH
    from eco_hip.networks.mpnn import MPNN
    g = torch.Generator().manual_seed(n)
    w = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    store = GraphStore.random("BA" if n == 500 else "ER", B, n, 4 if n == 500 else 0.15, seed=n)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    gids = torch.arange(B, dtype=torch.int32, device="cuda")
    q = net.forward_graphs(x.cuda(), store, gids, norm_scope=ECO_NORM_PER_GRAPH).cpu().numpy()
    for b in [0, 1, B // 2, B - 1]:
        J = store.dense(b)
        obs = torch.from_numpy(np.vstack([x[b, :, :7].numpy().T.astype(np.float64), J])).float()
        ref = mo.forward(w, obs).numpy()
        _close(q[b], ref)


def test_fused_act_greedy_and_epsilon():
    from eco_hip.graphs import GraphStore
    from eco_hip._lib import ActConfig
    from eco_hip.networks.mpnn import MPNN
    n, B = 200, 1024
    g = torch.Generator().manual_seed(1)
    net = MPNN(device="cuda")
    net.load_state_dict(mo.init_weights(g, std=0.1))
    store = GraphStore.random("ER", B, n, 0.15, seed=2)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g)
    x = x.cuda()
    gids = torch.arange(B, dtype=torch.int32, device="cuda")
    q = torch.empty(B, n, device="cuda")
    acts = torch.empty(B, dtype=torch.int32, device="cuda")
    act = ActConfig(0.0, 1, 0.0, 7, 0)
    net.forward_graphs(x, store, gids, q_out=q, act=act, actions_out=acts)
    assert torch.equal(acts.long(), q.argmax(1))
    act = ActConfig(1.0, 1, 0.0, 7, 1)
    net.forward_graphs(x, store, gids, q_out=q, act=act, actions_out=acts)
    a = acts.cpu().numpy()
    assert a.min() >= 0 and a.max() < n and len(np.unique(a)) > 150
    # irreversible masking: only vertices whose feature 0 equals allowed_value
    x[:, :, 0] = 1.0
    x[:, 5, 0] = -1.0
    x[:, 17, 0] = -1.0
    for eps in (0.0, 1.0):
        act = ActConfig(eps, 0, -1.0, 7, 2)
        net.forward_graphs(x, store, gids, q_out=q, act=act, actions_out=acts)
        assert set(np.unique(acts.cpu().numpy())) <= {5, 17}


def test_teacher_forced_greedy_rollout_pretrained_er200():
    """Env + MPNN on one ER-200 graph, reference actions injected; our greedy argmax must
    equal the reference's wherever the reference's top-1/top-2 margin exceeds fp32 noise."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    f = np.load(os.path.join(GOLDEN, "greedy_er200.npz"))
    w = np.load(os.path.join(GOLDEN, "mpnn_fwd.npz"))
    net = _net(w, "er200/")
    J = f["J"].astype(np.float64)
    n = J.shape[0]
    store = GraphStore.from_dense([J])
    env = VecSpinSystem(store, 1, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    x = env.reset(graph_ids=[0], spins=f["spins"][None].astype(np.int64))
    gids = torch.zeros(1, dtype=torch.int32, device="cuda")
    act = torch.zeros(1, dtype=torch.int32, device="cuda")
    agree = checked = 0
    for t, (a_ref, margin) in enumerate(zip(f["actions"], f["margins"])):
        q = net.forward_graphs(x, store, gids)
        if margin > 1e-4:
            checked += 1
            agree += int(q[0].argmax().item() == a_ref)
        act.fill_(int(a_ref))
        x, r, d = env.step(act)
        assert r.item() == f["rewards"][t]
    assert checked > 300 and agree == checked
    assert env.read()["best_solution"][0].item() == f["best_solution"]
