"""Parity of the HIP DQN training path: MPNN backward vs torch autograd of the oracle,
train_step vs the reference's own three train steps (tests/golden/dqn_step.npz),
device replay semantics, and a short batched learn() run.

Floating-point tolerances are stated per test (fp32 throughout)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import mpnn_oracle as mo

pytestmark = pytest.mark.gpu


def _split(obs, n_obs=7):
    obs = np.asarray(obs)
    x = np.zeros((obs.shape[0], obs.shape[2], 8), np.float32)
    x[:, :, :n_obs] = obs[:, :n_obs, :].transpose(0, 2, 1).astype(np.float32)
    return torch.from_numpy(x).cuda(), [a for a in obs[:, n_obs:, :]]


def _flat_to_dict(flat):
    from eco_hip.networks.mpnn import param_layout
    out, off = {}, 0
    for name, shape in param_layout(7):
        n = int(np.prod(shape))
        out[name] = flat[off:off + n].reshape(shape)
        off += n
    return out


@pytest.mark.parametrize("kind,n,B,param", [("ER", 20, 64, 0.15), ("ER", 200, 12, 0.15), ("BA", 60, 20, 4),
                                          ("BA", 300, 6, 4), ("BA", 500, 4, 4)])
def test_backward_matches_autograd(kind, n, B, param):
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL
    g = torch.Generator().manual_seed(n + B)
    w = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    store = GraphStore.random(kind, B, n, param, seed=n)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    dq = torch.randn(B, n, generator=g)
    xc, dqc = x.cuda(), dq.cuda()
    gids = torch.arange(B, dtype=torch.int32, device="cuda")
    saved = torch.empty(MPNN.saved_bytes(n, B), dtype=torch.uint8, device="cuda")
    q = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL, saved=saved)
    grad = torch.zeros_like(net.flat)
    net.backward_graphs(xc, store, gids, saved, dqc, grad)
    # oracle: autograd through the fp32 torch restatement on the batch (norm.max over the batch)
    obs = torch.from_numpy(np.stack([np.vstack([x[b, :, :7].numpy().T.astype(np.float64), store.dense(b)])
                                     for b in range(B)])).float()
    wg = {k: v.clone().requires_grad_(True) for k, v in w.items()}
    qr = mo.forward(wg, obs)
    np.testing.assert_allclose(q.cpu().numpy(), qr.detach().numpy(), rtol=1e-4, atol=1e-5)
    (qr * dq).sum().backward()
    got = _flat_to_dict(grad.cpu())
    for k in mo.KEYS:
        ref = wg[k].grad
        err = (got[k] - ref).norm() / max(ref.norm(), 1e-12)
        assert err < 2e-4, (k, float(err), float(ref.norm()))
    # bitwise reproducible (fixed-order reductions)
    grad2 = torch.zeros_like(net.flat)
    net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL, saved=saved)
    net.backward_graphs(xc, store, gids, saved, dqc, grad2)
    assert torch.equal(grad, grad2)


def _dqn_for(store, n, B=16, **kw):
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    env = VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    args = dict(init_weight_std=0.01, double_dqn=True, clip_Q_targets=False, replay_start_size=500,
                replay_buffer_size=4096, gamma=0.95, update_target_frequency=1000, update_learning_rate=False,
                initial_learning_rate=1e-4, peak_learning_rate=1e-4, final_learning_rate=1e-4,
                update_frequency=32, minibatch_size=64, final_exploration_rate=0.05, final_exploration_step=150000,
                adam_epsilon=1e-8, seed=3)
    args.update(kw)
    return DQN(env, lambda: MPNN(device="cuda"), **args)


def test_train_step_matches_reference_three_steps():
    f = np.load(os.path.join(GOLDEN, "dqn_step.npz"))
    from eco_hip.graphs import GraphStore
    n, M = 20, 16
    # every transition carries its own graph (s and s' share it)
    states = [f[f"s{s}/states"] for s in range(int(f["steps"]))]
    adj = [a for st in states for a in st[:, 7:, :]]
    store = GraphStore.from_dense(adj)
    agent = _dqn_for(store, n, B=M, minibatch_size=M)
    agent.network.load_state_dict({k: torch.from_numpy(f["w0/" + k]) for k in mo.KEYS})
    agent.target_network.load_state_dict({k: torch.from_numpy(f["target/" + k]) for k in mo.KEYS})
    for s in range(int(f["steps"])):
        p = f"s{s}/"
        xs, _ = _split(f[p + "states"])
        xn, _ = _split(f[p + "states_next"])
        gid = torch.arange(s * M, (s + 1) * M, dtype=torch.int32, device="cuda")
        act = torch.from_numpy(f[p + "actions"][:, 0].astype(np.int32)).cuda()
        rew = torch.from_numpy(f[p + "rewards"][:, 0]).cuda()
        done = torch.from_numpy(f[p + "dones"][:, 0]).cuda()
        loss = agent.train_step((xs, act, rew, xn, done, gid))
        ref_loss = float(f[p + "loss"])
        assert abs(loss - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss)), (s, loss, ref_loss)
        got = _flat_to_dict(agent.network.flat.cpu())
        for k in mo.KEYS:
            ref = f[p + "w/" + k]
            # Adam moves every weight by ~lr = 1e-4 per step; agree to 2% of that
            np.testing.assert_allclose(got[k].numpy(), ref, rtol=0, atol=2e-6, err_msg=f"step {s} {k}")


def test_replay_push_sample_distinct_and_consistent():
    from eco_hip.agents.dqn.utils import ReplayBuffer
    n, B, C = 20, 64, 200
    rb = ReplayBuffer(C, n, device="cuda", seed=1)
    for k in range(4):   # wraps the ring
        xs = torch.full((B, n, 8), float(k), device="cuda")
        xs[:, 0, 0] = torch.arange(B, dtype=torch.float32, device="cuda") + 1000 * k
        xn = xs + 0.5
        gids = torch.arange(B, dtype=torch.int32, device="cuda") + 100 * k
        acts = torch.arange(B, dtype=torch.int32, device="cuda") % n
        rews = torch.arange(B, dtype=torch.float64, device="cuda") * 0.25
        dones = (torch.arange(B, device="cuda") % 2).to(torch.uint8)
        rb.add_batch(xs, xn, gids, acts, rews, dones)
    assert len(rb) == C
    xs, act, rew, xn, done, gid = rb.sample(150)
    ident = xs[:, 0, 0].cpu().numpy()
    assert len(np.unique(ident)) == 150                       # without replacement
    torch.testing.assert_close(xn, xs + 0.5)
    b = (ident % 1000).astype(np.int64)
    k = (ident // 1000).astype(np.int64)
    np.testing.assert_array_equal(gid.cpu().numpy(), b + 100 * k)
    np.testing.assert_array_equal(act.cpu().numpy(), b % n)
    np.testing.assert_array_equal(rew.cpu().numpy(), (b * 0.25).astype(np.float32))
    np.testing.assert_array_equal(done.cpu().numpy(), (b % 2).astype(np.float32))
    # slots 0..55 of the ring were overwritten by the 4th batch (positions 192..255 wrap)
    assert set(np.unique(k)) <= {0, 1, 2, 3}


def test_learn_short_run_updates_and_is_finite():
    from eco_hip.graphs import GraphStore
    n, B = 20, 256
    store = GraphStore.random("ER", 1024, n, 0.15, seed=4)
    agent = _dqn_for(store, n, B=B, replay_start_size=2 * B, train_minibatch=128, update_target_frequency=500)
    w0 = agent.network.flat.clone()
    losses = agent.learn(timesteps=B * 2 * n * 3)
    assert agent.grad_steps > 0 and len(losses) > 0
    assert all(np.isfinite(l) for _, l in losses)
    assert not torch.equal(w0, agent.network.flat)
    assert torch.isfinite(agent.network.flat).all()
    # target sync happened at least once and tracks the online net exactly when it does
    agent.sync_target()
    assert torch.equal(agent.target_network.flat, agent.network.flat)
