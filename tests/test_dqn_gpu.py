"""Parity of the HIP DQN training path: MPNN backward vs torch autograd of the oracle,
train_step vs the reference's own three train steps (tests/golden/dqn_step.npz),
device replay semantics, and a short batched learn() run.

Floating-point tolerances are stated per test (fp32 throughout)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import graphs as og
from oracle import mpnn_oracle as mo
from oracle import spinsystem_oracle as so

pytestmark = pytest.mark.gpu


def _split(obs, n_obs=7):
    obs = np.asarray(obs)
    x = np.zeros((obs.shape[0], obs.shape[2], 8 if n_obs <= 8 else 16), np.float32)
    x[:, :, :n_obs] = obs[:, :n_obs, :].transpose(0, 2, 1).astype(np.float32)
    return torch.from_numpy(x).cuda(), [a for a in obs[:, n_obs:, :]]


def _flat_to_dict(flat, n_obs=7):
    from eco_hip.networks.mpnn import param_layout
    out, off = {}, 0
    for name, shape in param_layout(n_obs):
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
                adam_epsilon=1e-8, seed=3, evaluate=False, test_save_path=None)
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


def _s2v_env(store, n, B, T=None):
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (Observable, RewardSignal, ExtraAction, OptimisationTarget, SpinBasis)
    # experiments/train_eco.py:311-315 S2V settings
    return VecSpinSystem(store, B, T or n, observables=[Observable.SPIN_STATE], reward_signal=RewardSignal.DENSE,
                         extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                         spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=None,
                         reversible_spins=False)


def _s2v_dqn(env, **kw):
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    args = dict(init_weight_std=0.01, double_dqn=True, clip_Q_targets=False, replay_start_size=64,
                replay_buffer_size=4096, gamma=0.95, update_target_frequency=1000, update_learning_rate=False,
                initial_learning_rate=1e-4, peak_learning_rate=1e-4, final_learning_rate=1e-4,
                update_frequency=32, minibatch_size=64, final_exploration_rate=0.05, final_exploration_step=150000,
                adam_epsilon=1e-8, seed=4, evaluate=False, test_save_path=None)
    args.update(kw)
    return DQN(env, lambda: MPNN(n_obs_in=1, device="cuda"), **args)


def test_train_step_s2v_matches_reference_three_steps():
    """Irreversible (S2V) train_step (dqn.py:414-428): disallowed actions masked before the double-DQN
    argmax, terminal next states (every spin flipped: all masked, argmax 0) included -- against three
    consecutive reference train steps (tests/golden/dqn_step_s2v.npz).  Bars as the ECO test."""
    f = np.load(os.path.join(GOLDEN, "dqn_step_s2v.npz"))
    from eco_hip.graphs import GraphStore
    n, M = 20, 16
    states = [f[f"s{s}/states"] for s in range(int(f["steps"]))]
    adj = [a for st in states for a in st[:, 1:, :]]
    store = GraphStore.from_dense(adj)
    agent = _s2v_dqn(_s2v_env(store, n, M), minibatch_size=M)
    assert agent.allowed_value == float(f["allowed_action_state"])
    agent.network.load_state_dict({k: torch.from_numpy(f["w0/" + k]) for k in mo.KEYS})
    agent.target_network.load_state_dict({k: torch.from_numpy(f["target/" + k]) for k in mo.KEYS})
    for s in range(int(f["steps"])):
        p = f"s{s}/"
        xs, _ = _split(f[p + "states"], 1)
        xn, _ = _split(f[p + "states_next"], 1)
        gid = torch.arange(s * M, (s + 1) * M, dtype=torch.int32, device="cuda")
        act = torch.from_numpy(f[p + "actions"][:, 0].astype(np.int32)).cuda()
        rew = torch.from_numpy(f[p + "rewards"][:, 0]).cuda()
        done = torch.from_numpy(f[p + "dones"][:, 0]).cuda()
        loss = agent.train_step((xs, act, rew, xn, done, gid))
        ref_loss = float(f[p + "loss"])
        assert np.isfinite(loss)
        assert abs(loss - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss)), (s, loss, ref_loss)
        # terminal s' has no allowed action: the fused argmax returns 0 like masked_fill(-1e4).argmax
        term = f[p + "dones"][:, 0] == 1
        assert (agent.a_star.cpu().numpy()[term] == 0).all()
        got = _flat_to_dict(agent.network.flat.cpu(), 1)
        for k in mo.KEYS:
            np.testing.assert_allclose(got[k].numpy(), f[p + "w/" + k], rtol=0, atol=2e-6, err_msg=f"step {s} {k}")


def test_learn_s2v_resets_finished_episodes():
    """S2V episodes end after N flips, before max_steps = 2N: iteration() resets them at once, so no
    dead steps are pushed (every stored transition comes from a live episode: exactly one terminal per
    episode) and every episode restarts from all -1 spins."""
    from eco_hip.graphs import GraphStore
    n, B = 20, 64
    store = GraphStore.random("ER", 256, n, 0.15, seed=9)
    env = _s2v_env(store, n, B, T=2 * n)
    agent = _s2v_dqn(env, replay_buffer_size=B * 2 * n * 4, replay_start_size=B * n, compact_replay=False)
    agent.start()
    for _ in range(3 * n):
        agent.iteration()
    assert agent.grad_steps > 0
    rb = agent.replay_buffer
    size = len(rb)
    assert size == B * 3 * n
    dones = rb.done[:size].cpu().numpy().reshape(3 * n, B)
    # episodes of exactly n steps, back to back: terminal at vector steps n-1, 2n-1, 3n-1
    expect = np.zeros(3 * n)
    expect[[n - 1, 2 * n - 1, 3 * n - 1]] = 1
    np.testing.assert_array_equal(dones, np.repeat(expect[:, None], B, axis=1))
    # s of the first step of each episode is all -1 (irreversible reset, spinsystem.py:295-297)
    xs = rb.xs[:size].cpu().numpy().reshape(3 * n, B, n, 8)
    for t0 in (0, n, 2 * n):
        assert (xs[t0, :, :, 0] == -1).all()
    assert np.isfinite(agent.losses()).all()


def _oracle_greedy_chunk(w, mats, inits, T, metric_rows):
    """Lockstep greedy rollouts of one evaluate_agent batch: predict couples norm.max() over the
    active batch (dqn.py:546-547).  Returns per episode (best_score, best_solution, final score,
    final cut, cumulative reward, tie flag)."""
    envs = [so.SpinSystemOracle(J, T, basin_reward=1. / J.shape[0]) for J in mats]
    obs = [e.reset(spins=s) for e, s in zip(envs, inits)]
    cum = [0.0] * len(envs)
    tie = np.zeros(len(envs), bool)   # per episode: its own argmax only depends on its own state
    for _ in range(T):
        q = mo.forward(w, torch.from_numpy(np.array(obs)).float()).reshape(len(envs), -1)
        top = torch.topk(q, 2, dim=1).values
        tie |= (top[:, 0] - top[:, 1] < 1e-4 * (1 + top[:, 0].abs())).numpy()
        acts = q.argmax(1)
        for i, e in enumerate(envs):
            obs[i], r, _, _ = e.step(int(acts[i]))
            cum[i] += r
    return [(e.best_score, e.best_solution, e.score, so.calculate_cut(e.state[0], e.matrix), c, bool(t))
            for e, c, t in zip(envs, cum, tie)]


@pytest.mark.parametrize("metric", ["BEST", "FINAL", "CUMULATIVE_REWARD", "ENERGY_ERROR"])
def test_evaluate_agent_matches_oracle(metric):
    """evaluate_agent (dqn.py:514-602): 6 test episodes in batches of 4 (a refill batch of 2 couples
    norm.max() over 2 graphs), graphs taken in order, greedy MPNN rollouts vs the oracle's."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.agents.dqn.utils import TestMetric
    n, T = 20, 40
    rng = np.random.default_rng(31)
    mats = [og.er_graph(n, 0.3, rng) for _ in range(6)]
    store = GraphStore.from_dense(mats)
    kw = dict(observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS, extra_action=ExtraAction.NONE,
              optimisation_target=OptimisationTarget.CUT, spin_basis=SpinBasis.SIGNED, norm_rewards=True,
              basin_reward=1. / n)
    test_env = VecSpinSystem(store, 4, T, **kw)
    agent = _dqn_for(GraphStore.random("ER", 8, n, 0.15, seed=1), n, B=8, test_envs=test_env, test_episodes=6,
                     minibatch_size=4, test_metric=TestMetric[metric])
    w = mo.init_weights(torch.Generator().manual_seed(8), std=0.5)  # well-separated Q (no argmax near-ties)
    agent.network.load_state_dict(w)
    score, sol = agent.evaluate_agent()
    # the initial spins evaluate_agent drew: the same masked resets on a twin env
    twin = VecSpinSystem(store, 4, T, **kw)
    inits = []
    for seed, gids in ((agent.seed, [0, 1, 2, 3]), (agent.seed + 4, [4, 5])):
        mask = np.zeros(4, np.uint8)
        mask[:len(gids)] = 1
        twin.reset(graph_ids=np.array(gids + [0] * (4 - len(gids))), mask=mask, seed=seed)
        sp = twin.read(spins=True)["spins"].cpu().numpy()
        inits.append(sp[:len(gids)].astype(np.int64))
    res = (_oracle_greedy_chunk(w, mats[:4], inits[0], T, None) + _oracle_greedy_chunk(w, mats[4:], inits[1], T, None))
    col = {"BEST": (0, 1), "FINAL": (2, 3), "CUMULATIVE_REWARD": (4, None), "ENERGY_ERROR": (None, None)}[metric]
    got_s, got_o = agent.last_evaluation
    # episodes complete in lockstep: batch 1 in slot order, then batch 2
    assert len(got_s) == 6
    checked = 0
    for i, r in enumerate(res):
        if r[5]:
            continue   # a near-tie argmax in the oracle rollout: trajectories may legitimately differ
        checked += 1
        assert got_s[i] == (r[col[0]] if col[0] is not None else 0.0), (i, got_s[i], r)
        assert got_o[i] == (r[col[1]] if col[1] is not None else 0.0), (i, got_o[i], r)
    assert checked >= 3, "too many near-ties to check the rollouts"
    if checked == 6:
        assert score == pytest.approx(np.mean(got_s), rel=1e-15) and sol == pytest.approx(np.mean(got_o), rel=1e-15)
    # the next call continues with the following graphs in order (ordered SetGraphGenerator)
    assert test_env._eval_next_graph == 0
    # every test episode in one fill (4 episodes, 4 slots, lockstep): the sync-free path of evaluate_agent takes
    # graphs 0..3 from the same spins as the first refill batch above, so it must reproduce those rollouts
    agent.test_episodes = 4
    score4, sol4 = agent.evaluate_agent()
    got_s4, got_o4 = agent.last_evaluation
    assert len(got_s4) == 4 and test_env._eval_next_graph == 4
    for i, r in enumerate(res[:4]):
        if r[5]:
            continue
        assert got_s4[i] == (r[col[0]] if col[0] is not None else 0.0), (i, got_s4[i], r)
        assert got_o4[i] == (r[col[1]] if col[1] is not None else 0.0), (i, got_o4[i], r)
    assert got_s4 == got_s[:4] and got_o4 == got_o[:4]


def test_learn_evaluates_saves_and_pickles(tmp_path):
    """learn() side effects (dqn.py:349-394): evaluate every test_frequency env-steps once training
    is ready, `_best` network on a new best, periodic checkpoints, and the three pickles."""
    import pickle
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.agents.dqn.utils import TestMetric
    n, B = 20, 64
    store = GraphStore.random("ER", 256, n, 0.15, seed=4)
    test_env = VecSpinSystem(GraphStore.random("ER", 8, n, 0.15, seed=5), 8, 2 * n,
                             **{k: v for k, v in _dqn_for(store, n, B=B).env.env_args.items()})
    net_path = str(tmp_path / "network.pth")
    agent = _dqn_for(store, n, B=B, replay_start_size=2 * B, train_minibatch=64, evaluate=True,
                     test_envs=test_env, test_episodes=8, test_frequency=B * 10, test_metric=TestMetric.BEST,
                     save_network_frequency=B * 20, network_save_path=net_path,
                     test_save_path=str(tmp_path / "test_scores.pkl"))
    agent.learn(timesteps=B * 41)
    with open(tmp_path / "test_scores.pkl", "rb") as fh:
        ts = pickle.load(fh)
    assert [int(t) for t in ts[:, 0]] == [B * 10, B * 20, B * 30, B * 40]
    assert (tmp_path / "network_best.pth").exists()
    for k in (20, 40):
        assert (tmp_path / f"network{B * k}.pth").exists()
    with open(tmp_path / "losses.pkl", "rb") as fh:
        lo = pickle.load(fh)
    assert lo.shape[1] == 2 and len(lo) == agent.grad_steps and np.isfinite(lo).all()
    with open(tmp_path / "solution.pkl", "rb") as fh:
        sol = pickle.load(fh)
    assert sol.shape == (4, 2)
    # the saved checkpoint is a plain state_dict with the reference's keys
    sd = torch.load(tmp_path / f"network{B * 40}.pth", map_location="cpu", weights_only=True)
    assert list(sd) == mo.KEYS


def test_overlapped_evaluation_matches_synchronous(tmp_path):
    """learn() runs its one-fill evaluations on a side stream on a snapshot of the weights while training goes on
    (DQN.overlap_evaluation, default on), each evaluation after the first replaying its rollout from a HIP graph
    (DQN.eval_graphs).  Against the same run with synchronous, eagerly launched evaluate_agent() calls: the same
    test scores and solutions at the same timesteps, the same `_best` network file, the same training losses; and
    likewise for synchronous calls that replay the graph."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.agents.dqn.utils import TestMetric
    n, B = 20, 64
    out = []
    for overlap, graphs in ((False, False), (True, True), (False, True)):
        store = GraphStore.random("ER", 256, n, 0.15, seed=4)
        test_env = VecSpinSystem(GraphStore.random("ER", 8, n, 0.15, seed=5), 8, 2 * n,
                                 **{k: v for k, v in _dqn_for(store, n, B=B).env.env_args.items()})
        d = tmp_path / f"{overlap}_{graphs}"
        d.mkdir()
        agent = _dqn_for(store, n, B=B, replay_start_size=2 * B, train_minibatch=64, evaluate=True,
                         test_envs=test_env, test_episodes=8, test_frequency=B * 5, test_metric=TestMetric.BEST,
                         save_network_frequency=B * 1000, network_save_path=str(d / "network.pth"),
                         test_save_path=None, overlap_evaluation=overlap)
        agent.eval_graphs = graphs
        assert agent._one_fill_ok(test_env, None)
        losses = agent.learn(timesteps=B * 41)
        best = torch.load(d / "network_best.pth", map_location="cpu", weights_only=True)
        replayed = sum(r["graph"] is not None for r in agent._eval_graphs.values())
        out.append((agent.test_scores, agent.test_solutions, losses, best, agent._eval_net is not None, replayed))
    (s0, o0, l0, b0, e0, g0), (s1, o1, l1, b1, e1, g1), (s2, o2, l2, b2, e2, g2) = out
    assert not e0 and e1 and not e2  # the second run did overlap
    assert g0 == 0 and g1 == 1 and g2 == 1  # the eager run captured nothing; the others replayed a HIP graph
    assert [t for t, _ in s0] == [B * k for k in range(5, 41, 5)]
    # eager launches, the overlapped graph replay and the synchronous graph replay: identical scores, _best, losses
    assert s0 == s1 == s2 and o0 == o1 == o2 and l0 == l1 == l2
    assert all(torch.equal(b0[k], b1[k]) and torch.equal(b0[k], b2[k]) for k in b0)


@pytest.mark.parametrize("n,B,basis,kind", [(20, 64, "SIGNED", "ER"), (200, 16, "BINARY", "ER"),
                                            (257, 12, "SIGNED", "ER"), (500, 8, "SIGNED", "BA")])
def test_compact_replay_matches_feature_replay(n, B, basis, kind):
    """The compact replay (integer env state per transition, features rebuilt on sample) returns exactly
    the transitions the fp32 feature ring returns for the same pushes and the same sampling keys: node
    features bitwise, actions, rewards, dones, graph ids -- across a masked reset (new s rows) and a
    ring wrap.  The compact ring stores one state per transition: 4N + 80 B against 64N B (<= 1 KB at N=200).
    N = 257 and BA-500 (configs[3]) take the sample kernel's 128-thread path for N > 256 (several vertices per
    thread, csrc/eco_train.hip replay_compact_sample)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.agents.dqn.utils import ReplayBuffer, CompactReplayBuffer
    store = GraphStore.random(kind, 2 * B, n, 0.15 if kind == "ER" else 4, seed=n)
    env = VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis[basis], norm_rewards=True, basin_reward=1. / n)
    C = B * 5
    feat = ReplayBuffer(C, n, device="cuda", seed=17)
    comp = CompactReplayBuffer(C, env, seed=17)
    # bytes: one u32 per vertex + 80 B of scalars per slot (+ 256-B alignment of the 7 arrays)
    assert comp.bytes_per_transition <= 4 * n + 80 + 7 * 256 / (C + B)
    assert n != 200 or comp.bytes_per_transition <= 1024
    env.reset(graph_ids=np.arange(B), seed=3)
    comp.snapshot()
    g = torch.Generator(device="cuda").manual_seed(5)
    x = env.obs_x.clone()
    for t in range(8):
        acts = torch.randint(0, n, (B,), generator=g, device="cuda", dtype=torch.int32)
        nxt = torch.empty_like(x)
        _, rew, done = env.step(acts, obs_out=nxt)
        feat.add_batch(x, nxt, env.graph_ids, acts, rew, done)
        comp.add_step(acts, rew, done)
        x = nxt.clone()
        if t == 3:  # masked reset of half the episodes onto new graphs
            mask = (torch.arange(B, device="cuda") % 2).to(torch.uint8)
            env.reset(graph_ids=np.arange(B) + B, mask=mask, seed=9)
            comp.snapshot(mask)
            x = env.obs_x.clone()
    env.check_errors()
    assert len(feat) == len(comp) == C
    for m in (C // 2, C):
        a = feat.sample(m)
        b = comp.sample(m)
        for u, v in zip(a, b):
            assert torch.equal(u.view(torch.int32) if u.dtype == torch.float32 else u,
                               v.view(torch.int32) if v.dtype == torch.float32 else v)


@pytest.mark.parametrize("flag", [False, True])
def test_update_exploration_quirk_matches_reference(flag):
    """dqn.py:161 stores `update_exploration` as a one-tuple, so learn() decays epsilon even when False is
    passed (:285-286).  tests/golden/exploration.npz records the reference's epsilon after every
    update_epsilon call of a 60-step learn(); one episode (B = 1) reproduces that sequence exactly."""
    from eco_hip.graphs import GraphStore
    f = np.load(os.path.join(GOLDEN, "exploration.npz"))
    key = str(int(flag))
    assert bool(f[key + "/attr_truthy"])
    n = 20
    store = GraphStore.random("ER", 4, n, 0.15, seed=8)
    agent = _dqn_for(store, n, B=1, update_exploration=flag, initial_exploration_rate=1, final_exploration_rate=0.1,
                     final_exploration_step=40, replay_start_size=10 ** 6, replay_buffer_size=1000)
    assert bool(agent.update_exploration)
    trace = []
    agent.learn(timesteps=len(f[key + "/eps"]), on_vector_step=lambda t: trace.append(agent.epsilon))
    np.testing.assert_array_equal(np.array(trace), f[key + "/eps"])
    assert agent.epsilon == float(f[key + "/final_eps"])


def test_regenerate_graphs_with_replay_longer_than_an_episode_batch():
    """replay capacity > B * max_steps.  Lockstep episodes need ceil(C / (B T)) + 1 batches of B
    graph slots in rotation (a smaller store is rejected); with them every episode batch runs on graphs
    regenerated on the device, and no slot is regenerated while a stored transition may reference it."""
    from eco_hip.graphs import GraphStore, edge_cap
    from eco_hip.agents.dqn.dqn import graph_slots_needed
    n, B = 20, 64
    T = 2 * n
    C = B * T * 2 + 100                       # 2.04 episode batches of transitions
    need = graph_slots_needed(B, T, C)
    assert need == 4 * B
    with pytest.raises(ValueError, match="GraphStore.slots"):
        _dqn_for(GraphStore.slots(2 * B, n, edge_cap("ER", n, 0.15)), n, B=B, replay_buffer_size=C,
                 regenerate_graphs=("ER", 0.15))
    st = GraphStore.slots(need, n, edge_cap("ER", n, 0.15))
    agent = _dqn_for(st, n, B=B, replay_buffer_size=C, replay_start_size=B * 4, train_minibatch=128,
                     regenerate_graphs=("ER", 0.15))
    seen = []

    def snap(t):
        if agent._steps_in_episode == 0:       # a full reset just happened
            seen.append((agent.env.graph_ids.cpu().numpy().copy(), st.edges.clone(), agent._pushed))
    agent.learn(timesteps=B * T * 6, on_vector_step=snap)
    agent.env.check_errors()
    assert agent.graphs_reused == 0 and agent.graphs_regenerated == B * 7
    assert len(seen) == 6
    for i in range(1, len(seen)):
        ids_prev, ids = seen[i - 1][0], seen[i][0]
        assert not set(ids_prev) & set(ids)                       # a new batch of slots each time
        # the slots handed out were regenerated: their edges differ from what they held before
        assert not torch.equal(seen[i][1], seen[i - 1][1])
    # slot batch k is reused at batch k + 4: by then >= C pushes have passed since it was left
    assert np.array_equal(np.sort(seen[4][0]), np.sort(seen[0][0]))
    assert seen[4][2] - seen[1][2] >= C
    assert agent.grad_steps > 0 and torch.isfinite(agent.network.flat).all()


def test_evaluation_on_the_regenerated_training_store_is_synchronous(tmp_path):
    """with regenerate_graphs and test_envs=None the test env reads the training slot store,
    which the main stream regenerates while training goes on; learn() must not overlap such an evaluation (no event
    orders the regeneration after the side stream).  Overlap on and off give the same scores, solutions, losses and
    `_best` file, and the overlap-on run evaluated synchronously."""
    from eco_hip.graphs import GraphStore, edge_cap
    from eco_hip.agents.dqn.dqn import graph_slots_needed
    from eco_hip.agents.dqn.utils import TestMetric
    n, B = 20, 64
    T = 2 * n
    C = B * T
    out = []
    for overlap in (False, True):
        st = GraphStore.slots(graph_slots_needed(B, T, C), n, edge_cap("ER", n, 0.15))
        d = tmp_path / str(overlap)
        d.mkdir()
        agent = _dqn_for(st, n, B=B, replay_buffer_size=C, replay_start_size=2 * B, train_minibatch=64,
                         regenerate_graphs=("ER", 0.15), evaluate=True, test_envs=None, test_episodes=8,
                         test_frequency=B * 10, test_metric=TestMetric.BEST, save_network_frequency=B * 1000,
                         network_save_path=str(d / "network.pth"), test_save_path=None, overlap_evaluation=overlap)
        assert not agent._overlap_ok(agent._test_env())
        losses = agent.learn(timesteps=B * T * 2)
        best = torch.load(d / "network_best.pth", map_location="cpu", weights_only=True)
        out.append((agent.test_scores, agent.test_solutions, losses, best, agent._eval_net is not None))
    (s0, o0, l0, b0, e0), (s1, o1, l1, b1, e1) = out
    assert not e0 and not e1  # neither run overlapped
    assert len(s0) == B * T * 2 // (B * 10) and s0 == s1 and o0 == o1 and l0 == l1
    assert all(torch.equal(b0[k], b1[k]) for k in b0)


def test_learn_with_staggered_dones_resets_only_finished_episodes():
    """with Stopping.EARLY (spinsystem.py:541-556, done after 15 steps without a new best)
    episodes finish at different steps, so learn() takes the partial-reset path of iteration() (dqn.py:306-327
    resets each finished env on its own) without regenerate_graphs.  Every reset episode gets a pool graph,
    the live ones keep theirs, and training proceeds; a second learn() reports only its own losses
    (the reference's `losses` list is local to learn(), dqn.py:269)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis, Stopping)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    n, B = 20, 64
    pool = np.arange(100, 228)
    store = GraphStore.random("ER", 256, n, 0.15, seed=12)
    env = VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n,
                        stopping=Stopping.EARLY)
    agent = DQN(env, lambda: MPNN(device="cuda"), init_weight_std=0.01, replay_start_size=4 * B,
                replay_buffer_size=4096, gamma=0.95, update_target_frequency=1000, update_learning_rate=False,
                initial_learning_rate=1e-4, peak_learning_rate=1e-4, final_learning_rate=1e-4, update_frequency=32,
                minibatch_size=64, final_exploration_rate=0.05, final_exploration_step=20000, seed=21,
                evaluate=False, test_save_path=None, graph_pool_ids=pool)
    hist = {"partial": 0}
    prev = {}

    def watch(t):
        gids = agent.env.graph_ids.cpu().numpy()
        steps = agent.env.read()["current_step"].cpu().numpy()
        assert np.isin(gids, pool).all()
        if "steps" in prev:
            reset = steps == 0
            if reset.any() and not reset.all():
                hist["partial"] += 1
                # episodes that were not reset kept their graph and advanced by one step
                keep = ~reset
                np.testing.assert_array_equal(gids[keep], prev["gids"][keep])
                np.testing.assert_array_equal(steps[keep], prev["steps"][keep] + 1)
        prev["gids"], prev["steps"] = gids, steps

    first = agent.learn(timesteps=B * 60, on_vector_step=watch)
    assert not agent._lockstep
    assert hist["partial"] > 0, "no staggered resets happened"
    assert agent.grad_steps > 0 and torch.isfinite(agent.network.flat).all()
    n1 = len(agent.losses())
    assert n1 == agent.grad_steps and len(first) == min(100, n1)
    agent.learn(timesteps=B * 20)
    second = agent.losses()
    assert len(second) == agent.grad_steps - n1 > 0


def test_stagger_episodes_spreads_phases_with_fresh_graphs():
    """DQN.stagger_episodes on a lockstep env (reversible spins, Stopping.NORMAL): episode b's first episode is cut
    after T - (b T // B) steps, then every episode runs the full T steps, so the B episodes sit at evenly spread
    phases.  Checked every vector step against the env's own step counters: each episode's current step follows
    that schedule, exactly the episodes whose counters wrap are reset (fresh graph slots with regenerate_graphs,
    the others keep theirs), and training proceeds.  The truncated transition is not terminal: the env's done flag
    is set only at max_steps, which the replay stores as it is (the steps before the truncation all read done 0)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN, graph_slots_needed
    n, B = 20, 64
    T = 2 * n
    cap = B * 8
    store = GraphStore.generated("ER", graph_slots_needed(B, T, cap), n, 0.15, seed=5, device="cuda")
    env = VecSpinSystem(store, B, T, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    agent = DQN(env, lambda: MPNN(device="cuda"), init_weight_std=0.01, replay_start_size=2 * B,
                replay_buffer_size=cap, gamma=0.95, update_target_frequency=1000, update_learning_rate=False,
                initial_learning_rate=1e-4, peak_learning_rate=1e-4, final_learning_rate=1e-4, update_frequency=32,
                minibatch_size=64, final_exploration_rate=0.05, final_exploration_step=20000, seed=21,
                evaluate=False, test_save_path=None, regenerate_graphs=("ER", 0.15))
    agent.stagger_episodes = True
    first_len = T - (np.arange(B) * T) // B
    k = {"v": 0}
    prev = {}

    def watch(t):
        k["v"] += 1
        kv = k["v"]
        steps = agent.env.read()["current_step"].cpu().numpy().astype(np.int64)
        gids = agent.env.graph_ids.cpu().numpy()
        expect = np.where(kv < first_len, kv, (kv - first_len) % T)
        np.testing.assert_array_equal(steps, expect)
        if prev:
            reset = expect == 0
            np.testing.assert_array_equal(gids[~reset], prev["gids"][~reset])
            assert not np.isin(gids[reset], prev["gids"]).any()  # fresh slots (none shared with live episodes)
        prev["gids"] = gids

    agent.learn(timesteps=B * 3 * T, on_vector_step=watch)
    assert agent._stagger and agent.graphs_regenerated > 0
    assert agent.grad_steps > 0 and torch.isfinite(agent.network.flat).all()
    # phases are spread: after the first truncations every step resets B / T episodes
    assert sorted(set(((k["v"] - first_len) % T).tolist())) == list(range(T))
