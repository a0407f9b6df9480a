"""ECO training for the set problems: the MPNN with all 13 MAIN_OBSERVABLES as node features
(n_obs_in = 13, 16-float feature rows, CSR-gather kernels) fed by the generic-scorer env.

Bars as test_dqn_gpu / test_mpnn_gpu (fp32): Q within 5e-5 (1 + |q|) of the torch oracle of mpnn.py;
gradients within 2e-4 relative L2 error of torch autograd per parameter tensor."""
import numpy as np
import pytest
import torch

from oracle import mpnn_oracle as mo

pytestmark = pytest.mark.gpu

NOBS = 13


def _weights(n_obs, seed, std=0.1):
    from eco_hip.networks.mpnn import param_layout
    g = torch.Generator().manual_seed(seed)
    w = {}
    for k, shape in param_layout(n_obs):
        w[k] = (torch.rand(shape, generator=g) * 2 - 1) / 128 ** 0.5 if k.endswith("bias") else \
            torch.randn(shape, generator=g) * std
    return w


def _flat_to_dict(flat, n_obs):
    from eco_hip.networks.mpnn import param_layout
    out, off = {}, 0
    for name, shape in param_layout(n_obs):
        n = int(np.prod(shape))
        out[name] = flat[off:off + n].reshape(shape)
        off += n
    return out


def _scaled_err(a, b):
    return float(((a - b).abs() / (1 + b.abs())).max())


@pytest.mark.parametrize("kind,n,B,param", [("ER", 40, 16, 0.2), ("ER", 200, 6, 0.15), ("BA", 130, 8, 4)])
def test_wide_mpnn_forward_backward_matches_autograd(kind, n, B, param):
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL, obs_x_stride
    w = _weights(NOBS, n + B)
    net = MPNN(n_obs_in=NOBS, device="cuda")
    net.load_state_dict(w)
    store = GraphStore.random(kind, B, n, param, seed=n, weights="uniform")
    g = torch.Generator().manual_seed(7 * n)
    x = torch.zeros(B, n, obs_x_stride(NOBS))
    x[:, :, :NOBS] = torch.rand(B, n, NOBS, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    dq = torch.randn(B, n, generator=g)
    xc, dqc = x.cuda(), dq.cuda()
    gids = torch.arange(B, dtype=torch.int32, device="cuda")
    saved = torch.empty(MPNN.saved_bytes(n, B), dtype=torch.uint8, device="cuda")
    q = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL, saved=saved)
    grad = torch.zeros_like(net.flat)
    net.backward_graphs(xc, store, gids, saved, dqc, grad)
    obs = torch.from_numpy(np.stack([np.vstack([x[b, :, :NOBS].numpy().T.astype(np.float64), store.dense(b)])
                                     for b in range(B)])).float()
    wg = {k: v.clone().requires_grad_(True) for k, v in w.items()}
    qr = mo.forward(wg, obs, n_obs_in=NOBS)
    assert _scaled_err(q.cpu(), qr.detach()) <= 5e-5
    (qr * dq).sum().backward()
    got = _flat_to_dict(grad.cpu(), NOBS)
    for k in mo.KEYS:
        ref = wg[k].grad
        err = float((got[k] - ref).norm() / max(float(ref.norm()), 1e-12))
        assert err < 2e-4, (k, err)


def _set_env(store, B, n, target="MIN_COVER"):
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import MAIN_OBSERVABLES, ExtraAction, OptimisationTarget, RewardSignal
    return VecSpinSystem(store, B, 2 * n, want_f64=True, observables=MAIN_OBSERVABLES,
                         reward_signal=RewardSignal.BLS, extra_action=ExtraAction.NONE,
                         optimisation_target=OptimisationTarget[target], norm_rewards=True, basin_reward=1. / n,
                         reversible_spins=True)


@pytest.mark.parametrize("target", ["MIN_COVER", "MAX_CLIQUE", "MIN_DOM_SET"])
def test_env_features_feed_the_wide_mpnn(target):
    """obs_x of the generic-scorer env (16-float rows) through the MPNN = oracle on the float64 rows."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_GRAPH
    n, B = 40, 8
    store = GraphStore.random("ER", B, n, 0.2, seed=5, weights="uniform")
    env = _set_env(store, B, n, target)
    env.reset(graph_ids=np.arange(B), seed=3)
    rng = np.random.default_rng(1)
    for _ in range(5):
        env.step(torch.tensor(rng.integers(0, n, B), dtype=torch.int32, device="cuda"))
    env.check_errors()
    w = _weights(NOBS, 11, std=0.05)
    net = MPNN(n_obs_in=NOBS, device="cuda")
    net.load_state_dict(w)
    q = net.forward_graphs(env.obs_x, store, env.graph_ids, norm_scope=ECO_NORM_PER_GRAPH).cpu()
    rows = env.obs_f64.cpu().numpy()
    for b in range(B):
        obs = torch.from_numpy(np.vstack([rows[b], store.dense(b)])).float()
        assert _scaled_err(q[b], mo.forward(w, obs, n_obs_in=NOBS)) <= 5e-5, b


@pytest.mark.parametrize("target", ["MIN_COVER", "MAX_IND_SET"])
def test_learn_set_problem_main_observables(target):
    """A short batched learn() run of the reference's ECO configuration for a set problem
    (experiments/train_eco.py:245-305: MAIN_OBSERVABLES, BLS, basin reward 1/N, UNIFORM graphs)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    n, B = 20, 256
    store = GraphStore.random("ER", 1024, n, 0.15, seed=4, weights="uniform")
    env = _set_env(store, B, n, target)
    agent = DQN(env, lambda: MPNN(n_obs_in=NOBS, device="cuda"), init_weight_std=0.01, double_dqn=True,
                clip_Q_targets=False, replay_start_size=2 * B, replay_buffer_size=4096, gamma=0.95,
                update_target_frequency=500, update_learning_rate=False, initial_learning_rate=1e-4,
                peak_learning_rate=1e-4, final_learning_rate=1e-4, update_frequency=32, minibatch_size=64,
                final_exploration_rate=0.05, final_exploration_step=150000, adam_epsilon=1e-8, seed=3,
                train_minibatch=128)
    w0 = agent.network.flat.clone()
    losses = agent.learn(timesteps=B * 2 * n * 3)
    assert agent.grad_steps > 0 and len(losses) > 0
    assert all(np.isfinite(l) for _, l in losses)
    assert not torch.equal(w0, agent.network.flat)
    assert torch.isfinite(agent.network.flat).all()
