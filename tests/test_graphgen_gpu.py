"""On-device ER/BA graph generation: structural invariants, distribution
(parity is distributional: the reference draws from numpy/networkx streams), determinism, and
that generated graphs drive the env exactly like the oracle on their dense copies."""
import numpy as np
import pytest
import torch

from oracle import spinsystem_oracle as so

pytestmark = pytest.mark.gpu


def _check_structure(store, g):
    J = store.dense(g)
    assert np.array_equal(J, J.T) and not np.diag(J).any()
    rp = store.row_ptr[g].cpu().numpy()
    b = int(store.edge_base[g].item())
    cols = (store.edges[b:b + rp[-1]].cpu().numpy().view(np.uint32) & 0xFFFFFF).astype(np.int64)
    for i in range(J.shape[0]):      # rows sorted, no duplicates
        row = cols[rp[i]:rp[i + 1]]
        assert np.all(np.diff(row) > 0)
    return J


def test_er_generation_statistics_and_determinism():
    from eco_hip.graphs import GraphStore
    n, p, G = 200, 0.15, 256
    st = GraphStore.generated("ER", G, n, p, seed=3)
    st.generate(0, 1, "ER", p, seed=3)            # regenerate in place: same seed, same graph
    nnz = np.diff(st.row_ptr.cpu().numpy(), axis=1).sum(1)
    pairs = n * (n - 1) / 2
    assert abs(nnz.mean() / 2 - p * pairs) < 4 * np.sqrt(p * (1 - p) * pairs / G)
    J0 = _check_structure(st, 0)
    st2 = GraphStore.generated("ER", 4, n, p, seed=3)
    np.testing.assert_array_equal(J0, st2.dense(0))
    w = np.concatenate([st.dense(g)[np.triu_indices(n, 1)] for g in range(8)])
    w = w[w != 0]
    assert set(np.unique(w)) == {-1.0, 1.0} and abs((w > 0).mean() - 0.5) < 0.02
    assert int(st.valid.sum().item()) == G


def test_ba_generation_structure():
    from eco_hip.graphs import GraphStore
    n, m, G = 500, 4, 64
    st = GraphStore.generated("BA", G, n, m, seed=9, weights="uniform")
    nnz = np.diff(st.row_ptr.cpu().numpy(), axis=1).sum(1)
    assert np.all(nnz == 2 * m * (n - m))
    J = _check_structure(st, 5)
    deg = (J != 0).sum(1)
    assert deg[m:].min() >= m and deg.max() > 5 * m          # preferential attachment hubs
    assert set(np.unique(J)) <= {0.0, 1.0}


def test_generated_graphs_drive_env_like_oracle():
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    n, B = 60, 32
    st = GraphStore.generated("BA", B, n, 4, seed=1)
    env = VecSpinSystem(st, B, 2 * n, want_f64=True, observables=DEFAULT_OBSERVABLES,
                        reward_signal=RewardSignal.BLS, extra_action=ExtraAction.NONE,
                        optimisation_target=OptimisationTarget.CUT, spin_basis=SpinBasis.SIGNED,
                        norm_rewards=True, basin_reward=1. / n)
    rng = np.random.default_rng(0)
    spins = 2 * rng.integers(0, 2, (B, n)) - 1
    env.reset(graph_ids=np.arange(B), spins=spins)
    o = so.SpinSystemOracle(st.dense(7), 2 * n, basin_reward=1. / n)
    o.reset(spins=spins[7])
    for t in range(2 * n):
        a = rng.integers(0, n, B)
        _, r, _ = env.step(torch.from_numpy(a).to(torch.int32).cuda())
        _, orew, _, _ = o.step(int(a[7]))
        assert r[7].item() == orew
    np.testing.assert_array_equal(env.obs_f64[7].cpu().numpy().view(np.uint64), o.state_rows().view(np.uint64))


def test_learn_with_fresh_graphs_per_episode():
    from eco_hip.graphs import GraphStore, edge_cap
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    n, B = 20, 128
    st = GraphStore.slots(2 * B, n, edge_cap("ER", n, 0.15))
    env = VecSpinSystem(st, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    agent = DQN(env, lambda: MPNN(device="cuda"), init_weight_std=0.01, gamma=0.95, replay_start_size=256,
                replay_buffer_size=B * 2 * n, update_target_frequency=500, update_learning_rate=False,
                initial_learning_rate=1e-4, update_frequency=32, minibatch_size=64, train_minibatch=128,
                regenerate_graphs=("ER", 0.15), seed=2)
    agent.learn(timesteps=B * 2 * n * 3)
    env.check_errors()
    assert agent.grad_steps > 0 and torch.isfinite(agent.network.flat).all()
