"""Training quality of the batched DQN.learn (SURVEY.md 8a D3's statistical pin; VERDICT r02 "missing" #1).

The reference trains ECO-DQN on ER(20, 0.15) +-1 graphs (experiments/train_eco.py:114-169, 255-264, 338-347) and
reaches a mean best cut of ~10.57 on its ER_20 test graphs against a best-known mean of 10.68
(ER_20spin/eco/max_cut/network/training_curve.png): a ratio of ~0.99.  Here the batched learn() trains on fresh
device-generated ER(20, 0.15) graphs per episode (regenerate_graphs) with the reference's hyper-parameters and is
evaluated on the 50 seeded graphs of tests/golden/er20_opt.npz, whose optima are exact (2^19 enumeration,
tests/golden/make_er20_opt.py): one greedy episode (T = 2N, BEST metric, dqn.py:514-602) per graph from seeded
random spins, scored as mean best cut / mean optimum; and the best of 50 such attempts per graph (test_network's
batched multi-attempt search, experiments/utils.py:33-303).

  * reference-like: 64 episodes, minibatch 64, lr 1e-4 (the reference's replay ratio 64/32 and its step counts);
  * the bench's minibatch-to-episode ratio (M = B/4): 2048 episodes, minibatch 512, with the large-batch recipe:
    target sync every update_target_frequency / update_frequency GRADIENT steps (dqn.py:332-347 at M = 64;
    target_sync="grad_steps") and lr scaled by sqrt(M / 64).  Syncing per env-step's worth of samples instead
    re-targets every ~4 gradient steps at M = 512 and measured 0.965-0.98.
Bar: >= 0.98 single attempt (the reference ~0.99), >= 0.995 best of 50."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _agent(B, M, lr, seed):
    from eco_hip.graphs import GraphStore, edge_cap
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN, graph_slots_needed
    n = 20
    T = 2 * n
    C = max(5000, 2 * B * T)
    st = GraphStore.slots(graph_slots_needed(B, T, C), n, edge_cap("ER", n, 0.15))
    env = VecSpinSystem(st, B, T, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    return DQN(env, lambda: MPNN(device="cuda"), init_weight_std=0.01, double_dqn=True, clip_Q_targets=False,
               replay_start_size=500, replay_buffer_size=C, gamma=0.95, update_target_frequency=1000,
               update_learning_rate=False, initial_learning_rate=lr, peak_learning_rate=lr, final_learning_rate=lr,
               update_frequency=32, minibatch_size=64, train_minibatch=M, initial_exploration_rate=1,
               final_exploration_rate=0.05, final_exploration_step=150000, adam_epsilon=1e-8, seed=seed,
               evaluate=False, test_save_path=None, regenerate_graphs=("ER", 0.15), target_sync="grad_steps")


@torch.no_grad()
def _evaluate(net, attempts, seed):
    from eco_hip import _lib
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    f = np.load(os.path.join(GOLDEN, "er20_opt.npz"))
    G, n = f["graphs"].shape[:2]
    store = GraphStore.from_dense([g.astype(np.float64) for g in f["graphs"]])
    env = VecSpinSystem(store, G * attempts, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    spins = 2 * np.random.default_rng(seed).integers(0, 2, (G * attempts, n)) - 1
    env.reset(graph_ids=np.tile(np.arange(G), attempts), spins=spins)
    acts = torch.empty(env.n_envs, dtype=torch.int32, device="cuda")
    greedy = _lib.ActConfig(0.0, 1, 0.0, 0, 0)
    for _ in range(env.max_steps):
        net.forward_graphs(env.obs_x, store, env.graph_ids, norm_scope=_lib.ECO_NORM_PER_CALL, act=greedy,
                           actions_out=acts)
        env.step(acts)
    env.check_errors()
    best = env.read()["best_solution"].cpu().numpy().reshape(attempts, G).max(0)
    return float(best.mean() / f["opt_cut"].mean())


@pytest.mark.parametrize("B,M,lr,steps", [(64, 64, 1e-4, 400_000), (2048, 512, 1e-4 * (512 / 64) ** 0.5, 1_000_000)])
def test_learn_reaches_reference_quality_on_er20(B, M, lr, steps):
    agent = _agent(B, M, lr, seed=1)
    before = _evaluate(agent.network, 1, seed=0)
    agent.learn(timesteps=steps)
    agent.env.check_errors()
    one = _evaluate(agent.network, 1, seed=0)
    fifty = _evaluate(agent.network, 50, seed=1)
    print(f"B={B} M={M} lr={lr:.2e}: {agent.grad_steps} gradient steps; mean best / mean optimum "
          f"{before:.3f} untrained -> {one:.3f} (1 attempt), {fifty:.3f} (best of 50)")
    assert agent.graphs_reused == 0
    assert one >= 0.98, one
    assert fifty >= 0.995, fifty
    assert before < 0.5  # the untrained network is far from it: the bar measures learning
