"""Shared harness of the training-quality pins (not a test module): bench.build_train_agent -- the benched agent,
fresh graphs per episode -- trained with DQN.learn() for the reference's 10 M env-steps, the network selected by
learn()'s own `_best` evaluation on 50 held-out validation graphs at the reference cadence (every 50 k env-steps,
BEST metric: /root/reference/src/agents/dqn/dqn.py:349-361, experiments/train_eco.py:368-377), then rolled out
greedily on 50 separate test graphs beside the reference's pretrained network for that family."""
import os
import sys
import tempfile
import time

import numpy as np
import torch

from conftest import REPO

N_GRAPHS = 50


@torch.no_grad()
def best_cuts(net, graphs, attempts, seed, basis, n):
    """Greedy rollouts of `net` (T = 2N, fused argmax, norm.max() per graph) of `attempts` episodes per graph from
    seeded random spins: per graph the best cut over the attempts."""
    from eco_hip import _lib
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    G = len(graphs)
    store = GraphStore.from_dense(graphs)
    env = VecSpinSystem(store, G * attempts, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis[basis], norm_rewards=True, basin_reward=1. / n)
    spins = 2 * np.random.default_rng(seed).integers(0, 2, (G * attempts, n)) - 1
    env.reset(graph_ids=np.tile(np.arange(G), attempts), spins=spins)
    acts = torch.empty(env.n_envs, dtype=torch.int32, device="cuda")
    greedy = _lib.ActConfig(0.0, 1, 0.0, 0, 0)
    for _ in range(env.max_steps):
        net.forward_graphs(env.obs_x, store, env.graph_ids, norm_scope=_lib.ECO_NORM_PER_GRAPH, act=greedy,
                           actions_out=acts)
        env.step(acts)
    env.check_errors()
    return env.read()["best_solution"].cpu().numpy().reshape(attempts, G).max(0)


def family_graphs(kind, n, seed):
    from oracle import graphs as og
    rng = np.random.default_rng(seed)
    if kind == "ER":
        return [og.er_graph(n, 0.15, rng) for _ in range(N_GRAPHS)]
    return [og.ba_graph(n, 4, rng) for _ in range(N_GRAPHS)]


def train_and_select(kind, param, n, seed, steps=10_000_000, B=8192, M=2048, configure=None, replay_episodes=None):
    """The benched agent trained by learn(); returns (the `_best` network, info).  configure: optional callable on
    the agent before training (tools/r06/quality_sweep.py); replay_episodes: the replay ring in episode batches of
    B x T transitions (default: bench.REPLAY_EPISODES, the benched ring)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.utils import TestMetric
    sys.path.insert(0, REPO)
    import bench
    dev = torch.device("cuda", 0)
    agent, _, env, lr = bench.build_train_agent(dev, B, n, kind, param, M, seed=seed,
                                                 **({} if replay_episodes is None else
                                                    {"replay_episodes": replay_episodes}))
    val = VecSpinSystem(GraphStore.from_dense(family_graphs(kind, n, 9000 + (kind == "BA"))), 64, 2 * n,
                        **env.env_args)
    tmp = tempfile.mkdtemp(prefix=f"eco_quality_{kind}{n}_{seed}_")
    agent.evaluate, agent.test_envs, agent.test_episodes = True, val, N_GRAPHS
    agent.test_frequency, agent.test_metric = 50_000, TestMetric.BEST
    agent.network_save_path = os.path.join(tmp, "net.pth")
    agent.test_save_path = os.path.join(tmp, "test_scores")
    agent.save_network_frequency = 10 ** 12
    if configure is not None:
        configure(agent)
    t0 = time.perf_counter()
    agent.learn(timesteps=steps)
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    agent.env.check_errors()
    best = MPNN(device="cuda")
    best.load_state_dict(torch.load(os.path.join(tmp, "net_best.pth"), map_location="cpu", weights_only=True))
    scores = np.array([s for _, s in agent.test_scores])
    info = {"seed": seed, "lr": lr, "steps": agent._timestep, "grad_steps": agent.grad_steps, "train_s": secs,
            "evaluations": len(scores), "best_val": float(scores.max()), "best_at": int(agent.test_scores[
                int(np.argmax(scores))][0]), "graphs_regenerated": agent.graphs_regenerated,
            "graphs_reused": agent.graphs_reused, "final_net": agent.network}
    return best, info


def pretrained(npz, prefix):
    from oracle import mpnn_oracle as mo
    from eco_hip.networks.mpnn import MPNN
    f = np.load(npz)
    net = MPNN(device="cuda")
    net.load_state_dict({k: torch.from_numpy(f[prefix + k]) for k in mo.KEYS})
    return net
