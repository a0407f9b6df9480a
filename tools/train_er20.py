"""Training-quality probe (VERDICT r02 "missing" #1): batched DQN.learn on ER(20, 0.15) +-1 graphs, fresh
graphs per episode generated on the device, evaluated every --eval-every env-steps on the 50 graphs of
tests/golden/er20_opt.npz (exact optima) by one greedy episode per graph from seeded random spins (the
reference's evaluate_agent with TestMetric.BEST, dqn.py:514-602), reported as mean best cut / mean optimum.

    python tools/train_er20.py --envs 64 --minibatch 64 --lr 1e-4 --steps 1000000
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "eco-dqn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def make_agent(B, M, lr, seed, n=20, lr_final=None, target_freq=1000, capacity=None, eps_step=150000,
               target_sync="grad_steps"):
    from eco_hip.graphs import GraphStore, edge_cap
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN, graph_slots_needed
    T = 2 * n
    C = capacity or max(5000, 2 * B * T)
    st = GraphStore.slots(graph_slots_needed(B, T, C), n, edge_cap("ER", n, 0.15))
    env = VecSpinSystem(st, B, T, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    # experiments/train_eco.py:114-161 with the ER_20 dqn_params (:338-347)
    return DQN(env, lambda: MPNN(device="cuda"), init_weight_std=0.01, double_dqn=True, clip_Q_targets=False,
               replay_start_size=500, replay_buffer_size=C, gamma=0.95, update_target_frequency=target_freq,
               update_learning_rate=lr_final is not None, initial_learning_rate=lr, peak_learning_rate=lr,
               peak_learning_rate_step=1, final_learning_rate=lr_final if lr_final is not None else lr,
               final_learning_rate_step=10 ** 6, update_frequency=32, minibatch_size=64, train_minibatch=M,
               initial_exploration_rate=1, final_exploration_rate=0.05, final_exploration_step=eps_step,
               adam_epsilon=1e-8, seed=seed, evaluate=False, test_save_path=None, regenerate_graphs=("ER", 0.15),
               target_sync=target_sync)


class Evaluator:
    """One greedy episode (T = 2N, fused argmax, BEST metric) per test graph from fixed random spins."""

    def __init__(self, path=None, attempts=1, seed=0):
        from eco_hip.graphs import GraphStore
        from eco_hip.envs.batched import VecSpinSystem
        from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                        SpinBasis)
        f = np.load(path or os.path.join(REPO, "tests", "golden", "er20_opt.npz"))
        self.opt = f["opt_cut"]
        G, n = f["graphs"].shape[:2]
        self.G, self.n, self.attempts = G, n, attempts
        self.store = GraphStore.from_dense([g.astype(np.float64) for g in f["graphs"]])
        B = G * attempts
        self.env = VecSpinSystem(self.store, B, 2 * n, observables=DEFAULT_OBSERVABLES,
                                 reward_signal=RewardSignal.BLS, extra_action=ExtraAction.NONE,
                                 optimisation_target=OptimisationTarget.CUT, spin_basis=SpinBasis.SIGNED,
                                 norm_rewards=True, basin_reward=1. / n)
        rng = np.random.default_rng(seed)
        self.spins = 2 * rng.integers(0, 2, (B, n)) - 1
        self.gids = np.tile(np.arange(G), attempts)

    @torch.no_grad()
    def __call__(self, net):
        from eco_hip import _lib
        env = self.env
        env.reset(graph_ids=self.gids, spins=self.spins)
        acts = torch.empty(env.n_envs, dtype=torch.int32, device="cuda")
        greedy = _lib.ActConfig(0.0, 1, 0.0, 0, 0)
        for _ in range(env.max_steps):
            net.forward_graphs(env.obs_x, self.store, env.graph_ids, norm_scope=_lib.ECO_NORM_PER_CALL,
                               act=greedy, actions_out=acts)
            env.step(acts)
        best = env.read()["best_solution"].cpu().numpy().reshape(self.attempts, self.G).max(0)
        return float(best.mean() / self.opt.mean()), float((best / self.opt).mean()), float((best == self.opt).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--minibatch", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--lr-final", type=float, default=None)
    ap.add_argument("--target-freq", type=int, default=1000)
    ap.add_argument("--eps-step", type=int, default=150000)
    ap.add_argument("--steps", type=int, default=1000000)
    ap.add_argument("--eval-every", type=int, default=100000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--target-sync", default="grad_steps", choices=["grad_steps", "samples"])
    a = ap.parse_args()
    agent = make_agent(a.envs, a.minibatch, a.lr, a.seed, lr_final=a.lr_final, target_freq=a.target_freq,
                       eps_step=a.eps_step, target_sync=a.target_sync)
    ev = Evaluator()
    ev50 = Evaluator(attempts=50, seed=1)
    curve = [(0, *ev(agent.network))]
    t0 = time.time()
    nxt = [a.eval_every]

    def hook(t):
        if t >= nxt[0]:
            nxt[0] += a.eval_every
            r = ev(agent.network)
            curve.append((t, *r))
            print(json.dumps({"t": t, "ratio_of_means": r[0], "mean_ratio": r[1], "frac_opt": r[2],
                              "grad_steps": agent.grad_steps, "eps": agent.epsilon,
                              "wall_s": round(time.time() - t0, 1)}), flush=True)
    agent.learn(a.steps, on_vector_step=hook)
    torch.cuda.synchronize()
    r50 = ev50(agent.network)
    res = {"envs": a.envs, "minibatch": a.minibatch, "lr": a.lr, "lr_final": a.lr_final, "steps": a.steps,
           "target_sync": a.target_sync,
           "grad_steps": agent.grad_steps, "wall_s": time.time() - t0, "curve": curve,
           "final_1attempt": curve[-1][1:], "final_50attempts": r50}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh)


if __name__ == "__main__":
    main()
