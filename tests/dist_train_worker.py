"""One rank of tests/test_parallel_gpu.py (not a test module): the sharded DQN training path
on the GPU -- each rank its own graph pool, env batch, replay and seed; one gradient all-reduce per
optimiser step (eco_hip.parallel.allreduce_gradients) -- over gloo with every rank on GPU 0 (a one-GPU
box rehearsal of the RCCL path).  Rank 0 prints one line: DIST_OK <grad steps> <max |w_r - w_0|> ...
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "eco-dqn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    n, B = 20, 128
    store = GraphStore.random("ER", 512, n, 0.15, seed=40 + rank, device="cuda:0")
    env = VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    agent = DQN(env, lambda: MPNN(device="cuda:0"), init_weight_std=0.01, double_dqn=True, clip_Q_targets=False,
                replay_start_size=2 * B, replay_buffer_size=4096, gamma=0.95, update_target_frequency=1000,
                update_learning_rate=False, initial_learning_rate=1e-4, peak_learning_rate=1e-4,
                final_learning_rate=1e-4, update_frequency=32, minibatch_size=64, train_minibatch=128,
                final_exploration_rate=0.05, final_exploration_step=150000, adam_epsilon=1e-8, seed=11 + rank,
                evaluate=False, test_save_path=None)
    w0 = agent.network.flat.clone()
    all0 = [torch.zeros_like(w0) for _ in range(world)]
    dist.all_gather(all0, w0)
    agent.learn(timesteps=B * world * 2 * n * 2)
    w = agent.network.flat.clone()
    allw = [torch.zeros_like(w) for _ in range(world)]
    dist.all_gather(allw, w)
    steps = torch.tensor([float(agent.grad_steps)], device="cuda:0")
    alls = [torch.zeros_like(steps) for _ in range(world)]
    dist.all_gather(alls, steps)
    if rank == 0:
        init_same = max(float((a - all0[0]).abs().max()) for a in all0)
        diff = max(float((a - allw[0]).abs().max()) for a in allw)
        moved = float((allw[0] - all0[0]).abs().max())
        print("DIST_OK", int(agent.grad_steps), diff, init_same, moved, [int(s) for s in alls],
              bool(torch.isfinite(w).all()), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
