"""One rank of tests/test_parallel_gpu.py (not a test module): the sharded DQN training path
on the GPU -- each rank its own graph pool, env batch, replay and seed; one gradient all-reduce per
optimiser step (eco_hip.parallel.allreduce_gradients) -- over gloo with every rank on GPU 0 (a one-GPU
box rehearsal of the RCCL path).  Rank 0 prints one line: DIST_OK <grad steps> <max |w_r - w_0|> ...

For the first gradient steps the worker also checks the exchange itself: every rank's LOCAL gradient is
all-gathered before allreduce_gradients runs; afterwards the reduced buffer must equal the rank-order fp32
sum of those locals bitwise, the returned scale must be 1/world, and the Adam kernel's first moment must
have moved by (1 - beta1) x (mean gradient - m): Adam is nearly invariant to a constant gradient scale, so
its weights alone could not reveal a missing average, but its moment estimate does.  Rank 0 prints
EXCHANGE_OK <steps checked> <max rel error of m>.
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
    import eco_hip.agents.dqn.dqn as dqn_mod
    real_allreduce = dqn_mod.allreduce_gradients_async
    rec = {"checked": 0, "m_err": 0.0}

    def spy_allreduce(grad, group=None):
        locals_ = [torch.zeros_like(grad) for _ in range(world)]
        dist.all_gather(locals_, grad)                         # every rank's local gradient, rank order
        work, scale = real_allreduce(grad, group)
        assert work is not None, "no collective was started"
        work.wait()
        total = locals_[0].clone()
        for g in locals_[1:]:
            total += g
        assert torch.equal(grad, total), "all-reduced gradient != rank-order sum of the local gradients"
        assert scale == 1.0 / world, scale
        rec["mean"] = total * scale
        return None, scale   # already complete
    dqn_mod.allreduce_gradients_async = spy_allreduce
    real_train_step = agent.train_step

    def spy_train_step(tr, sync_loss=True, loss_out=None, overlap=None):
        if rec["checked"] >= 3:
            return real_train_step(tr, sync_loss=sync_loss, loss_out=loss_out, overlap=overlap)
        m0 = agent.exp_avg.clone()
        out = real_train_step(tr, sync_loss=sync_loss, loss_out=loss_out, overlap=overlap)
        expect = m0 + 0.1 * (rec["mean"] - m0)               # adam_kernel: m + (1 - b1)(g * scale - m)
        scale_ = m0.abs() + 0.1 * rec["mean"].abs() + 1e-30   # error relative to the terms (no cancellation)
        err = float(((agent.exp_avg - expect).abs() / scale_).max())
        assert err < 1e-5, ("Adam's input is not the mean gradient", err)
        rec["m_err"] = max(rec["m_err"], err)
        rec["checked"] += 1
        return out
    agent.train_step = spy_train_step
    agent.learn(timesteps=B * world * 2 * n * 2)
    dqn_mod.allreduce_gradients_async = real_allreduce
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
        print("EXCHANGE_OK", rec["checked"], rec["m_err"], flush=True)
        print("DIST_OK", int(agent.grad_steps), diff, init_same, moved, [int(s) for s in alls],
              bool(torch.isfinite(w).all()), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
