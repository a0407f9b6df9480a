"""One rank of tests/test_rccl_gpu.py (not a test module): torch.distributed over the nccl backend (RCCL on ROCm)
with world size 1 on GPU 0 -- the backend the driver's multi-GPU bench uses, on the one-GPU box.  Runs the
collectives DQN uses on device tensors (all_reduce sync and async + work.wait() stream ordering, broadcast,
MAX all-reduce of bench.py's timing) and two DQN.learn() vector-step iterations inside the process group.
Prints RCCL_OK <backend> <world>."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "eco-dqn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    dev = torch.device("cuda", 0)
    g = torch.arange(58425, dtype=torch.float32, device=dev)
    dist.all_reduce(g)
    w = dist.all_reduce(g, async_op=True)
    w.wait()  # orders the current stream behind the collective
    t = torch.tensor([1.5, -2.0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.broadcast(g, src=0)
    torch.cuda.synchronize()
    assert torch.equal(g, torch.arange(58425, dtype=torch.float32, device=dev))
    assert t.cpu().tolist() == [1.5, -2.0]
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    n, B = 20, 64
    store = GraphStore.random("ER", 128, n, 0.15, seed=3, device="cuda:0")
    env = VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    agent = DQN(env, lambda: MPNN(device="cuda:0"), init_weight_std=0.01, replay_start_size=B,
                replay_buffer_size=1024, minibatch_size=64, update_frequency=32, seed=5, evaluate=False,
                test_save_path=None)
    assert agent.dist and agent.world == 1
    agent.learn(timesteps=B * 4)
    assert agent.grad_steps > 0 and torch.isfinite(agent.network.flat).all()
    print("RCCL_OK", dist.get_backend(), dist.get_world_size(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
