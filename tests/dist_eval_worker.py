"""One rank of tests/test_parallel_gpu.py::test_two_ranks_evaluate_once_per_crossing (not a test module):
DQN.learn() with evaluations over gloo, both ranks on GPU 0.  B x world = 256 env-steps per vector step against
test_frequency = 200, so EVERY vector step crosses a test point (the regime of configs[3] at 8 GPUs).  Each
crossing must be one evaluation of the job (owner = evaluation index mod world), every rank must record the same
test scores, and the `_best` checkpoint rank 0 writes must reproduce the best recorded score when evaluated again on the graphs of
that evaluation's job-wide index.  learn()'s steady state must not synchronise the host with the device.
Rank 0 prints EVAL_OK <evaluations> <per-rank counts> <best score>."""
import os
import sys
import tempfile

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
    from eco_hip.agents.dqn.utils import TestMetric
    n, B = 20, 128
    kw = dict(observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS, extra_action=ExtraAction.NONE,
              optimisation_target=OptimisationTarget.CUT, spin_basis=SpinBasis.SIGNED, norm_rewards=True,
              basin_reward=1. / n)
    store = GraphStore.random("ER", 512, n, 0.15, seed=60 + rank, device="cuda:0")
    env = VecSpinSystem(store, B, 2 * n, **kw)
    # the same test graphs on every rank (train_eco.py's fixed test set); more graphs (25) than episodes per
    # evaluation (10), so each evaluation's graphs depend on its job-wide index (cursor0 + idx x 10 mod 25)
    test = VecSpinSystem(GraphStore.random("ER", 25, n, 0.15, seed=777, device="cuda:0"), 16, 2 * n, **kw)
    tmp = tempfile.mkdtemp(prefix=f"eco_eval_r{rank}_")
    agent = DQN(env, lambda: MPNN(device="cuda:0"), init_weight_std=0.01, double_dqn=True, replay_start_size=2 * B,
                replay_buffer_size=4096, gamma=0.95, update_target_frequency=1000, update_learning_rate=False,
                initial_learning_rate=1e-3, peak_learning_rate=1e-3, final_learning_rate=1e-3, update_frequency=32,
                minibatch_size=16, train_minibatch=128, final_exploration_rate=0.05, final_exploration_step=20000,
                seed=21 + rank, evaluate=True, test_envs=test, test_episodes=10, test_frequency=200,
                test_metric=TestMetric.BEST, test_save_path=os.path.join(tmp, "scores"),
                network_save_path=os.path.join(tmp, "net.pth"), save_network_frequency=10 ** 9)
    timesteps = B * world * 2 * n * 2
    # no host synchronisation inside learn()'s steady state: torch's sync-debug mode raises on any implicit
    # device synchronisation (item(), cpu(), blocking copies, stream / device synchronize) from the 4th vector
    # step after training is ready (the first evaluation of each rank has captured its rollout graph by then)
    # to the last one, and the device error check (eco_check_errors) must not be called meanwhile
    # gloo stages a CUDA tensor's all-reduce through the host on its own thread (a synchronisation the nccl backend
    # does not have: RCCL runs on its own stream and work.wait() only orders the streams), so this gloo rehearsal
    # runs the per-gradient-step exchange to completion with the check off; everything else learn() does is checked
    import eco_hip.agents.dqn.dqn as dqn_mod
    real_allreduce = dqn_mod.allreduce_gradients_async

    def allreduce_exempt(grad, group=None):
        mode = torch.cuda.get_sync_debug_mode()
        torch.cuda.set_sync_debug_mode(0)
        try:
            work, scale = real_allreduce(grad, group)
            if work is not None:
                work.wait()
            torch.cuda.synchronize()
        finally:
            torch.cuda.set_sync_debug_mode(mode)
        return None, scale
    dqn_mod.allreduce_gradients_async = allreduce_exempt
    steady = {"n": 0, "on": False, "checks": 0}
    real_check = agent.graphs.check_errors

    def counting_check(*a, **k):
        if steady["on"]:
            steady["checks"] += 1
        return real_check(*a, **k)
    agent.graphs.check_errors = counting_check

    def on_step(t):
        if agent._ready:
            steady["n"] += 1
        on = 4 <= steady["n"] and t < timesteps
        if on != steady["on"]:
            torch.cuda.set_sync_debug_mode("error" if on else "default")
            steady["on"] = on
    agent.learn(timesteps=timesteps, on_vector_step=on_step)
    torch.cuda.set_sync_debug_mode("default")
    assert steady["n"] > 20 and steady["checks"] == 0, steady
    # crossings of the timed loop: every vector step once training is ready
    ts = np.array([t for t, _ in agent.test_scores])
    sc = torch.tensor([s for _, s in agent.test_scores], dtype=torch.float64)
    allsc = [torch.zeros_like(sc) for _ in range(world)]
    dist.all_gather(allsc, sc)
    runs = torch.tensor([float(agent.evaluations_run)])
    allruns = [torch.zeros_like(runs) for _ in range(world)]
    dist.all_gather(allruns, runs)
    # constructed on every rank (the constructor's parameter / seed broadcasts are collective)
    chk = DQN(env, lambda: MPNN(device="cuda:0"), init_weight_std=0.01, replay_start_size=2 * B,
              replay_buffer_size=4096, minibatch_size=16, seed=21 + rank, evaluate=False, test_envs=test,
              test_episodes=10, test_metric=TestMetric.BEST, test_save_path=None)
    if rank == 0:
        assert all(torch.equal(a, allsc[0]) for a in allsc), "ranks recorded different test scores"
        assert len(ts) == len(np.unique(ts)) and np.all(np.diff(ts) > 0)
        per_vec = B * world
        first_ready = ts[0]
        expect = [t for t in range(first_ready, timesteps + 1, 200)]
        # one evaluation per vector step that crosses k * 200 (every step here): count the crossed steps
        steps = np.arange(per_vec, timesteps + 1, per_vec)
        crossed = [t for t in steps if t // 200 > (t - per_vec) // 200 and t >= first_ready]
        assert len(ts) == len(crossed), (len(ts), len(crossed), len(expect))
        counts = [int(r.item()) for r in allruns]
        assert sum(counts) == len(ts) and max(counts) - min(counts) <= 1, counts
        # the _best checkpoint reproduces the best score (evaluation seed = rank 0's on every rank)
        best = float(sc.max())
        chk.load(os.path.join(tmp, "net_best.pth"))
        i_best = int(np.argmax(sc.numpy()))  # first occurrence = the evaluation that saved _best
        test._eval_next_graph = (i_best * 10) % 25
        again, _ = chk.evaluate_agent()
        assert again == best, (again, best)
        print("EVAL_OK", len(ts), counts, best, flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
