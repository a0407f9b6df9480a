"""Two ranks on one GPU (gloo): the wall time an overlapped evaluation adds to 8 vector steps of training, with the
rollout replayed from its HIP graph (learn()'s default) and with eager launches, and 8 vector steps alone.
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/r06/ov_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    torch.distributed.init_process_group(os.environ.get("OV_BACKEND", "gloo"))
    dev = torch.device("cuda", 0)
    B, n = 8192, 200
    agent, store, env, lr = bench.build_train_agent(dev, B, n, "ER", 0.15, 2048, 1234 + rank, spare_batches=1)
    agent.start()
    for _ in range(5):
        agent.iteration()
    test = bench.make_test_env(agent, dev)
    from eco_hip.agents.dqn.utils import TestMetric
    agent.test_envs, agent.test_episodes, agent.test_metric = test, test.graphs.n_graphs, TestMetric.BEST

    def run(ov, k=8):
        torch.cuda.synchronize()
        torch.distributed.barrier()
        t0 = time.perf_counter()
        p = agent._evaluate_overlapped(0) if ov else None
        t1 = time.perf_counter()
        for _ in range(k):
            agent.iteration()
        t2 = time.perf_counter()
        if p is not None:
            agent._eval_one_fill_finish(p)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        return [round((t - t0) * 1e3, 1) for t in (t1, t2, t3)]

    for graphs in (True, False):
        agent.eval_graphs = graphs
        agent._eval_graphs.clear()
        for _ in range(2):
            agent._eval_one_fill_finish(agent._evaluate_overlapped(0))
        for ov in (False, True, False, True):
            r = run(ov)
            if rank == 0:
                print(f"eval_graphs={graphs} overlapped={ov}: launch / 8 iterations issued / done (ms) {r}", flush=True)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
