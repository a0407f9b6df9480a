#!/usr/bin/env python
"""Benchmark: env-steps/sec (batched episodes) on ER-200 MaxCut (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload rollout|train] [--envs B]

One "step" = one vector step over B=8192 concurrent ER-200 episodes (each on its own
graph): MPNN forward + fused epsilon-greedy act + env step, all on the GPU
(workload "rollout"); "train" adds the DQN update (replay + TD + backward + Adam)
once it is available.  value = B * K * world / max-over-ranks(time).  Episodes
shard across ranks with no data-path collective (scaling "weak").

Prints ONE JSON line on rank 0 with roofline (dominant kernel: mpnn_forward,
MFMA-bound) and cpu_baseline (oracle = reference-cost numpy restatement of
SpinSystem.step + torch-CPU MPNN forward, timed on this host on a bounded sample).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "eco-dqn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32-input MFMA peak


def mpnn_flops(nnz, n):
    """algorithmic forward FLOPs of one graph = 1392*nnz + 107,648*N + 8,192."""
    return 1392.0 * nnz + 107648.0 * n + 8192.0


def cpu_baseline(n=200, seconds=12.0):
    """Oracle (CPU 'port') env + MPNN forward, B=1 greedy act (dqn.py:282 path), ER-200."""
    sys.path.insert(0, REPO)
    from oracle import spinsystem_oracle as so
    from oracle import mpnn_oracle as mo
    from oracle import graphs as og
    rng = np.random.default_rng(0)
    w = mo.init_weights(torch.Generator().manual_seed(0), std=0.01)
    steps = 0
    t0 = time.perf_counter()
    with torch.no_grad():
        while time.perf_counter() - t0 < seconds:
            J = og.er_graph(n, 0.15, rng)
            env = so.SpinSystemOracle(J, 2 * n, basin_reward=1. / n)
            obs = env.reset(rng=np.random.RandomState(int(rng.integers(1 << 31))))
            done = False
            while not done and time.perf_counter() - t0 < seconds:
                q = mo.forward(w, torch.from_numpy(obs).float())
                obs, _, done, _ = env.step(int(q.argmax()))
                steps += 1
    dt = time.perf_counter() - t0
    return dict(value=steps / dt, unit="env-steps/s", cores=torch.get_num_threads(), kind="port",
                sample=f"{steps} ER-200 env-steps (oracle SpinSystem.step + torch-CPU MPNN fwd, B=1 greedy), "
                       f"{dt:.1f}s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--workload", default="rollout", choices=["rollout"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl")
    dev = torch.device("cuda", local)

    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ActConfig

    B, n = args.envs, args.n
    T = 2 * n
    seed = 1234 + rank
    store = GraphStore.random("ER", B, n, 0.15, seed=seed, device=dev)
    nnz = np.diff(store.row_ptr.cpu().numpy(), axis=1).sum(axis=1)
    flops_per_fwd = float(sum(mpnn_flops(z, n) for z in nnz))
    env = VecSpinSystem(store, B, T, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    net = MPNN(device=dev)
    net.init_normal_(0.01, generator=torch.Generator().manual_seed(seed))
    gids = torch.arange(B, dtype=torch.int32, device=dev)
    actions = torch.zeros(B, dtype=torch.int32, device=dev)
    q = torch.empty(B, n, dtype=torch.float32, device=dev)
    x = env.reset(graph_ids=gids, seed=seed)
    counter = [0]

    def vec_step():
        # epsilon from the C3 schedule mid-way (dqn.py:467-471): greedy with prob 1-eps
        counter[0] += 1
        act = ActConfig(0.05, 1, 0.0, seed, counter[0])
        net.forward_graphs(x, store, gids, q_out=q, act=act, actions_out=actions)
        env.step(actions)
        if counter[0] % T == 0:  # all episodes finish together (same T): reset on new spins
            env.reset(graph_ids=gids, seed=seed + counter[0])

    for _ in range(args.warmup):
        vec_step()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        counter[0] += 1
        act = ActConfig(0.05, 1, 0.0, seed, counter[0])
        ev[i][0].record()
        net.forward_graphs(x, store, gids, q_out=q, act=act, actions_out=actions)
        ev[i][1].record()
        env.step(actions)
        if counter[0] % T == 0:
            env.reset(graph_ids=gids, seed=seed + counter[0])
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()
    fwd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    achieved = flops_per_fwd / (fwd_ms * 1e-3) / 1e12
    value = B * args.steps * world / dt
    if rank == 0:
        out = {
            "metric": "env-steps/sec (batched episodes) on ER-200 MaxCut",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (MPNN, exact-f32 MFMA) / f64+int (env)",
            "data": "synthetic: seeded ER(200, p=0.15) +-1 graphs, one per episode; random-init MPNN",
            "config": {"workload": "ER_200spin x8192 envs/GPU: MPNN fwd + eps-greedy act + env step "
                                   "(rollout half of configs[2]; DQN update not yet in the timed step)",
                       "n_spins": n, "envs_per_gpu": B, "max_steps": T, "parallelism": f"episodes sharded dp{world}"},
            "roofline": {"bound": "mfma", "kernel": "mpnn_forward_kernel", "achieved": achieved,
                         "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                         "traffic": None, "fwd_ms": fwd_ms,
                         "flops_per_launch": flops_per_fwd},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(n)
        print(json.dumps(out))
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
