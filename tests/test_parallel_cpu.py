"""World-size-2 gloo tests of the multi-GPU plumbing (eco_hip/parallel.py) on CPU:
gradient sum + mean scale, parameter broadcast, max-over-ranks timing, best-cut
selection, and that two ranks applying the same averaged Adam update stay identical."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from eco_hip.parallel import (allreduce_gradients, allreduce_gradients_async, broadcast_parameters,
                                      max_over_ranks, best_cut_over_ranks, rank_seed)
        # gradient all-reduce: sum, scale 1/world
        g = torch.full((58425,), float(rank + 1))
        scale = allreduce_gradients(g)
        assert scale == 1.0 / world
        assert torch.all(g == sum(range(1, world + 1)))
        # the overlapped form (DQN.train_step): start, independent work, wait -> the same sum
        g2 = torch.full((58425,), float(10 * (rank + 1)))
        work, scale2 = allreduce_gradients_async(g2)
        other = torch.arange(1000.0).sum()   # independent work while the collective runs
        assert work is not None and scale2 == 1.0 / world and float(other) == 499500.0
        work.wait()
        assert torch.all(g2 == 10 * sum(range(1, world + 1)))
        # parameter broadcast from rank 0
        p = torch.randn(58425, generator=torch.Generator().manual_seed(rank_seed(7, rank)))
        broadcast_parameters(p)
        ref = torch.randn(58425, generator=torch.Generator().manual_seed(rank_seed(7, 0)))
        assert torch.equal(p, ref)
        # identical averaged Adam step on every rank (the eco_adam formula, fp32)
        grad = torch.randn(58425, generator=torch.Generator().manual_seed(100 + rank))
        s = allreduce_gradients(grad)
        m = torch.zeros_like(p); v = torch.zeros_like(p)
        gi = grad * s
        m = m + 0.1 * (gi - m)
        v = v * 0.999 + 0.001 * gi * gi
        p2 = p - (1e-4 / 0.1) * (m / (v.sqrt() / (0.001 ** 0.5) + 1e-8))
        allp = [torch.zeros_like(p2) for _ in range(world)]
        dist.all_gather(allp, p2)
        assert all(torch.equal(allp[0], x) for x in allp)
        # timing: max over ranks
        assert max_over_ranks(1.0 + rank) == float(world)
        # best cut: highest cut wins, its spins are broadcast
        cut = [10.0, 12.0][rank]
        spins = torch.full((20,), float(rank), dtype=torch.float64)
        bc, bs = best_cut_over_ranks(cut, spins)
        assert bc == 12.0 and torch.all(bs == 1.0)
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_world_size_2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
