"""configs[3] at its own size on one GPU: bench.build_train_agent(..., "BA", 4, 2048) -- BA(500,
m = 4) graphs, 8192 episodes, fresh graphs per episode, minibatch M = 2048, the compact replay ring of one episode's
worth (8192 x 1000 = 8.2 M transitions, ~17 GB) -- through the B = 8192 act launch (the DL forward kernel), the
N = 500 env step at 8192 episodes and three training vector steps (K = 8 gradient steps each: replay sample from
the full-size ring, s' pair, training forward, backward, weight gradients, Adam).  Properties checked: every loss
finite, no device error, parameters moved and finite, and on sampled minibatches the compact ring's rebuilt s' rows
are consistent with its s rows: exactly the action's spin flipped, its time-since-flip feature reset to 0, every other
vertex's counter advanced by one step, and finite features throughout (the compact ring itself is checked bitwise
against the fp32 feature ring at N = 500 in test_dqn_gpu.py::test_compact_replay_matches_feature_replay)."""
import sys

import numpy as np
import pytest
import torch

from conftest import REPO

pytestmark = pytest.mark.gpu


def test_configs3_ba500_b8192_trains():
    sys.path.insert(0, REPO)
    import bench
    dev = torch.device("cuda", 0)
    B, n = 8192, 500
    agent, store, env, lr = bench.build_train_agent(dev, B, n, "BA", 4, 2048, seed=77)
    assert agent.compact_replay and agent.replay_buffer._capacity == B * 2 * n
    w0 = agent.network.flat.clone()
    agent.start()
    steps = 0
    while not agent._ready or steps < 3:
        agent.iteration()
        steps += agent._ready
    torch.cuda.synchronize()
    env.check_errors()
    store.check_errors()
    losses = agent.losses()
    assert len(losses) >= 3 * agent._k_per_vec
    assert all(np.isfinite(l) for _, l in losses)
    w = agent.network.flat
    assert torch.isfinite(w).all() and float((w - w0).abs().max()) > 0
    T = env.max_steps
    for _ in range(2):
        xs, act, rew, xn, done, gid = agent.replay_buffer.sample(2048)
        assert torch.isfinite(xs).all() and torch.isfinite(xn).all() and torch.isfinite(rew).all()
        assert int(gid.min()) >= 0 and int(gid.max()) < store.n_graphs
        assert int(act.min()) >= 0 and int(act.max()) < n
        flipped = (xs[:, :, 0] != xn[:, :, 0])
        assert torch.equal(flipped.sum(1), torch.ones(2048, dtype=flipped.sum(1).dtype, device="cuda"))
        rows = torch.arange(2048, device="cuda")
        assert torch.equal(flipped.nonzero()[:, 1].to(torch.int32), act)
        assert torch.equal(xn[rows, act.long(), 0], -xs[rows, act.long(), 0])
        assert (xn[rows, act.long(), 2] == 0).all()          # TIME_SINCE_FLIP of the flipped vertex reset
        others = torch.ones_like(flipped)
        others[rows, act.long()] = False
        step = 1.0 / T                                        # the counter feature advances by 1 / T per step
        d = (xn[:, :, 2] - xs[:, :, 2])[others]
        assert float((d - step).abs().max()) <= 1e-6
    print(f"configs[3] B={B} N={n}: {len(losses)} gradient steps, last loss {losses[-1][1]:.4g}, ring "
          f"{agent.replay_buffer.ring.numel() / 2**30:.1f} GiB, graphs regenerated {agent.graphs_regenerated}")
