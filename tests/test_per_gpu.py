"""PrioritisedReplayBuffer on the device (eco_hip.agents.dqn.utils): the reference's scripted call sequences
(tests/golden/per.npz, recorded from src/agents/dqn/utils.py:86-277) replayed through the Python class under
the same numpy seed -- same ranks, buffer positions, importance weights, and the sampled transitions are
the ones the reference returned -- plus the vector-env path (add_batch -> eco_replay_push, sample ->
eco_replay_gather kernel) checked row by row against the transitions pushed."""
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "eco-dqn_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from test_per_cpu import OP_ADD, OP_SAMPLE, OP_UPDATE, case_params, close_f32, ops, GOLD  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ci", [0, 1, 2])
def test_prioritised_replay_matches_reference_script(ci):
    from eco_hip.agents.dqn.utils import PrioritisedReplayBuffer
    cap, alpha, beta0, anneal = case_params(ci)
    seed = int(GOLD["cases"][ci][2])
    np.random.seed(seed + 1000)          # make_per_golden.run_case seeds the reference's global RNG so
    buf = PrioritisedReplayBuffer(capacity=cap, alpha=alpha, beta0=beta0, device="cuda")
    buf.configure_beta_anneal_time(anneal)
    counter = 0
    n_samples = 0
    for op, n, abp, atd, hbp, htd, beta, parts, ranks, sbp, sw, sids in ops(ci):
        if op == OP_ADD:
            for _ in range(n):
                counter += 1
                t = torch.full((3,), float(counter))
                buf.add(t, torch.tensor([counter]), torch.tensor([0.5]), t + 0.5, torch.tensor([0.]))
        elif op == OP_UPDATE:
            buf.update_priorities(abp.tolist(), torch.tensor(atd, dtype=torch.float64))
        elif op == OP_SAMPLE:
            batch, w, bps = buf.sample(n)
            assert list(bps) == sbp.tolist()
            assert buf.partitions == [tuple(p) for p in parts.tolist()]
            assert batch[1].reshape(-1).cpu().tolist() == sids.tolist()
            assert torch.equal(batch[0][:, 0].cpu(), torch.tensor(sids, dtype=torch.float32))
            assert torch.equal(batch[3][:, 1].cpu(), torch.tensor(sids, dtype=torch.float32) + 0.5)
            assert w.shape == (n, 1) and w.device.type == "cuda"
            assert close_f32(w.cpu().numpy().ravel(), sw)
            n_samples += 1
        else:
            buf.rebalance()
        assert len(buf) == len(hbp)
        assert buf.beta == beta
    assert n_samples > 5


def test_prioritised_replay_vector_env_gather():
    from eco_hip.agents.dqn.utils import PrioritisedReplayBuffer
    dev = "cuda"
    cap, N, B = 300, 40, 64
    np.random.seed(5)
    buf = PrioritisedReplayBuffer(capacity=cap, alpha=0.7, beta0=0.5, device=dev)
    buf.configure_beta_anneal_time(100)
    newest = {}
    g = torch.Generator().manual_seed(0)
    rng = np.random.default_rng(1)
    counter = 0
    for it in range(9):                  # 576 pushes: the ring wraps, the heap fills and reuses slots
        xs = torch.randn(B, N, 8, generator=g)
        xn = torch.randn(B, N, 8, generator=g)
        gid = torch.arange(counter, counter + B, dtype=torch.int32)
        act = torch.randint(0, N, (B,), generator=g, dtype=torch.int32)
        rew = torch.randn(B, generator=g, dtype=torch.float64)
        done = (torch.rand(B, generator=g) < 0.2).to(torch.uint8)
        start = (counter % cap) + 1
        buf.add_batch(xs.to(dev), xn.to(dev), gid.to(dev), act.to(dev), rew.to(dev), done.to(dev))
        for b in range(B):
            newest[((start - 1 + b) % cap) + 1] = (xs[b], xn[b], int(gid[b]), int(act[b]), float(rew[b]), float(done[b]))
        counter += B
        live = sorted(newest)
        pick = rng.choice(live, size=20, replace=False)
        buf.update_priorities(pick.tolist(), rng.exponential(1.0, 20))
        (bxs, bact, brew, bxn, bdone, bgid), w, bps = buf.sample(32)
        torch.cuda.synchronize()
        for m, bp in enumerate(bps):
            exs, exn, egid, eact, erew, edone = newest[bp]
            assert torch.equal(bxs[m].cpu(), exs) and torch.equal(bxn[m].cpu(), exn)
            assert int(bgid[m]) == egid and int(bact[m]) == eact
            assert float(brew[m]) == float(np.float32(erew)) and float(bdone[m]) == edone
        assert float(w.max()) == 1.0 and w.min() > 0
    assert buf.full and len(buf) == cap
    buf.rebalance()
    _, w, bps = buf.sample(32)
    assert len(set(bps)) == len(bps)     # one rank per disjoint partition: distinct heap positions
