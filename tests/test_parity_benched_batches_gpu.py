"""Parity at the EXACT batch shapes bench.py times for its inference workloads (VERDICT r02 "next" #1):

  (a) configs[4] (`bench.py --workload gset`): one G22-like ER(2000, 0.01) unit-weight graph shared by
      B = 1024 episodes.  That batch runs the persistent multi-item loops of the shared-graph kernels
      (eco_mpnn_shared.h: shared_agg_kernel's register prefetch of the next (slice, chunk, episode) block,
      items = 16 * ceil(B/4) = 4096 > 256 workgroups; shared_lin_kernel's tile loop) that smaller tests
      never enter.  Every one of the 1024 episodes is compared with mpnn_forward_large_kernel on a
      store holding the same graph once per episode (one CSR, n_graphs = B: the per-episode path), and
      episodes {0, 63, 64, 511, 1023} with the fp32 oracle (mpnn.py:40-159).  Then three steps of the
      greedy best-cut search (experiments/utils.py:154-187): the shared path's actions must be argmaxes
      of the per-episode path's Q (within the fp32 bar), exactly equal wherever the top-1/top-2 margin
      exceeds it, and both envs must stay bitwise identical.
  (b) configs[1] (`--workload er20`): 4096 ER-20 episodes on their own graphs, graphs_per_block(20,
      4096) = 9 per dense block (455 full blocks + a 1-graph tail), norm.max() over the whole call
      (mpnn.py:102): all 4096 Q rows against the oracle with the call-global norm max, and the fused
      greedy act against the argmax.

Bar: |q - q_ref| <= 5e-7 (1 + |q_ref|) (fp32, different summation order; tests/test_mpnn_gpu.py)."""
import numpy as np
import pytest
import torch

from oracle import mpnn_oracle as mo

pytestmark = pytest.mark.gpu
TOL = 5e-7


@pytest.fixture(autouse=True)
def _no_tf32():
    old = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False
    yield
    torch.backends.cuda.matmul.allow_tf32 = old


def _env(store, B, n):
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    return VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                         extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                         spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)


def _scaled_err(q, ref):
    return float(((q - ref).abs() / (1 + ref.abs())).max())


def _bench_net(dev="cuda"):
    """The random-init network of bench.py inference_bench (std 0.1, generator seed 0)."""
    from eco_hip.networks.mpnn import MPNN
    net = MPNN(device=dev)
    net.init_normal_(0.1, generator=torch.Generator().manual_seed(0))
    return net


def _weights(net):
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


def _obs(x, adj, n_obs=7):
    return torch.cat([x[:, :, :n_obs].transpose(1, 2), adj], dim=1)


def _check_greedy(acts, q_ref, label):
    """acts must be argmaxes of q_ref within the fp32 bar, and THE argmax where the margin is clear."""
    top2 = q_ref.topk(2, dim=1).values
    qa = q_ref.gather(1, acts.long().unsqueeze(1)).squeeze(1)
    slack = TOL * (1 + top2[:, 0].abs())
    assert bool((qa >= top2[:, 0] - 2 * slack).all()), label
    clear = (top2[:, 0] - top2[:, 1]) > 4 * slack
    assert int(clear.sum()) > 0.5 * len(acts), (label, int(clear.sum()))
    assert torch.equal(acts.long()[clear], q_ref.argmax(1)[clear]), label


def test_gset_shared_graph_b1024_matches_per_episode_and_oracle():
    from eco_hip.graphs import GraphStore
    from eco_hip._lib import ActConfig, ECO_NORM_PER_CALL
    n, B = 2000, 1024
    one = GraphStore.random("ER", 1, n, 0.01, seed=1234, weights="uniform")   # bench.py's configs[4] graph
    # the same graph once per episode: B row_ptr rows over ONE edge array (edge_base 0) -> the per-episode
    # large kernel (the shared path needs n_graphs == 1)
    rep = GraphStore(one.row_ptr.expand(B, n + 1).contiguous(), torch.zeros(B, dtype=torch.int64, device="cuda"),
                     one.edges, device="cuda")
    assert rep.n_graphs == B and rep.unit_weights
    net = _bench_net()
    w = _weights(net)
    rng = np.random.default_rng(22)
    spins = 2 * rng.integers(0, 2, (B, n)) - 1
    env1, envr = _env(one, B, n), _env(rep, B, n)
    x1 = env1.reset(graph_ids=np.zeros(B, np.int64), spins=spins)
    xr = envr.reset(graph_ids=np.arange(B), spins=spins)
    assert torch.equal(x1, xr)
    adj = torch.from_numpy(one.dense(0)).float().cuda().unsqueeze(0)
    g0 = torch.zeros(B, dtype=torch.int32, device="cuda")
    gr = torch.arange(B, dtype=torch.int32, device="cuda")
    acts = torch.empty(B, dtype=torch.int32, device="cuda")
    greedy = ActConfig(0.0, 1, 0.0, 0, 0)
    for step in range(4):
        q1 = torch.empty(B, n, device="cuda")
        net.forward_graphs(env1.obs_x, one, g0, norm_scope=ECO_NORM_PER_CALL, q_out=q1, act=greedy,
                           actions_out=acts)
        qr = net.forward_graphs(envr.obs_x, rep, gr, norm_scope=ECO_NORM_PER_CALL)
        assert torch.isfinite(q1).all()
        err = _scaled_err(q1, qr)
        assert err <= TOL, (step, err)
        assert torch.equal(acts.long(), q1.argmax(1)), step        # fused act = argmax of its own Q
        if step == 0:
            for b in (0, 63, 64, 511, 1023):
                with torch.no_grad():
                    ref = mo.forward({k: v.cuda() for k, v in w.items()}, _obs(env1.obs_x[b:b + 1], adj))
                assert _scaled_err(q1[b], ref) <= TOL, b
        if step == 3:
            break
        _check_greedy(acts, qr, f"step {step}")
        _, r1, d1 = env1.step(acts)
        _, rr, dr = envr.step(acts)
        assert torch.equal(env1.obs_x, envr.obs_x) and torch.equal(r1, rr) and torch.equal(d1, dr)
    env1.check_errors()
    envr.check_errors()
    s1, sr = env1.read(), envr.read()
    for k in ("score", "best_score", "best_solution", "current_step"):
        assert torch.equal(s1[k], sr[k]), k


def test_er20_b4096_blocks_match_oracle():
    from eco_hip.graphs import GraphStore
    from eco_hip._lib import ActConfig, ECO_NORM_PER_CALL
    from test_parity_bench_sizes_gpu import dense_batch
    n, B = 20, 4096
    store = GraphStore.random("ER", B, n, 0.15, seed=1234, weights="discrete")  # bench.py's configs[1] pool
    net = _bench_net()
    w = {k: v.cuda() for k, v in _weights(net).items()}
    env = _env(store, B, n)
    env.reset(graph_ids=np.arange(B), seed=1234)
    gids = env.graph_ids
    acts = torch.empty(B, dtype=torch.int32, device="cuda")
    nmax = float(store.max_deg.max().clamp(min=1))
    greedy = ActConfig(0.0, 1, 0.0, 0, 0)
    for step in range(3):
        q = torch.empty(B, n, device="cuda")
        net.forward_graphs(env.obs_x, store, gids, norm_scope=ECO_NORM_PER_CALL, q_out=q, act=greedy,
                           actions_out=acts)
        ref = torch.empty_like(q)
        with torch.no_grad():
            for c0 in range(0, B, 512):
                ids = torch.arange(c0, c0 + 512)
                ref[c0:c0 + 512] = mo.forward(w, _obs(env.obs_x[ids], dense_batch(store, ids)), norm_max=nmax)
        err = (q - ref).abs() / (1 + ref.abs())
        # per block of 9 graphs: the first, a middle and the 1-graph tail block are all in range
        for blk in (0, 227, 455):
            assert float(err[blk * 9:(blk + 1) * 9].max()) <= TOL, (step, blk)
        assert float(err.max()) <= TOL, (step, float(err.max()))
        assert torch.equal(acts.long(), q.argmax(1)), step
        _check_greedy(acts, ref, f"step {step}")
        env.step(acts)
    env.check_errors()
