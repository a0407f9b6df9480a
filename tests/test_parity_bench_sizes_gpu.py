"""Parity at the sizes bench.py times (VERDICT r01 "weak #1"):

  (a) ER-200, M = 2048 graphs: the training forward + mpnn_backward (+ the weight-gradient
      reduction) -- exactly the launch configuration of every benched gradient step -- against
      autograd through the torch oracle evaluated in float64 (the fp32 oracle's own error at this
      size is printed beside ours: a gradient summed over 409,600 nodes with cancellation is only
      as accurate as its accumulation order).  The oracle runs in chunks of graphs with the
      batch-global norm.max() passed explicitly (mpnn.py:102 couples the whole batch).
      Bar: 2e-4 relative L2 per tensor, or the fp32 oracle's own error vs float64 at this size where
      that is larger (see the test); Q within 1e-4 relative + 1e-5 absolute.
  (b) DQN.learn() at N = 200, B = 256 episodes, minibatch 256: the first train_step of the
      loop checked against oracle.train_step (dqn.py:403-451) on the same sampled minibatch.
      Bar: loss within 1e-4 relative; dLoss/dparams 2e-4 relative L2 per tensor; new weights
      within 2 lr (Adam's first step moves each weight by lr * g / (|g| + eps): a gradient
      entry at the fp32 noise floor may flip sign) and 99% of them within 2e-6.
  (c) N = 2000 (configs[4], G22-like ER(2000, 0.01) with unit weights) large forward against
      the oracle, one graph and several episodes SHARING it (the bench layout).  Bar: 5e-5 (1+|q|).

The torch oracle runs on the GPU here (plain fp32 torch ops, TF32 off): at these sizes its
dense [B, N, N, 63] edge tensors would take minutes on the host."""
import numpy as np
import pytest
import torch

from oracle import graphs as og
from oracle import mpnn_oracle as mo

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_tf32():
    old = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False
    yield
    torch.backends.cuda.matmul.allow_tf32 = old


def dense_batch(store, gids):
    """[k, N, N] float32 adjacency of graphs gids of a GraphStore, built on the device from its CSR."""
    n = store.n_spins
    gids = torch.as_tensor(gids, device=store.device).long()
    rp = store.row_ptr[gids].long()                       # [k, N+1]
    cnt = rp[:, -1]
    out = torch.zeros(len(gids), n, n, device=store.device)
    k_idx = torch.repeat_interleave(torch.arange(len(gids), device=store.device), cnt)
    starts = torch.repeat_interleave(store.edge_base[gids] - torch.cat([cnt.new_zeros(1), cnt.cumsum(0)[:-1]]), cnt)
    flat = torch.arange(int(cnt.sum()), device=store.device) + starts
    e = store.edges[flat].long() & 0xFFFFFFFF
    deg = rp[:, 1:] - rp[:, :-1]
    rows = torch.repeat_interleave(torch.arange(n, device=store.device).repeat(len(gids)), deg.flatten())
    w = ((e >> 24) & 0xFF).to(torch.int8).float()
    out[k_idx, rows, e & 0xFFFFFF] = w
    return out


def _obs(x, adj, n_obs=7):
    """Reference observation rows [k, n_obs + N, N] from node features [k, N, W] and adjacency."""
    return torch.cat([x[:, :, :n_obs].transpose(1, 2), adj], dim=1)


def _flat_to_dict(flat, n_obs=7):
    from eco_hip.networks.mpnn import param_layout
    out, off = {}, 0
    for name, shape in param_layout(n_obs):
        k = int(np.prod(shape))
        out[name] = flat[off:off + k].reshape(shape)
        off += k
    return out


def _rel(a, b):
    return float((a - b).norm() / max(float(b.norm()), 1e-12))


def test_backward_er200_m2048_matches_autograd():
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL
    n, M, chunk = 200, 2048, 64
    g = torch.Generator().manual_seed(2048)
    w = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    store = GraphStore.random("ER", M, n, 0.15, seed=77)
    x = torch.zeros(M, n, 8)
    x[:, :, :7] = torch.rand(M, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    dq = torch.randn(M, n, generator=g)
    xc, dqc = x.cuda(), dq.cuda()
    gids = torch.arange(M, dtype=torch.int32, device="cuda")
    saved = torch.empty(MPNN.saved_bytes(n, M), dtype=torch.uint8, device="cuda")
    q = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL, saved=saved)
    grad = torch.zeros_like(net.flat)
    net.backward_graphs(xc, store, gids, saved, dqc, grad)
    torch.cuda.synchronize()
    nmax = float(store.max_deg.max())
    # autograd through the oracle in float64 (the truth) and in float32 (the reference's own precision)
    w64 = {k: v.cuda().double().clone().requires_grad_(True) for k, v in w.items()}
    w32 = {k: v.cuda().clone().requires_grad_(True) for k, v in w.items()}
    for c0 in range(0, M, chunk):
        ids = torch.arange(c0, c0 + chunk)
        obs = _obs(xc[ids], dense_batch(store, ids))
        q64 = mo.forward(w64, obs.double(), norm_max=nmax)
        torch.testing.assert_close(q[c0:c0 + chunk].double(), q64.detach(), rtol=1e-4, atol=1e-5)
        (q64 * dqc[ids].double()).sum().backward()
        (mo.forward(w32, obs, norm_max=nmax) * dqc[ids]).sum().backward()
    got = _flat_to_dict(grad)
    report = {}
    for k in mo.KEYS:
        report[k] = (_rel(got[k].double(), w64[k].grad), _rel(w32[k].grad.double(), w64[k].grad))
    print("relative L2 error vs float64 autograd (eco-hip, fp32 torch oracle):", report)
    # At M = 2048 a gradient is a sum over 409,600 nodes, and a ReLU whose pre-activation lies within
    # fp32 rounding of 0 flips between any two fp32 evaluations: each flip moves a weight gradient by
    # ~1e-4 relative.  The fp32 reference itself is ~4.5e-4 from float64 here, so the bar is 2e-4 or
    # the fp32 reference's own accuracy at this size, whichever is looser: every tensor within 1.5x the
    # fp32 oracle's worst tensor error, and on average within 2x its average error.
    worst32 = max(e32 for _, e32 in report.values())
    for k, (err, err32) in report.items():
        assert err < max(2e-4, 1.5 * worst32), (k, err, err32)
    mean = np.mean([e for e, _ in report.values()])
    mean32 = np.mean([e32 for _, e32 in report.values()])
    assert mean <= max(2e-4, 2 * mean32), (mean, mean32)


def test_backward_ba500_m2048_matches_autograd():
    """configs[3]'s gradient step: BA(500, 4) +-1 graphs at M = 2048 through the dense kernels for one graph of
    224 < N <= 512 per workgroup (eco_mpnn_dl.h) + the weight-gradient reduction, against float64 autograd of the
    oracle (chunks of 8 graphs: the oracle's [k, N, N, 63] edge tensor).  Bars as the ER-200 test above."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL
    n, M, chunk = 500, 2048, 8
    g = torch.Generator().manual_seed(500)
    w = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    store = GraphStore.random("BA", M, n, 4, seed=78)
    assert store.unit_weights and store.adjbits is not None
    x = torch.zeros(M, n, 8)
    x[:, :, :7] = torch.rand(M, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    dq = torch.randn(M, n, generator=g)
    xc, dqc = x.cuda(), dq.cuda()
    gids = torch.arange(M, dtype=torch.int32, device="cuda")
    saved = torch.empty(MPNN.saved_bytes(n, M), dtype=torch.uint8, device="cuda")
    q = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL, saved=saved)
    grad = torch.zeros_like(net.flat)
    net.backward_graphs(xc, store, gids, saved, dqc, grad)
    torch.cuda.synchronize()
    nmax = float(store.max_deg.max())
    w64 = {k: v.cuda().double().clone().requires_grad_(True) for k, v in w.items()}
    w32 = {k: v.cuda().clone().requires_grad_(True) for k, v in w.items()}
    for c0 in range(0, M, chunk):
        ids = torch.arange(c0, c0 + chunk)
        obs = _obs(xc[ids], dense_batch(store, ids))
        q64 = mo.forward(w64, obs.double(), norm_max=nmax)
        torch.testing.assert_close(q[c0:c0 + chunk].double(), q64.detach(), rtol=1e-4, atol=1e-5)
        (q64 * dqc[ids].double()).sum().backward()
        (mo.forward(w32, obs, norm_max=nmax) * dqc[ids]).sum().backward()
    got = _flat_to_dict(grad)
    report = {k: (_rel(got[k].double(), w64[k].grad), _rel(w32[k].grad.double(), w64[k].grad)) for k in mo.KEYS}
    print("BA-500 M=2048 relative L2 error vs float64 autograd (eco-hip, fp32 torch oracle):", report)
    worst32 = max(e32 for _, e32 in report.values())
    for k, (err, err32) in report.items():
        assert err < max(2e-4, 1.5 * worst32), (k, err, err32)
    mean = np.mean([e for e, _ in report.values()])
    mean32 = np.mean([e32 for _, e32 in report.values()])
    assert mean <= max(2e-4, 2 * mean32), (mean, mean32)


def test_learn_er200_first_train_step_matches_oracle():
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    n, B, M = 200, 256, 256
    store = GraphStore.random("ER", B, n, 0.15, seed=5)
    env = VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    agent = DQN(env, lambda: MPNN(device="cuda"), init_weight_std=0.01, double_dqn=True, clip_Q_targets=False,
                replay_start_size=2 * B, replay_buffer_size=B * 8, gamma=0.95, update_target_frequency=4000,
                update_learning_rate=False, initial_learning_rate=1e-4, peak_learning_rate=1e-4,
                final_learning_rate=1e-4, update_frequency=32, minibatch_size=64, train_minibatch=M,
                initial_exploration_rate=1, final_exploration_rate=0.05, final_exploration_step=800000,
                adam_epsilon=1e-8, seed=11, evaluate=False, test_save_path=None)
    # target differs from online so double DQN's argmax/gather pairing matters
    with torch.no_grad():
        agent.target_network.flat.add_(torch.randn(agent.target_network.flat.shape, device="cuda",
                                                   generator=torch.Generator(device="cuda").manual_seed(1)) * 0.01)
    rec = {}
    orig = agent.train_step

    def spy(tr, sync_loss=True, loss_out=None, overlap=None):
        if not rec:
            rec["tr"] = [t.clone() for t in tr]
            rec["w"] = _flat_to_dict(agent.network.flat.clone())
            rec["tw"] = _flat_to_dict(agent.target_network.flat.clone())
            loss = orig(tr, sync_loss=True, loss_out=loss_out, overlap=overlap)
            rec["loss"] = loss
            rec["grad"] = _flat_to_dict(agent.grad.clone())
            rec["w1"] = _flat_to_dict(agent.network.flat.clone())
            return torch.tensor([loss], device="cuda")
        return orig(tr, sync_loss=sync_loss, loss_out=loss_out, overlap=overlap)

    agent.train_step = spy
    agent.learn(timesteps=B * 4)
    assert rec, "learn() never trained"
    xs, act, rew, xn, done, gid = rec["tr"]
    assert xs.shape[0] == M
    adj = dense_batch(store, gid)
    st = {"step": 0, "m": {}, "v": {}}
    w1, loss = mo.train_step(rec["w"], st, _obs(xs, adj), act.long().unsqueeze(1), rew.unsqueeze(1),
                             _obs(xn, adj), done.unsqueeze(1), gamma=0.95, lr=1e-4, eps=1e-8,
                             target_w=rec["tw"])
    assert abs(rec["loss"] - loss) <= 1e-4 * abs(loss), (rec["loss"], loss)
    for k in mo.KEYS:
        assert _rel(rec["grad"][k], st["grad"][k]) < 2e-4, k
        d = (rec["w1"][k] - w1[k]).abs()
        assert float(d.max()) <= 2e-4 + 1e-6, k
        assert float((d > 2e-6).float().mean()) <= 0.01, k


def test_learn_ba500_first_train_step_matches_oracle():
    """configs[3]'s training path at N = 500 (BA m=4, +-1 weights): DQN.learn() with the compact replay (its
    sample kernel's N > 256 path rebuilds s and s' of 500 vertices), the double-DQN s' pair and training
    forward through the one-graph-per-workgroup dense kernels (eco_mpnn_dl.h), the backward and the
    weight-gradient reduction; the first train_step against oracle.train_step on the same sampled minibatch
    (evaluated 16 graphs at a time with the batch's norm.max()).  Bars as the ER-200 test above."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN
    n, B, M = 500, 256, 256
    store = GraphStore.random("BA", B, n, 4, seed=55)
    env = VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    agent = DQN(env, lambda: MPNN(device="cuda"), init_weight_std=0.01, double_dqn=True, clip_Q_targets=False,
                replay_start_size=2 * B, replay_buffer_size=B * 8, gamma=0.95, update_target_frequency=4000,
                update_learning_rate=False, initial_learning_rate=1e-4, peak_learning_rate=1e-4,
                final_learning_rate=1e-4, update_frequency=32, minibatch_size=64, train_minibatch=M,
                initial_exploration_rate=1, final_exploration_rate=0.05, final_exploration_step=800000,
                adam_epsilon=1e-8, seed=13, evaluate=False, test_save_path=None)
    assert agent.compact_replay
    with torch.no_grad():
        agent.target_network.flat.add_(torch.randn(agent.target_network.flat.shape, device="cuda",
                                                   generator=torch.Generator(device="cuda").manual_seed(2)) * 0.01)
    rec = {}
    orig = agent.train_step

    def spy(tr, sync_loss=True, loss_out=None, overlap=None):
        if not rec:
            rec["tr"] = [t.clone() for t in tr]
            rec["w"] = _flat_to_dict(agent.network.flat.clone())
            rec["tw"] = _flat_to_dict(agent.target_network.flat.clone())
            loss = orig(tr, sync_loss=True, loss_out=loss_out, overlap=overlap)
            rec["loss"] = loss
            rec["grad"] = _flat_to_dict(agent.grad.clone())
            rec["w1"] = _flat_to_dict(agent.network.flat.clone())
            return torch.tensor([loss], device="cuda")
        return orig(tr, sync_loss=sync_loss, loss_out=loss_out, overlap=overlap)

    agent.train_step = spy
    agent.learn(timesteps=B * 3)
    assert rec, "learn() never trained"
    xs, act, rew, xn, done, gid = rec["tr"]
    assert xs.shape[0] == M
    adj = dense_batch(store, gid)
    st = {"step": 0, "m": {}, "v": {}}
    w1, loss = mo.train_step(rec["w"], st, _obs(xs, adj), act.long().unsqueeze(1), rew.unsqueeze(1),
                             _obs(xn, adj), done.unsqueeze(1), gamma=0.95, lr=1e-4, eps=1e-8,
                             target_w=rec["tw"], chunk=16)
    assert abs(rec["loss"] - loss) <= 1e-4 * abs(loss), (rec["loss"], loss)
    for k in mo.KEYS:
        assert _rel(rec["grad"][k], st["grad"][k]) < 2e-4, k
        d = (rec["w1"][k] - w1[k]).abs()
        assert float(d.max()) <= 2e-4 + 1e-6, k
        assert float((d > 2e-6).float().mean()) <= 0.01, k


@pytest.mark.parametrize("episodes", [1, 4])
def test_large_forward_n2000_matches_oracle(episodes):
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ActConfig, ECO_NORM_PER_GRAPH, ECO_NORM_PER_CALL
    n = 2000
    rng = np.random.default_rng(2000)
    J = og.er_graph(n, 0.01, rng, weights="uniform")
    store = GraphStore.from_dense([J])
    g = torch.Generator().manual_seed(22)
    w = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    x = torch.zeros(episodes, n, 8)
    x[:, :, :7] = torch.rand(episodes, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    xc = x.cuda()
    gids = torch.zeros(episodes, dtype=torch.int32, device="cuda")  # every episode on the one graph
    q = net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_GRAPH)
    wc = {k: v.cuda() for k, v in w.items()}
    adj = torch.from_numpy(J).float().cuda().unsqueeze(0)
    for b in range(episodes):
        with torch.no_grad():
            ref = mo.forward(wc, _obs(xc[b:b + 1], adj))
        err = float(((q[b] - ref).abs() / (1 + ref.abs())).max())
        assert err <= 5e-5, (b, err)
    acts = torch.empty(episodes, dtype=torch.int32, device="cuda")
    qc = torch.empty(episodes, n, device="cuda")
    net.forward_graphs(xc, store, gids, norm_scope=ECO_NORM_PER_CALL, q_out=qc,
                       act=ActConfig(0.0, 1, 0.0, 1, 0), actions_out=acts)
    assert torch.equal(acts.long(), qc.argmax(1))
    torch.testing.assert_close(qc, q, rtol=0, atol=0)  # one graph: per-call max == per-graph max


@pytest.mark.parametrize("weights", ["uniform", "discrete"])
def test_shared_graph_forward_matches_per_episode_and_oracle(weights):
    """The node-major shared-graph path (one graph, many episodes: eco_mpnn_shared.h) against the
    per-episode large kernel on the same graph replicated per episode, and against the oracle for a few
    episodes; 37 episodes = two full 16-episode slices + a padded one; +-1 weights exercise A- (V rows).
    Fused greedy act, and irreversible epsilon-greedy act restricted to allowed vertices."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ActConfig, ECO_NORM_PER_CALL
    n, B = 600, 37
    rng = np.random.default_rng(600)
    J = og.er_graph(n, 0.02, rng, weights=weights)
    one = GraphStore.from_dense([J])
    rep = GraphStore.from_dense([J] * B)
    g = torch.Generator().manual_seed(6)
    w = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    xc = x.cuda()
    q1 = net.forward_graphs(xc, one, torch.zeros(B, dtype=torch.int32, device="cuda"), norm_scope=ECO_NORM_PER_CALL)
    qr = net.forward_graphs(xc, rep, torch.arange(B, dtype=torch.int32, device="cuda"), norm_scope=ECO_NORM_PER_CALL)
    err = float(((q1 - qr).abs() / (1 + qr.abs())).max())
    assert err <= 5e-5, err
    wc = {k: v.cuda() for k, v in w.items()}
    adj = torch.from_numpy(J).float().cuda().unsqueeze(0)
    for b in (0, 15, 16, 36):
        with torch.no_grad():
            ref = mo.forward(wc, _obs(xc[b:b + 1], adj))
        assert float(((q1[b] - ref).abs() / (1 + ref.abs())).max()) <= 5e-5, b
    gz = torch.zeros(B, dtype=torch.int32, device="cuda")
    acts = torch.empty(B, dtype=torch.int32, device="cuda")
    qa = torch.empty(B, n, device="cuda")
    net.forward_graphs(xc, one, gz, norm_scope=ECO_NORM_PER_CALL, q_out=qa, act=ActConfig(0.0, 1, 0.0, 1, 0),
                       actions_out=acts)
    assert torch.equal(acts.long(), qa.argmax(1))
    # irreversible: only vertices whose feature 0 == -1 may be chosen (greedy and random)
    for eps in (0.0, 1.0):
        net.forward_graphs(xc, one, gz, norm_scope=ECO_NORM_PER_CALL, act=ActConfig(eps, 0, -1.0, 3, 1),
                           actions_out=acts)
        a = acts.long().cpu()
        assert bool((x[torch.arange(B), a, 0] == -1).all())
        if eps == 0.0:
            masked = qa.cpu().masked_fill(x[:, :, 0] != -1, float("-inf"))
            assert torch.equal(a, masked.argmax(1))


def test_shared_graph_forward_edge_table_beyond_lds():
    """Shared-graph path on a graph whose packed 16-bit edge table does NOT fit the aggregation's LDS next to the
    [N][8] block (ER(1500, 0.06): ~135k words = 270 KB; eco_mpnn_shared.h reads it from L2 then), +-1 weights, B = 9
    (two full slices and a padded one): against the per-episode kernel on the replicated graph and the oracle."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL
    n, B = 1500, 9
    rng = np.random.default_rng(1500)
    J = og.er_graph(n, 0.06, rng, weights="discrete")
    assert int((J != 0).sum()) * 2 > 160 * 1024 - n * 32  # the table cannot sit in the LDS
    one = GraphStore.from_dense([J])
    rep = GraphStore.from_dense([J] * B)
    g = torch.Generator().manual_seed(8)
    wts = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(wts)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    xc = x.cuda()
    q1 = net.forward_graphs(xc, one, torch.zeros(B, dtype=torch.int32, device="cuda"), norm_scope=ECO_NORM_PER_CALL)
    qr = net.forward_graphs(xc, rep, torch.arange(B, dtype=torch.int32, device="cuda"), norm_scope=ECO_NORM_PER_CALL)
    assert torch.isfinite(q1).all()
    err = float(((q1 - qr).abs() / (1 + qr.abs())).max())
    assert err <= 5e-5, err
    wc = {k: v.cuda() for k, v in wts.items()}
    adj = torch.from_numpy(J).float().cuda().unsqueeze(0)
    for b in (0, 8):
        with torch.no_grad():
            ref = mo.forward(wc, _obs(xc[b:b + 1], adj))
        assert float(((q1[b] - ref).abs() / (1 + ref.abs())).max()) <= 5e-5, b


def test_shared_graph_forward_hub_and_isolated_nodes():
    """Shared-graph path on a graph with a hub adjacent to every other vertex (one CSR row of N - 1 edges: the
    longest aggregation tile row) and isolated vertices (empty rows, norm clamped to 1), +-1 weights, B = 6
    (one full and one padded slice): against the per-episode kernel on the replicated graph and the oracle."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL
    n, B = 700, 6
    rng = np.random.default_rng(700)
    J = og.er_graph(n, 0.01, rng, weights="discrete")
    J[5, :] = 0
    J[:, 5] = 0
    J[17, :] = 0
    J[:, 17] = 0                                   # isolated vertices 5 and 17
    hub = 3
    w = np.where(rng.random(n) < 0.5, 1.0, -1.0)
    w[[hub, 5, 17]] = 0
    J[hub, :] = w
    J[:, hub] = w
    one = GraphStore.from_dense([J])
    rep = GraphStore.from_dense([J] * B)
    g = torch.Generator().manual_seed(7)
    wts = mo.init_weights(g, std=0.1)
    net = MPNN(device="cuda")
    net.load_state_dict(wts)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    xc = x.cuda()
    q1 = net.forward_graphs(xc, one, torch.zeros(B, dtype=torch.int32, device="cuda"), norm_scope=ECO_NORM_PER_CALL)
    qr = net.forward_graphs(xc, rep, torch.arange(B, dtype=torch.int32, device="cuda"), norm_scope=ECO_NORM_PER_CALL)
    assert torch.isfinite(q1).all()
    err = float(((q1 - qr).abs() / (1 + qr.abs())).max())
    assert err <= 5e-5, err
    wc = {k: v.cuda() for k, v in wts.items()}
    adj = torch.from_numpy(J).float().cuda().unsqueeze(0)
    for b in (0, 5):
        with torch.no_grad():
            ref = mo.forward(wc, _obs(xc[b:b + 1], adj))
        assert float(((q1[b] - ref).abs() / (1 + ref.abs())).max()) <= 5e-5, b


def test_shared_graph_tables_cache():
    """The shared-graph path keeps its degree ranking and tile tables in the MPNN workspace across calls, keyed
    by a hash of the graph and the layout (eco_mpnn_shared.h shared_key_kernel).  A repeated call (tables from
    the cache) must equal the first bitwise; a call on another graph, a call after the per-episode large kernel
    overwrote the workspace, and a call after the graph's edge words were changed IN PLACE must each equal a
    fresh network (own workspace, tables built in that call) bitwise."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL
    n, B = 600, 8
    rng = np.random.default_rng(601)
    J1 = og.er_graph(n, 0.02, rng, weights="discrete")
    J2 = og.er_graph(n, 0.02, rng, weights="discrete")
    one1, one2 = GraphStore.from_dense([J1]), GraphStore.from_dense([J2])
    rep1 = GraphStore.from_dense([J1] * B)
    g = torch.Generator().manual_seed(61)
    w = mo.init_weights(g, std=0.1)
    x = torch.zeros(B, n, 8)
    x[:, :, :7] = torch.rand(B, n, 7, generator=g) * 2 - 1
    x[:, :, 0] = torch.where(x[:, :, 0] > 0, 1.0, -1.0)
    xc = x.cuda()
    gz = torch.zeros(B, dtype=torch.int32, device="cuda")

    def fresh(store):
        other = MPNN(device="cuda")
        other.load_state_dict(w)
        return other.forward_graphs(xc, store, gz, norm_scope=ECO_NORM_PER_CALL).clone()

    net = MPNN(device="cuda")
    net.load_state_dict(w)
    qa = net.forward_graphs(xc, one1, gz, norm_scope=ECO_NORM_PER_CALL).clone()
    qb = net.forward_graphs(xc, one1, gz, norm_scope=ECO_NORM_PER_CALL).clone()
    assert torch.equal(qa, qb)
    qc = net.forward_graphs(xc, one2, gz, norm_scope=ECO_NORM_PER_CALL).clone()
    assert torch.equal(qc, fresh(one2))
    net.forward_graphs(xc, rep1, torch.arange(B, dtype=torch.int32, device="cuda"), norm_scope=ECO_NORM_PER_CALL)
    qd = net.forward_graphs(xc, one1, gz, norm_scope=ECO_NORM_PER_CALL).clone()
    assert torch.equal(qd, qa)
    # flip every edge weight in place (+1 <-> -1: still unit weights with both signs, same degrees)
    e = one1.edges.view(torch.int32)
    wsign = e >> 24
    e.copy_((e & 0xFFFFFF) | ((-wsign) << 24))
    qe = net.forward_graphs(xc, one1, gz, norm_scope=ECO_NORM_PER_CALL).clone()
    assert not torch.equal(qe, qa)
    assert torch.equal(qe, fresh(one1))


def test_shared_graph_tables_cache_across_batch_sizes():
    """The cached tables live at batch-dependent offsets of the workspace: calls on one graph alternating between
    two batch sizes (the key includes B) must each equal a fresh network's result bitwise."""
    from eco_hip.graphs import GraphStore
    from eco_hip.networks.mpnn import MPNN
    from eco_hip._lib import ECO_NORM_PER_CALL
    n = 600
    rng = np.random.default_rng(602)
    J = og.er_graph(n, 0.02, rng, weights="discrete")
    one = GraphStore.from_dense([J])
    g = torch.Generator().manual_seed(62)
    w = mo.init_weights(g, std=0.1)
    x = torch.zeros(12, n, 8)
    x[:, :, :7] = torch.rand(12, n, 7, generator=g) * 2 - 1
    xc = x.cuda()
    net = MPNN(device="cuda")
    net.load_state_dict(w)
    for B in (12, 5, 12, 5):
        gz = torch.zeros(B, dtype=torch.int32, device="cuda")
        q = net.forward_graphs(xc[:B].contiguous(), one, gz, norm_scope=ECO_NORM_PER_CALL).clone()
        other = MPNN(device="cuda")
        other.load_state_dict(w)
        ref = other.forward_graphs(xc[:B].contiguous(), one, gz, norm_scope=ECO_NORM_PER_CALL)
        assert torch.equal(q, ref), B
