"""Pin the CPU oracle (oracle/) against the reference's own outputs (tests/golden/)."""
import hashlib
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import spinsystem_oracle as so
from oracle import mpnn_oracle as mo
from oracle import graphs as og


def _digest(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.uint64)[0]


def _make(f, p):
    J = f[p + "J"].astype(np.float64)
    n = J.shape[0]
    mode = str(f[p + "mode"])
    basis = str(f[p + "basis"])
    T = int(f[p + "T"])
    if mode == "s2v":
        env = so.SpinSystemOracle(J, T, observables=so.S2V_OBSERVABLES, reward_signal="DENSE",
                                  basin_reward=None, reversible_spins=False, spin_basis=basis)
    else:
        env = so.SpinSystemOracle(J, T, basin_reward=1. / n, spin_basis=basis)
    return env


def _run(f, p, check_obs):
    env = _make(f, p)
    obs = env.reset(spins=f[p + "spins"].astype(np.int64))
    n_obs = len(env.observables)
    assert env.mlr == f[p + "mlr"] and env.qn == f[p + "qn"] and env.lb == f[p + "lb"]
    check_obs(0, obs[:n_obs])
    assert env.score == f[p + "score"][0] and env.normalized_score == f[p + "nscore"][0]
    rews = f[p + "rew"]
    for t, a in enumerate(f[p + "actions"][:len(rews)]):
        obs, rew, done, _ = env.step(int(a))
        check_obs(t + 1, obs[:n_obs])
        assert float(rew) == rews[t], (p, t, rew, rews[t])       # bit-exact f64
        assert done == f[p + "done"][t]
        assert env.score == f[p + "score"][t + 1]
        assert env.normalized_score == f[p + "nscore"][t + 1]
        assert env.best_score == f[p + "best_score"][t + 1]
        assert env.best_score_normalized == f[p + "best_nscore"][t + 1]
        assert env.best_solution == f[p + "best_solution"][t + 1]
    if bool(f[p + "raised_past_end"]):
        with pytest.raises(NotImplementedError):
            env.step(0)


def test_env_er20_bit_exact():
    f = np.load(os.path.join(GOLDEN, "env_er20.npz"))
    for c in range(int(f["n_cases"])):
        p = f"c{c}_"
        ref = f[p + "obs"]

        def check(t, o):
            np.testing.assert_array_equal(o.view(np.uint64), ref[t].view(np.uint64))  # bitwise (signed zeros)
        _run(f, p, check)


def test_env_large_digests():
    f = np.load(os.path.join(GOLDEN, "env_large.npz"))
    for c in range(int(f["n_cases"])):
        p = f"c{c}_"
        dig = f[p + "obs_digest"]
        steps = list(f[p + "obs_steps"])
        at = f[p + "obs_at"]

        def check(t, o):
            if t in steps:
                np.testing.assert_array_equal(o, at[steps.index(t)])
            assert _digest(o) == dig[t], (p, t)
        _run(f, p, check)


def _weights(f, prefix):
    return {k: torch.from_numpy(f[prefix + k]) for k in mo.KEYS}


def test_mpnn_forward_matches_reference():
    f = np.load(os.path.join(GOLDEN, "mpnn_fwd.npz"))
    w = _weights(f, "er200/")
    assert sum(v.numel() for v in w.values()) == mo.N_PARAMS == 58425
    obs = torch.from_numpy(f["er200/obs"]).float()
    for b in range(2):
        q = mo.forward(w, obs[b])
        np.testing.assert_allclose(q.numpy(), f["er200/q_b1"][b], rtol=1e-5, atol=1e-5)
    q2 = mo.forward(w, obs)
    np.testing.assert_allclose(q2.numpy(), f["er200/q_b2"], rtol=1e-5, atol=1e-5)
    # batch coupling through norm.max() (mpnn.py:102) is real at this size
    assert np.abs(f["er200/q_b2"] - f["er200/q_b1"]).max() > 1e-4
    qb = mo.forward(w, torch.from_numpy(f["er200/obs_binary"]).float())
    np.testing.assert_allclose(qb.numpy(), f["er200/q_binary"], rtol=1e-5, atol=1e-5)
    w20 = _weights(f, "er20/")
    q8 = mo.forward(w20, torch.from_numpy(f["er20/obs"]).float())
    np.testing.assert_allclose(q8.numpy(), f["er20/q_b8"], rtol=1e-5, atol=1e-6)


def test_dqn_train_step_matches_reference():
    f = np.load(os.path.join(GOLDEN, "dqn_step.npz"))
    w = _weights(f, "w0/")
    tw = _weights(f, "target/")
    st = {"step": 0, "m": {}, "v": {}}
    for s in range(int(f["steps"])):
        p = f"s{s}/"
        w, loss = mo.train_step(
            w, st, torch.from_numpy(f[p + "states"]).float(), torch.from_numpy(f[p + "actions"]),
            torch.from_numpy(f[p + "rewards"]), torch.from_numpy(f[p + "states_next"]).float(),
            torch.from_numpy(f[p + "dones"]), target_w=tw)
        assert abs(loss - float(f[p + "loss"])) <= 1e-6 * max(1.0, abs(float(f[p + "loss"])))
        for k in mo.KEYS:
            np.testing.assert_allclose(w[k].numpy(), f[p + "w/" + k], rtol=1e-5, atol=1e-7)


def test_greedy_solver_matches_reference():
    f = np.load(os.path.join(GOLDEN, "greedy_solver.npz"))
    for c in range(int(f["n_cases"])):
        p = f"c{c}_"
        J = f[p + "J"].astype(np.float64)
        n = J.shape[0]
        env = so.SpinSystemOracle(J, 2 * n, basin_reward=1. / n)
        env.reset(spins=f[p + "spins"].astype(np.int64))
        acts = so.greedy_solve(env)
        np.testing.assert_array_equal(acts, f[p + "actions"])
        assert env.best_solution == f[p + "best_solution"]


def test_oracle_train_step_s2v_matches_reference():
    """Irreversible (S2V) train_step: -10000 masking before the double-DQN argmax (dqn.py:414-428),
    terminal next states included (tests/golden/dqn_step_s2v.npz)."""
    f = np.load(os.path.join(GOLDEN, "dqn_step_s2v.npz"))
    w = _weights(f, "w0/")
    tw = _weights(f, "target/")
    st = {"step": 0, "m": {}, "v": {}}
    assert f["s0/dones"].sum() >= 3
    for s in range(int(f["steps"])):
        p = f"s{s}/"
        w, loss = mo.train_step(
            w, st, torch.from_numpy(f[p + "states"]).float(), torch.from_numpy(f[p + "actions"]),
            torch.from_numpy(f[p + "rewards"]), torch.from_numpy(f[p + "states_next"]).float(),
            torch.from_numpy(f[p + "dones"]), target_w=tw, n_obs_in=1, reversible=False,
            allowed_value=float(f["allowed_action_state"]))
        assert abs(loss - float(f[p + "loss"])) <= 1e-6 * max(1.0, abs(float(f[p + "loss"])))
        for k in mo.KEYS:
            np.testing.assert_allclose(w[k].numpy(), f[p + "w/" + k], rtol=1e-5, atol=1e-7)


def test_oracle_norm_max_chunking():
    """forward(norm_max=) evaluates a batch in chunks exactly as one call (mpnn.py:102 batch coupling)."""
    g = torch.Generator().manual_seed(5)
    w = mo.init_weights(g, std=0.1)
    rng = np.random.default_rng(3)
    obs = []
    for n_edges_p in (0.1, 0.3, 0.5, 0.2):
        J = og.er_graph(16, n_edges_p, rng)
        x = rng.random((7, 16))
        obs.append(np.vstack([x, J]))
    obs = torch.from_numpy(np.array(obs)).float()
    full = mo.forward(w, obs)
    nmax = float(((obs[:, 7:, :] != 0).sum(1)).clamp(min=1).max())
    parts = torch.cat([mo.forward(w, obs[i:i + 1], norm_max=nmax).reshape(1, -1) for i in range(4)])
    torch.testing.assert_close(parts, full, rtol=0, atol=1e-6)
    assert not torch.allclose(mo.forward(w, obs[0]), full[0], atol=1e-6)  # the coupling is real


def test_oracle_chunked_train_step_matches_whole_batch():
    """train_step(chunk=k) (used at the BA-500 M = 256 size, where the [B, N, N, 63] edge tensor of one call
    would not fit) equals the one-call train step on the reference's own fixture: same loss, gradients and
    Adam step within fp32 summation-order noise."""
    f = np.load(os.path.join(GOLDEN, "dqn_step.npz"))
    w = _weights(f, "w0/")
    tw = _weights(f, "target/")
    p = "s0/"
    args = (torch.from_numpy(f[p + "states"]).float(), torch.from_numpy(f[p + "actions"]),
            torch.from_numpy(f[p + "rewards"]), torch.from_numpy(f[p + "states_next"]).float(),
            torch.from_numpy(f[p + "dones"]))
    s1, s2 = {"step": 0, "m": {}, "v": {}}, {"step": 0, "m": {}, "v": {}}
    w1, l1 = mo.train_step(w, s1, *args, target_w=tw)
    w2, l2 = mo.train_step(w, s2, *args, target_w=tw, chunk=3)
    assert args[0].shape[0] > 3 and args[0].shape[0] % 3 != 0
    assert abs(l1 - l2) <= 1e-6 * max(1.0, abs(l1))
    for k in mo.KEYS:
        torch.testing.assert_close(s2["grad"][k], s1["grad"][k], rtol=1e-4, atol=1e-7)
        torch.testing.assert_close(w2[k], w1[k], rtol=1e-5, atol=2e-7)
