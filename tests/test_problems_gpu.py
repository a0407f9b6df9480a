"""Generic-scorer env kernels (eco_env_problems.hip) against the reference and the oracle.

* Reference trajectories (tests/golden/env_problems.npz): every OptimisationTarget except ENERGY, ECO mode
  (MAIN_OBSERVABLES for the set problems, DEFAULT_OBSERVABLES for the cut ones) and S2V mode; each episode
  is first reset on graph J0 and then on J, which pins the stale invalidity normaliser of the reference's
  first observation.  Greedy rollouts (solver.py:110-127) from the same starts.
* Batched random and greedy rollouts on larger graphs (several vertices per lane) against
  oracle/problems_oracle.py, which tests/test_problems_oracle.py pins to the same fixture.

Bar: rewards, scores and float64 observation rows equal (==) to the reference / oracle values; the fp32
node features are those rows rounded to float32; greedy actions identical."""
import os
import zlib

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import graphs as og
from oracle import problems_oracle as po

pytestmark = pytest.mark.gpu

F = np.load(os.path.join(GOLDEN, "env_problems.npz"))
CASES = [f"c{i}_" for i in range(int(F["n_cases"]))]


def _env_args(target_name, mode, n):
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, MAIN_OBSERVABLES, ExtraAction, Observable,
                                    OptimisationTarget, RewardSignal)
    t = OptimisationTarget[target_name]
    obs = DEFAULT_OBSERVABLES if target_name in ("CUT", "MIN_CUT") else MAIN_OBSERVABLES
    a = dict(observables=obs, reward_signal=RewardSignal.BLS, extra_action=ExtraAction.NONE, optimisation_target=t,
             norm_rewards=True, basin_reward=1. / n, reversible_spins=True)
    if mode == "s2v":
        a.update(observables=[Observable.SPIN_STATE], reward_signal=RewardSignal.DENSE, basin_reward=None,
                 reversible_spins=False)
    return a


def _oracle_kwargs(target_name, mode, n):
    t = getattr(po, target_name)
    obs = po.DEFAULT_OBSERVABLES if target_name in ("CUT", "MIN_CUT") else po.MAIN_OBSERVABLES
    kw = dict(target=t, observables=obs, reward_signal="BLS", basin_reward=1. / n, reversible_spins=True)
    if mode == "s2v":
        kw.update(observables=[po.SPIN_STATE], reward_signal="DENSE", basin_reward=None, reversible_spins=False)
    return kw


def _check_x(vec, rows_f64):
    """obs_x = the f64 rows rounded to fp32, zero beyond n_obs."""
    x = vec.obs_x.cpu().numpy()
    n_obs = rows_f64.shape[1]
    np.testing.assert_array_equal(x[:, :, :n_obs], np.transpose(rows_f64, (0, 2, 1)).astype(np.float32))
    assert not x[:, :, n_obs:].any()


@pytest.mark.parametrize("p", CASES)
def test_problem_env_matches_reference(p):
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.graphs import GraphStore
    f = F
    target, mode = str(f[p + "target"]), str(f[p + "mode"])
    J0, J = f[p + "J0"].astype(np.float64), f[p + "J"].astype(np.float64)
    n, T = J.shape[0], int(f[p + "T"])
    store = GraphStore.from_dense([J0, J])
    vec = VecSpinSystem(store, 1, T, want_f64=True, **_env_args(target, mode, n))
    vec.reset(graph_ids=[0], spins=-np.ones((1, n)))        # the reference constructor's own reset, on J0
    vec.reset(graph_ids=[1], spins=f[p + "spins"][None])
    vec.check_errors()
    ref = f[p + "obs"]
    np.testing.assert_array_equal(vec.obs_f64[0].cpu().numpy(), ref[0], err_msg=p + " reset")
    _check_x(vec, vec.obs_f64.cpu().numpy())
    st = vec.read()
    mlr, qn, inorm, lb = f[p + "norms"]
    assert st["max_local_reward"][0].item() == mlr and st["quality_normalizer"][0].item() == qn
    assert st["invalidity_normalizer"][0].item() == inorm and st["lower_bound"][0].item() == lb
    assert st["score"][0].item() == f[p + "score"][0] and st["normalized_score"][0].item() == f[p + "nscore"][0]
    assert st["best_solution"][0].item() == f[p + "best_solution"][0]
    rews = f[p + "rew"]
    for t, a in enumerate(f[p + "actions"][:len(rews)]):
        _, rew, done = vec.step(torch.tensor([int(a)], dtype=torch.int32, device="cuda"))
        vec.check_errors()
        np.testing.assert_array_equal(vec.obs_f64[0].cpu().numpy(), ref[t + 1], err_msg=f"{p} step {t}")
        assert rew[0].item() == rews[t], (p, t, rew[0].item(), rews[t])
        assert bool(done[0].item()) == bool(f[p + "done"][t])
        st = vec.read()
        for k, key in (("score", "score"), ("normalized_score", "nscore"), ("best_score", "best_score"),
                       ("best_score_normalized", "best_nscore"), ("best_solution", "best_solution")):
            assert st[k][0].item() == f[p + key][t + 1], (p, t, k, st[k][0].item(), f[p + key][t + 1])
    _check_x(vec, vec.obs_f64.cpu().numpy())


@pytest.mark.parametrize("p", CASES)
def test_problem_greedy_matches_reference(p):
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.graphs import GraphStore
    f = F
    target, mode = str(f[p + "target"]), str(f[p + "mode"])
    J = f[p + "J"].astype(np.float64)
    n, T = J.shape[0], int(f[p + "T"])
    vec = VecSpinSystem(GraphStore.from_dense([J]), 1, T, **_env_args(target, mode, n))
    vec.reset(graph_ids=[0], spins=f[p + "spins"][None])
    acts = []
    for _ in range(T):
        if bool(vec.read()["done"][0].item()):
            break
        a = vec.greedy_actions()
        if bool(vec.read()["done"][0].item()):   # the solver stopped (best change < 0)
            break
        acts.append(int(a[0].item()))
        vec.step(a)
    vec.check_errors()
    assert acts == list(f[p + "greedy_actions"]), p
    st = vec.read()
    assert st["best_solution"][0].item() == f[p + "greedy_best_solution"]
    assert st["best_score"][0].item() == f[p + "greedy_best_score"]


TARGETS = ["MIN_COVER", "MAX_IND_SET", "MAX_CLIQUE", "MIN_DOM_SET", "MIN_CUT", "CUT"]  # CUT: the MaxCut kernels


@pytest.mark.parametrize("target", TARGETS)
@pytest.mark.parametrize("mode", ["eco", "s2v"])
@pytest.mark.parametrize("n,kind", [(40, "ER"), (130, "BA")])
def test_problem_env_batched_vs_oracle(target, mode, n, kind):
    """B = 6 episodes on 3 graphs, random actions then greedy actions, every step against the oracle."""
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.graphs import GraphStore
    rng = np.random.default_rng(zlib.crc32(f"{target}/{mode}/{n}".encode()))
    w = "discrete" if target in ("MIN_CUT", "CUT") else "uniform"
    Js = [og.er_graph(n, 0.2, rng, w) if kind == "ER" else og.ba_graph(n, 4, rng, w) for _ in range(3)]
    B = 6
    gids = np.array([b % 3 for b in range(B)])
    T = 2 * n if mode == "eco" else n
    args = _env_args(target, mode, n)
    vec = VecSpinSystem(GraphStore.from_dense(Js), B, T, want_f64=True, **args)
    spins = (2 * rng.integers(0, 2, (B, n)) - 1) if mode == "eco" else -np.ones((B, n), dtype=np.int64)
    vec.reset(graph_ids=gids, spins=spins)
    vec.check_errors()
    envs = []
    for b in range(B):
        e = po.ProblemSpinSystemOracle(Js[gids[b]], T, init_reset=False, **_oracle_kwargs(target, mode, n))
        e.reset(spins=spins[b])
        envs.append(e)
    np.testing.assert_array_equal(vec.obs_f64.cpu().numpy(), np.stack([e.state_rows() for e in envs]))
    done = np.zeros(B, bool)
    n_random = T // 2 if mode == "eco" else n // 2
    for t in range(T):
        if t < n_random:
            if mode == "s2v":   # irreversible: pick among spins still at -1
                acts = np.array([rng.choice(np.flatnonzero(e.state[0] < 0)) if not d else 0
                                 for e, d in zip(envs, done)])
            else:
                acts = rng.integers(0, n, B)
            a_dev = torch.tensor(acts, dtype=torch.int32, device="cuda")
            greedy_stop = np.zeros(B, bool)
        else:
            a_dev = vec.greedy_actions()
            acts = a_dev.cpu().numpy()
            gacts = [po.greedy_action(e) if not d else None for e, d in zip(envs, done)]
            greedy_stop = np.array([g is None for g in gacts]) & ~done
            for b in range(B):
                if not done[b] and gacts[b] is not None:
                    assert acts[b] == gacts[b], (target, mode, b, t, acts[b], gacts[b])
            st = vec.read()
            assert np.array_equal(st["done"].cpu().numpy().astype(bool), done | greedy_stop)
            done |= greedy_stop
        _, rew, dn = vec.step(a_dev)
        vec.check_errors()
        rew, dn = rew.cpu().numpy(), dn.cpu().numpy().astype(bool)
        rows = vec.obs_f64.cpu().numpy()
        for b, e in enumerate(envs):
            if done[b]:
                assert rew[b] == 0.0 and dn[b]
                continue
            _, r, d, _ = e.step(int(acts[b]))
            assert rew[b] == r, (target, mode, b, t, rew[b], r)
            assert dn[b] == d
            np.testing.assert_array_equal(rows[b], e.state_rows(), err_msg=f"{target} {mode} b={b} t={t}")
            done[b] |= d
        if done.all():
            break
    st = vec.read()
    for b, e in enumerate(envs):
        assert st["score"][b].item() == e.score and st["normalized_score"][b].item() == e.normalized_score
        assert st["best_score"][b].item() == e.best_score and st["best_solution"][b].item() == e.best_solution
