"""Pin the multi-problem oracle (oracle/problems_oracle.py) against the reference's own trajectories
(tests/golden/env_problems.npz, made by tests/golden/make_golden.py env_problems): every scorer of
score_solver.py (MinCover, MaxIndSet, MaxClique, MinDomSet, MinCut, Cut), ECO mode with
MAIN_OBSERVABLES (set problems) or DEFAULT_OBSERVABLES (cut problems), and S2V mode.

Bar: rewards, scores and every observation row equal (==) to the reference's float64 values; greedy
rollouts take the same actions."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import problems_oracle as po

F = np.load(os.path.join(GOLDEN, "env_problems.npz"))
CASES = [f"c{i}_" for i in range(int(F["n_cases"]))]
TARGET = {"CUT": po.CUT, "MIN_COVER": po.MIN_COVER, "MIN_CUT": po.MIN_CUT, "MAX_IND_SET": po.MAX_IND_SET,
          "MAX_CLIQUE": po.MAX_CLIQUE, "MIN_DOM_SET": po.MIN_DOM_SET}


def env_kwargs(f, p):
    """experiments/train_eco.py:244-315 for the case's target and mode (mirrors make_golden.problem_args)."""
    target = TARGET[str(f[p + "target"])]
    n = f[p + "J"].shape[0]
    obs = po.DEFAULT_OBSERVABLES if target in (po.CUT, po.MIN_CUT) else po.MAIN_OBSERVABLES
    kw = dict(target=target, observables=obs, reward_signal="BLS", basin_reward=1. / n, reversible_spins=True)
    if str(f[p + "mode"]) == "s2v":
        kw.update(observables=[po.SPIN_STATE], reward_signal="DENSE", basin_reward=None, reversible_spins=False)
    return kw


def make_env(f, p):
    """Oracle env built on J0 (its own reset, as the reference constructor), then moved to J."""
    env = po.ProblemSpinSystemOracle(f[p + "J0"].astype(np.float64), int(f[p + "T"]), **env_kwargs(f, p),
                                     init_reset=False)
    env.reset(spins=-np.ones(env.n_spins))
    env.matrix = f[p + "J"].astype(np.float64)
    return env


@pytest.mark.parametrize("p", CASES)
def test_problem_trajectory_matches_reference(p):
    f = F
    env = make_env(f, p)
    n_obs = len(env.observables)
    obs = env.reset(spins=f[p + "spins"].astype(np.int64))
    sc = env.scorer
    assert [sc.mlr, sc.qn, sc.inorm, sc.lb] == list(f[p + "norms"]), p
    ref = f[p + "obs"]
    np.testing.assert_array_equal(obs[:n_obs], ref[0], err_msg=p + " reset")
    assert env.score == f[p + "score"][0] and env.normalized_score == f[p + "nscore"][0]
    assert env.best_solution == f[p + "best_solution"][0]
    rews = f[p + "rew"]
    for t, a in enumerate(f[p + "actions"][:len(rews)]):
        obs, rew, done, _ = env.step(int(a))
        np.testing.assert_array_equal(obs[:n_obs], ref[t + 1], err_msg=f"{p} step {t}")
        assert float(rew) == rews[t], (p, t, rew, rews[t])
        assert done == f[p + "done"][t]
        for k, v in (("score", env.score), ("nscore", env.normalized_score), ("best_score", env.best_score),
                     ("best_nscore", env.best_score_normalized), ("best_solution", env.best_solution)):
            assert v == f[p + k][t + 1], (p, t, k, v, f[p + k][t + 1])


@pytest.mark.parametrize("p", CASES)
def test_problem_greedy_matches_reference(p):
    f = F
    env = po.ProblemSpinSystemOracle(f[p + "J"].astype(np.float64), int(f[p + "T"]), **env_kwargs(f, p))
    env.reset(spins=f[p + "spins"].astype(np.int64))
    acts, done = [], False
    while not done:
        a = po.greedy_action(env)
        if a is None:
            break
        _, _, done, _ = env.step(a)
        acts.append(a)
    assert acts == list(f[p + "greedy_actions"]), p
    assert env.best_solution == f[p + "greedy_best_solution"]
    assert env.best_score == f[p + "greedy_best_score"]


def test_cut_targets_reject_validity_mask_observables():
    J = np.array([[0., 1.], [1., 0.]])
    with pytest.raises(TypeError):
        po.ProblemSpinSystemOracle(J, 4, target=po.MIN_CUT, observables=po.MAIN_OBSERVABLES)
