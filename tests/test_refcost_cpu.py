"""The reference-cost CPU restatement (oracle/refcost.py, bench.py's cpu_baseline) reproduces the
reference's values: ECO/SIGNED episodes of tests/golden/env_er20.npz and env_large.npz, bit-exact
(observation rows compared bitwise, rewards and scores ==), and its committed speed calibration
against the reference is within the +-15 % bar."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, REPO
from oracle import refcost


def _digest(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.uint64)[0]


def _cases(name):
    f = np.load(os.path.join(GOLDEN, name))
    for c in range(int(f["n_cases"])):
        p = f"c{c}_"
        if str(f[p + "mode"]) == "eco" and str(f[p + "basis"]) == "SIGNED":
            yield f, p


@pytest.mark.parametrize("name", ["env_er20.npz", "env_large.npz"])
def test_refcost_env_matches_reference(name):
    n_run = 0
    for f, p in _cases(name):
        J = f[p + "J"].astype(np.float64)
        env = refcost.RefCostEnv(int(f[p + "T"]))
        obs = env.reset(J, f[p + "spins"].astype(np.int64))
        full = p + "obs" in f.files
        steps = list(f[p + "obs_steps"]) if not full else None

        def check(t, o):
            o = o[:7]
            if full:
                np.testing.assert_array_equal(o.view(np.uint64), f[p + "obs"][t].view(np.uint64))
            else:
                assert _digest(o) == f[p + "obs_digest"][t], (p, t)
        check(0, obs)
        assert env.score == f[p + "score"][0]
        rews = f[p + "rew"]
        for t, a in enumerate(f[p + "actions"][:len(rews)]):
            obs, rew, done, _ = env.step(int(a))
            check(t + 1, obs)
            assert float(rew) == rews[t], (p, t)
            assert done == f[p + "done"][t]
            assert env.score == f[p + "score"][t + 1]
            assert env.best_solution == f[p + "best_solution"][t + 1]
        n_run += 1
    assert n_run >= 2


def test_refcost_calibration_within_bar():
    with open(os.path.join(REPO, "oracle", "refcost_calibration.json")) as fh:
        cal = json.load(fh)
    for case in cal["cases"]:
        assert abs(case["ratio"] - 1.0) <= 0.15, case
