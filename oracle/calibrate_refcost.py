"""Calibrate oracle/refcost.py's speed against the REFERENCE itself (build container only: needs
/root/reference; never run on the GPU box).

    OMP_NUM_THREADS=1 python oracle/calibrate_refcost.py

Times env.step with uniform random actions (configs[0]'s plumbing loop) for the reference's
SpinSystem (imported from /root/reference with the identity numba.jit shim of tests/golden/_shim, as
tests/golden/make_golden.py does) and for oracle/refcost.RefCostEnv, on the same seeded graphs,
spins and actions, one thread, interleaved in rounds; writes oracle/refcost_calibration.json with
the median rates and ratio = refcost / reference per size.  Bar: |ratio - 1| <= 0.15.
"""
import json
import os
import platform
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("MKL_NUM_THREADS", "1")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(REPO, "tests", "golden", "_shim"))

import numpy as np  # noqa: E402

import src.envs.core as ising_env  # noqa: E402
from src.envs.utils import (SingleGraphGenerator, RewardSignal, ExtraAction, OptimisationTarget,  # noqa: E402
                            SpinBasis, DEFAULT_OBSERVABLES)
from oracle import refcost  # noqa: E402
from oracle.graphs import er_graph  # noqa: E402


def ref_env(J, T):
    n = J.shape[0]
    args = {'observables': DEFAULT_OBSERVABLES, 'reward_signal': RewardSignal.BLS,
            'extra_action': ExtraAction.NONE, 'optimisation_target': OptimisationTarget.CUT,
            'spin_basis': SpinBasis.SIGNED, 'norm_rewards': True, 'memory_length': None,
            'horizon_length': None, 'stag_punishment': None, 'basin_reward': 1. / n, 'reversible_spins': True}
    return ising_env.make("SpinSystem", SingleGraphGenerator(J), T, **args)


def time_episodes(make, episodes):
    steps, busy = 0, 0.0
    for J, spins, acts in episodes:
        env = make(J)
        env.reset(spins)
        t0 = time.perf_counter()
        for a in acts:
            env.step(int(a))
        busy += time.perf_counter() - t0
        steps += len(acts)
    return steps / busy


def main():
    out = {"cpu": platform.processor() or platform.machine(), "threads": 1, "cases": []}
    try:
        with open("/proc/cpuinfo") as fh:
            out["cpu"] = next(ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    for n, n_ep, rounds in ((20, 60, 7), (200, 3, 7)):
        rng = np.random.default_rng(n)
        eps = []
        for _ in range(n_ep):
            J = er_graph(n, 0.15, rng)
            eps.append((J, 2 * rng.integers(0, 2, n) - 1, rng.integers(0, n, 2 * n)))
        r_ref, r_rc = [], []
        for _ in range(rounds):
            r_ref.append(time_episodes(lambda J: _RefAdapter(ref_env(J, 2 * J.shape[0])), eps))
            r_rc.append(time_episodes(lambda J: _RcAdapter(J), eps))
        ref, rc = float(np.median(r_ref)), float(np.median(r_rc))
        out["cases"].append({"workload": f"ER-{n} env.step, random actions, 1 thread", "reference_steps_per_s": ref,
                             "refcost_steps_per_s": rc, "ratio": rc / ref})
        print(out["cases"][-1])
    with open(os.path.join(HERE, "refcost_calibration.json"), "w") as fh:
        json.dump(out, fh, indent=1)


class _RefAdapter:
    def __init__(self, env):
        self.env = env

    def reset(self, spins):
        self.env.reset(spins=spins)

    def step(self, a):
        return self.env.step(a)


class _RcAdapter:
    def __init__(self, J):
        self.J = J
        self.env = refcost.RefCostEnv(2 * J.shape[0])

    def reset(self, spins):
        self.env.reset(self.J, spins)

    def step(self, a):
        return self.env.step(a)


if __name__ == "__main__":
    main()
