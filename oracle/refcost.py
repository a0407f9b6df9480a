"""Reference-cost CPU restatement of the MaxCut env step (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

Only bench.py's cpu_baseline leg and tests/ import this module; the product never does.

`oracle/spinsystem_oracle.py` restates the reference's *values* with vectorised shortcuts (it runs
~4x faster than the reference).  This module restates the reference's per-step *operation mix*, so
that timing it on the GPU box's host cores (where the reference itself cannot travel) measures what
the reference costs there (SURVEY.md 8d "CPU side-by-side"):

  per step (src/envs/spinsystem.py:355-559, MaximumCutUnbiasedScorer score_solver.py:343-419)
    * np.copy of the [7, N] float64 state                                    (:369)
    * 4 dense `s * (J @ s)` matvecs: score mask + normalised score mask for the action's delta
      (:393-394), then quality mask and score mask of the new spins (:414-416)
    * a Python list of N zeros for the (unused) MaxCut invalidity mask       (:415, score_solver.py:403-407)
    * the visited-state buffer: a dict of lists of Python sets, scanned linearly (utils.py:438-464)
    * on a new best: calculate_cut of the best spins                         (:459-463)
    * the observables loop with its if/elif dispatch; DISTANCE_FROM_BEST_SOLUTION evaluates two
      dense quadratic-form cuts with an N x N np.outer temporary each       (:486-535, :516-519)
    * get_observation: state copy + np.vstack with the N x N adjacency     (:561-574)

Values are the reference's own (bit-exact against tests/golden/env_er20.npz, env_large.npz:
tests/test_refcost_cpu.py).  Its speed is calibrated in the build container against the reference
imported from /root/reference by oracle/calibrate_refcost.py (result: oracle/refcost_calibration.json,
bar +-15 %).  No reference source is copied: this is an independent restatement.
"""
from enum import Enum

import numpy as np


class Obs(Enum):
    """Observable values of src/envs/utils.py:48-65; an Enum like the reference's, because its
    observables loop compares enum members (part of the per-step cost being restated)."""
    SPIN_STATE = 1
    IMMEDIATE_QUALITY_CHANGE = 2
    IMMEDIATE_VALIDITY_DIFFERENCE = 3
    IMMEDIATE_VALIDITY_CHANGE = 4
    TIME_SINCE_FLIP = 5
    EPISODE_TIME = 6
    TERMINATION_IMMANENCY = 7
    NUMBER_OF_QUALITY_IMPROVEMENTS = 8
    NUMBER_OF_VALIDITY_IMPROVEMENTS = 9
    DISTANCE_FROM_BEST_SOLUTION = 10
    DISTANCE_FROM_BEST_STATE = 11
    GLOBAL_VALIDITY_DIFFERENCE = 12
    VALIDITY_BIT = 13


class Reward(Enum):
    """RewardSignal (src/envs/utils.py:14-18)."""
    DENSE = 1
    BLS = 2
    SINGLE = 3
    CUSTOM_BLS = 4


class Stop(Enum):
    """Stopping (src/envs/utils.py:60-63)."""
    NORMAL = 1
    QUARTER = 2
    EARLY = 3


class Basis(Enum):
    """SpinBasis (src/envs/utils.py:26-28)."""
    SIGNED = 1
    BINARY = 2


DEFAULT_OBSERVABLES = [Obs.SPIN_STATE, Obs.IMMEDIATE_QUALITY_CHANGE, Obs.TIME_SINCE_FLIP,
                       Obs.DISTANCE_FROM_BEST_SOLUTION, Obs.DISTANCE_FROM_BEST_STATE,
                       Obs.NUMBER_OF_QUALITY_IMPROVEMENTS, Obs.TERMINATION_IMMANENCY]


def cut_value(spins, J):
    """utils.py:90-94: 1/4 sum J * (1 - s s^T), dense."""
    return 0.25 * np.sum(np.multiply(J, 1 - np.outer(spins, spins)))


def cut_gains(spins, J):
    """utils.py:97-102: s * (J @ s)."""
    return spins * np.matmul(J, spins)


class MaxCutScorer:
    """score_solver.py:175-200 + 343-419, as method calls (the reference's dispatch depth)."""

    def prepare(self, J):
        n = J.shape[0]
        empty = np.array([-1] * n, dtype=np.float64)
        q = self.quality_mask(empty, J)
        self.mlr = np.max(q[np.nonzero(q)])
        self.inv_norm = 1
        self.qn = max(1, np.sum(np.multiply(J, (J > 0))) / 2)
        self.lb = min(0, np.sum(np.multiply(J, (J < 0))) / 2)

    def solution(self, s, J):
        return cut_value(s, J)

    def quality(self, s, J):
        return self.solution(s, J) + abs(min(0, self.lb))

    def invalidity(self, s, J):
        return 0

    def valid(self, s, J):
        return self.invalidity(s, J) == 0

    def score(self, s, J):
        return self.valid(s, J) * self.quality(s, J) - self.invalidity(s, J)

    def normalized_score(self, s, J):
        return self.valid(s, J) * self.quality(s, J) / self.qn - self.invalidity(s, J) / self.inv_norm

    def quality_mask(self, s, J):
        return cut_gains(s, J)

    def invalidity_mask(self, s, J):
        return [0 for _ in range(len(s))]

    def score_mask(self, s, J):
        return self.quality_mask(s, J)

    def normalized_score_mask(self, s, J):
        return self.quality_mask(s, J) / self.qn


class VisitedSets:
    """utils.py:438-464: flipped-vertex sets bucketed by size in lists (linear membership scan)."""

    def __init__(self):
        self.buckets = {}
        self.cur = set()
        self.size = 0

    def update(self, a):
        nxt = self.cur.copy()
        if a in self.cur:
            nxt.remove(a)
            self.size -= 1
        else:
            nxt.add(a)
            self.size += 1
        lst = self.buckets.get(self.size)
        if lst is not None and nxt in lst:
            self.cur = nxt
            return False
        if lst is None:
            lst = []
        lst.append(nxt)
        self.cur = nxt
        self.buckets[self.size] = lst
        return True


class RefCostEnv:
    """ECO MaxCut SpinSystem (DEFAULT_OBSERVABLES, BLS, normalised rewards, basin reward 1/N,
    reversible spins, NORMAL stopping): reset(J, spins) / step(a) -> (obs, rew, done, None)."""

    def __init__(self, max_steps, basin_reward=True):
        self.max_steps = max_steps
        self.observables = list(enumerate(DEFAULT_OBSERVABLES))
        self.use_basin = basin_reward
        self.scorer = MaxCutScorer()
        # the configuration branches every reference step evaluates (ECO MaxCut values)
        self.reward_signal = Reward.BLS
        self.norm_rewards = True
        self.stag_punishment = None
        self.memory_length = None
        self.stopping = Stop.NORMAL
        self.reversible = True
        self.basis = Basis.SIGNED
        self.biased = False

    def reset(self, J, spins):
        self.J = np.asarray(J, dtype=np.float64)
        n = self.n = self.J.shape[0]
        self.basin_reward = 1. / n if self.use_basin else None
        self.t = 0
        self.early = 0
        self.scorer.prepare(self.J)
        st = np.zeros((len(self.observables), n))
        st[0, :] = np.asarray(spins, dtype=np.float64)
        st = st.astype('float')
        qm = self.scorer.quality_mask(st[0, :], self.J)
        self.scorer.invalidity_mask(st[0, :], self.J)
        for idx, ob in self.observables:
            if ob == Obs.IMMEDIATE_QUALITY_CHANGE:
                st[idx, :n] = qm / self.scorer.mlr
            elif ob == Obs.IMMEDIATE_VALIDITY_DIFFERENCE:
                pass
            elif ob == Obs.IMMEDIATE_VALIDITY_CHANGE:
                pass
            elif ob == Obs.NUMBER_OF_QUALITY_IMPROVEMENTS:
                st[idx, :] = np.sum(qm > 0) / n
        self.state = st
        self.score = self.scorer.score(st[0, :], self.J)
        self.nscore = self.scorer.normalized_score(st[0, :], self.J)
        self.best_score = self.best_obs_score = self.score
        self.best_nscore = self.best_obs_nscore = self.nscore
        self.best_solution = self.scorer.solution(st[0, :], self.J)
        self.best_spins = st[0, :].copy()
        self.best_obs_spins = st[0, :].copy()
        self.visited = VisitedSets()
        return self.observation()

    def observation(self):
        st = self.state.copy()
        if self.basis == Basis.BINARY:
            st[0, :] = (1 - st[0, :]) / 2
        if self.biased:
            raise NotImplementedError
        return np.vstack((st, self.J))

    def step(self, a):
        done = False
        rew = 0
        self.t += 1
        self.early += 1
        if self.t > self.max_steps:
            raise NotImplementedError
        sc, J = self.scorer, self.J
        n = self.n
        new = np.copy(self.state)
        if a == n:
            raise NotImplementedError("ExtraAction.NONE only")
        d = sc.score_mask(self.state[0, :], J)[a]
        dn = sc.normalized_score_mask(self.state[0, :], J)[a]
        new[0, a] = -self.state[0, a]
        self.score += d
        self.nscore += dn
        self.state = new
        qm = sc.quality_mask(new[0, :n], J)
        sc.invalidity_mask(new[0, :n], J)
        smask = sc.score_mask(new[0, :n], J)
        if self.score > self.best_obs_score:
            self.early = 0
            if self.reward_signal == Reward.BLS:
                if self.norm_rewards:
                    rew = self.nscore - self.best_obs_nscore
                else:
                    rew = self.score - self.best_obs_score
        if self.reward_signal == Reward.DENSE:
            rew = dn if self.norm_rewards else d
        if self.stag_punishment is not None or self.basin_reward is not None:
            new_state = self.visited.update(a)
        if self.stag_punishment is not None and not new_state:
            rew -= self.stag_punishment
        if self.basin_reward is not None:
            if np.all(smask <= 0):
                if new_state:
                    rew += self.basin_reward
        if self.score > self.best_score:
            self.best_score = self.score
            self.best_nscore = self.nscore
            self.best_spins = new[0, :n].copy()
            self.best_solution = sc.solution(self.best_spins, J)
        if self.memory_length is not None:
            raise NotImplementedError
        else:
            self.best_obs_score = self.best_score
            self.best_obs_nscore = self.best_nscore
            self.best_obs_spins = self.best_spins.copy()
        for idx, ob in self.observables:
            if ob == Obs.IMMEDIATE_QUALITY_CHANGE:
                self.state[idx, :n] = qm / sc.mlr
            elif ob == Obs.TIME_SINCE_FLIP:
                self.state[idx, :] += (1. / self.max_steps)
                self.state[idx, a] = 0
            elif ob == Obs.IMMEDIATE_VALIDITY_DIFFERENCE:
                pass
            elif ob == Obs.IMMEDIATE_VALIDITY_CHANGE:
                pass
            elif ob == Obs.EPISODE_TIME:
                self.state[idx, :] += (1. / self.max_steps)
            elif ob == Obs.TERMINATION_IMMANENCY:
                self.state[idx, :] = max(0, ((self.t - self.max_steps) / self.max_steps) + 1)
            elif ob == Obs.NUMBER_OF_QUALITY_IMPROVEMENTS:
                self.state[idx, :] = np.sum(qm > 0) / n
            elif ob == Obs.DISTANCE_FROM_BEST_SOLUTION:
                cq = sc.quality(self.state[0, :n], J)
                bq = sc.quality(self.best_spins[:n], J)
                self.state[idx, :] = np.abs(cq - bq) / sc.mlr
            elif ob == Obs.NUMBER_OF_VALIDITY_IMPROVEMENTS:
                pass
            elif ob == Obs.DISTANCE_FROM_BEST_STATE:
                self.state[idx, :] = np.count_nonzero(self.best_obs_spins[:n] - self.state[0, :n])
        if self.t == self.max_steps:
            done = True
        if self.stopping == Stop.EARLY and self.early == 15:
            done = True
        if self.stopping == Stop.QUARTER and self.t == self.max_steps // 4:
            done = True
        if not self.reversible:
            if len((self.state[0, :n] < 0).nonzero()[0]) == 0:
                done = True
        return self.observation(), rew, done, None


def random_policy_rate(n, p, seconds, seed=0):
    """configs[0]'s plumbing loop at size n: env.step with uniform random actions on fresh seeded
    ER(n, p) +-1 graphs; only step() is timed (graph generation and reset are not).
    Returns (steps, busy seconds)."""
    import time
    from oracle.graphs import er_graph
    rng = np.random.default_rng(seed)
    env = RefCostEnv(2 * n)
    steps, busy = 0, 0.0
    while busy < seconds:
        J = er_graph(n, p, rng)
        env.reset(J, 2 * rng.integers(0, 2, n) - 1)
        acts = rng.integers(0, n, 2 * n)
        t0 = time.perf_counter()
        for a in acts:
            env.step(int(a))
        busy += time.perf_counter() - t0
        steps += 2 * n
    return steps, busy


if __name__ == "__main__":
    # one baseline worker process: python -m oracle.refcost N SECONDS SEED -> "steps busy"
    import sys
    s, b = random_policy_rate(int(sys.argv[1]), float(sys.argv[4]) if len(sys.argv) > 4 else 0.15,
                              float(sys.argv[2]), int(sys.argv[3]))
    print(s, b)
