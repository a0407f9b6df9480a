"""CPU restatement of the reference's problem scorers and the generic SpinSystem step
(TEST INFRASTRUCTURE ONLY: imported by tests/ and never on the product path).

The reference scores a spin vector s in {-1,+1}^N (x = [s == 1] is "in the set") through a
ScoreSolver (src/envs/score_solver.py), and SpinSystemBase (src/envs/spinsystem.py) turns
its masks into rewards and the 13 observables.  This module restates every scorer in
vectorised numpy from the set quantities below (the reference loops over vertex flips for
MinDomSet and MaxClique, score_solver.py:692-700, :806-817), and reproduces the reference's
float64 operation order wherever a float result is produced, so rewards and observations
can be compared for equality.

  n1 = sum x                     A = J @ x  (weighted in-set neighbour sums)
  U  = J @ (1-x)                 P = (J > 0) @ x  (positive in-set neighbours, MinDomSet)

  target        measure  invalidity inv(s)            flip mask im_i = inv(s^i) - inv(s)
  MIN_COVER     n1       uncovered edges (1-x)J(1-x)/2   s_i U_i                     (:287-308)
  MAX_IND_SET   n1       edges inside xJx/2              -s_i A_i                    (:559-583)
  MAX_CLIQUE    n1       n1(n1-1) - xJx                  add: 2(n1-A_i); drop: 2(A_i-n1+1)  (:800-829)
  MIN_DOM_SET   n1       #{k: x_k=0, P_k=0}              neighbour counts, see _mds_imask (:672-712)
  CUT / MIN_CUT cut(s)   0 (mask is a python list: the validity observables raise TypeError upstream)

Normalisers (set_* methods) and the score algebra of MaximizationProblem / MinimizationProblem
(score_solver.py:175-229) and of the generic get_score_mask / get_normalized_score_mask
(:310-339 and copies) are restated in `Scorer`.
"""
import numpy as np

from .spinsystem_oracle import HistoryBuffer, calculate_cut, calculate_cut_changes

# OptimisationTarget (src/envs/utils.py:32-39)
CUT, ENERGY, MIN_COVER, MIN_CUT, MAX_IND_SET, MAX_CLIQUE, MIN_DOM_SET = 1, 2, 3, 4, 5, 6, 7
TARGET_NAMES = {CUT: "CUT", MIN_COVER: "MIN_COVER", MIN_CUT: "MIN_CUT", MAX_IND_SET: "MAX_IND_SET",
                MAX_CLIQUE: "MAX_CLIQUE", MIN_DOM_SET: "MIN_DOM_SET"}

# Observable (src/envs/utils.py:46-62)
(SPIN_STATE, IMMEDIATE_QUALITY_CHANGE, IMMEDIATE_VALIDITY_DIFFERENCE, IMMEDIATE_VALIDITY_CHANGE,
 TIME_SINCE_FLIP, EPISODE_TIME, TERMINATION_IMMANENCY, NUMBER_OF_QUALITY_IMPROVEMENTS,
 NUMBER_OF_VALIDITY_IMPROVEMENTS, DISTANCE_FROM_BEST_SOLUTION, DISTANCE_FROM_BEST_STATE,
 GLOBAL_VALIDITY_DIFFERENCE, VALIDITY_BIT) = range(1, 14)
MAIN_OBSERVABLES = list(range(1, 14))  # src/envs/utils.py:76-88 (all 13, in enum order)
DEFAULT_OBSERVABLES = [SPIN_STATE, IMMEDIATE_QUALITY_CHANGE, TIME_SINCE_FLIP, DISTANCE_FROM_BEST_SOLUTION,
                       DISTANCE_FROM_BEST_STATE, NUMBER_OF_QUALITY_IMPROVEMENTS, TERMINATION_IMMANENCY]
VALIDITY_MASK_OBSERVABLES = (IMMEDIATE_VALIDITY_DIFFERENCE, IMMEDIATE_VALIDITY_CHANGE,
                             NUMBER_OF_VALIDITY_IMPROVEMENTS)


class Scorer:
    """ScoreSolver (score_solver.py:11-172) + its Maximization/Minimization base (:175-229).
    Normalisers start at 1 / lower bound 0 (:15-21) and persist across resets, which the env's
    stale-normaliser quirk below depends on."""
    maximise = True
    cut_like = False

    def __init__(self, target):
        self.target = target
        self.mlr = 1
        self.qn = 1
        self.inorm = 1
        self.lb = 0

    # -- per-target pieces (overridden) --
    def measure(self, s, J):
        return np.sum(s == 1)

    def solution(self, s, J):
        raise NotImplementedError

    def inv(self, s, J):
        raise NotImplementedError

    def qmask(self, s, J):
        raise NotImplementedError

    def imask(self, s, J):
        raise NotImplementedError

    # -- shared algebra --
    def quality(self, s, J):
        if self.maximise:   # :196-200
            return self.measure(s, J) + abs(min(0, self.lb))
        return max(0, self.qn) - self.measure(s, J)  # :224-228

    def valid(self, s, J):
        return self.inv(s, J) == 0  # :166-171

    def vmask(self, s, J):
        return (self.inv(s, J) + self.imask(s, J)) == 0  # :156-164

    def score(self, s, J):  # :182-188 / :210-216
        return self.valid(s, J) * self.quality(s, J) - self.inv(s, J)

    def nscore(self, s, J):  # :190-194 / :218-222
        return self.valid(s, J) * self.quality(s, J) / self.qn - self.inv(s, J) / self.inorm

    def score_mask(self, s, J):  # generic form, :310-324
        uq = self.quality(s, J) + self.qmask(s, J)
        ui = self.inv(s, J) + self.imask(s, J)
        return self.vmask(s, J) * uq - ui - self.score(s, J)

    def nscore_mask(self, s, J):  # :326-339
        uq = (self.quality(s, J) + self.qmask(s, J)) / self.qn
        ui = (self.inv(s, J) + self.imask(s, J)) / self.inorm
        return self.vmask(s, J) * uq - ui - self.nscore(s, J)


class CutScorer(Scorer):
    """MaximumCutUnbiasedScorer (score_solver.py:343-419) and MinimumCutUnbiasedSolver (:423-505)."""
    cut_like = True

    def __init__(self, target):
        super().__init__(target)
        self.maximise = target == CUT
        self.sign = 1.0 if target == CUT else -1.0

    def set_normalisers(self, J):
        neg = np.sum(np.multiply(J, (J < 0)))
        if self.target == CUT:
            self.qn = max(1, np.sum(np.multiply(J, (J > 0))) / 2)   # :353-357
        else:
            self.qn = max(1, abs(neg))                               # :439-443 (not halved)
        self.inorm = 1                                               # :347-351, :433-437
        self.lb = min(0, neg / 2)                                    # :359-365, :455-461

    def set_mlr(self, J):   # :367-375, :445-453: max nonzero entry of the quality mask at s = -1
        qm = self.qmask(np.array([-1.0] * J.shape[0]), J)
        nz = qm[np.nonzero(qm)]
        if nz.size == 0:
            return False
        self.mlr = np.max(nz)
        return True

    def measure(self, s, J):
        return calculate_cut(s, J)

    def solution(self, s, J):
        return calculate_cut(s, J)

    def inv(self, s, J):
        return 0

    def qmask(self, s, J):
        g = calculate_cut_changes(s, J)
        return g if self.target == CUT else -g

    def imask(self, s, J):
        raise TypeError("invalidity mask is a python list for cut problems (score_solver.py:403-407, "
                        ":489-493): the validity observables raise TypeError in the reference")

    def score_mask(self, s, J):
        return self.qmask(s, J)

    def nscore_mask(self, s, J):
        return self.qmask(s, J) / self.qn


class SetScorer(Scorer):
    """MinimumVertexCover (:232-339), MaximumIndependentSet (:509-614), MinimumDominatingSet (:617-741),
    MaximumClique (:743-858)."""

    def __init__(self, target):
        super().__init__(target)
        self.maximise = target in (MAX_IND_SET, MAX_CLIQUE)

    def set_normalisers(self, J):
        n = J.shape[0]
        self.qn = n                                            # :254-258, :531-535, :624-628, :750-754
        self.lb = 0
        if self.target in (MIN_COVER, MAX_IND_SET):
            self.inorm = np.sum(J) / 2                         # :246-252, :513-517
        elif self.target == MAX_CLIQUE:
            self.inorm = np.sum(J)                             # :763-768
        else:
            self.inorm = n                                     # :637-641

    def set_mlr(self, J):
        n = J.shape[0]
        if self.target in (MIN_COVER, MAX_IND_SET):           # :236-244, :519-523 at s = -1: N + max row sum
            self.mlr = n + np.max(J @ np.ones(n))
        elif self.target == MAX_CLIQUE:
            self.mlr = n                                       # :756-761
        else:
            self.mlr = 2 * n                                   # :630-635
        return True

    def solution(self, s, J):   # :263-271, :537-544, :649-656, :776-783
        if not self.valid(s, J):
            return len(s) if not self.maximise else 0
        return np.sum(s == 1)

    def inv(self, s, J):
        x = (s == 1).astype(np.float64)
        if self.target == MIN_COVER:
            o = 1.0 - x
            return (o @ J @ o) / 2
        if self.target == MAX_IND_SET:
            return (x @ J @ x) / 2
        if self.target == MAX_CLIQUE:
            n1 = x.sum()
            return np.sum(x * (n1 - 1 - J @ x))
        P = (J > 0).astype(np.float64) @ x
        return float(np.sum((x == 0) & (P == 0)))

    def qmask(self, s, J):
        s = np.asarray(s, dtype=np.float64)
        return s.copy() if not self.maximise else -s   # :279-285, :552-557, :664-670, :791-798

    def imask(self, s, J):
        s = np.asarray(s, dtype=np.float64)
        x = (s == 1).astype(np.float64)
        if self.target == MIN_COVER:
            return s * (J @ (1.0 - x))
        if self.target == MAX_IND_SET:
            return -s * (J @ x)
        if self.target == MAX_CLIQUE:
            n1 = x.sum()
            A = J @ x
            return np.where(x == 1, 2 * (A - (n1 - 1)), 2 * (n1 - A))
        return self._mds_imask(x, J)

    @staticmethod
    def _mds_imask(x, J):
        Jp = (J > 0).astype(np.float64)
        P = Jp @ x
        out = x == 0
        c0 = (out & (P == 0)).astype(np.float64)
        c1 = (out & (P == 1)).astype(np.float64)
        alone = (P == 0).astype(np.float64)
        return np.where(x == 1, alone + Jp @ c1, -alone - Jp @ c0)


def make_scorer(target):
    """ScoreSolverFactory.get (score_solver.py:860-885), unbiased graphs."""
    if target in (CUT, MIN_CUT):
        return CutScorer(target)
    if target in (MIN_COVER, MAX_IND_SET, MAX_CLIQUE, MIN_DOM_SET):
        return SetScorer(target)
    raise NotImplementedError(f"Invalid optimization target: {target}")


class ProblemSpinSystemOracle:
    """SpinSystemBase (spinsystem.py:81-559) for every scorer and all 13 observables; ExtraAction.NONE,
    memory_length None, unbiased graphs.  Like the reference constructor (:168), __init__ runs one
    reset, so the first caller-visible reset already sees the scorer's normalisers of that graph."""

    def __init__(self, matrix, max_steps, target=CUT, observables=DEFAULT_OBSERVABLES, reward_signal="BLS",
                 norm_rewards=True, basin_reward=None, stag_punishment=None, reversible_spins=True,
                 spin_basis="SIGNED", horizon_length=None, stopping="NORMAL", init_reset=True, rng=None):
        assert observables[0] == SPIN_STATE, "First observable must be Observation.SPIN_STATE."
        self.matrix = np.asarray(matrix, dtype=np.float64)
        self.n_spins = self.matrix.shape[0]
        self.max_steps = max_steps
        self.observables = list(enumerate(observables))
        self.reward_signal = reward_signal
        self.norm_rewards = norm_rewards
        self.basin_reward = basin_reward
        self.stag_punishment = stag_punishment
        self.reversible_spins = reversible_spins
        self.spin_basis = spin_basis
        self.horizon_length = horizon_length if horizon_length is not None else max_steps
        self.stopping = stopping
        self.scorer = make_scorer(target)
        if self.scorer.cut_like and any(o in VALIDITY_MASK_OBSERVABLES for o in observables):
            raise TypeError("validity-mask observables with a cut target (TypeError in the reference)")
        if init_reset:
            self.reset(rng=rng)

    def _signed(self, spins):   # spinsystem.py:595-606
        spins = np.asarray(spins)
        if self.spin_basis == "BINARY":
            if not np.isin(spins, [0, 1]).all():
                raise Exception("SpinSystem is configured for binary spins ([0,1]).")
            return 2 * spins - 1
        if not np.isin(spins, [-1, 1]).all():
            raise Exception("SpinSystem is configured for signed spins ([-1,1]).")
        return spins

    def reset(self, spins=None, rng=None):
        """spinsystem.py:183-259 + _reset_state :283-330."""
        n, J, sc = self.n_spins, self.matrix, self.scorer
        self.current_step = 0
        self.early_stopping = 0
        if not sc.set_mlr(J):   # :203-213 (nonzero check only fails for cut problems)
            raise ValueError("graph has no nonzero local reward")
        state = np.zeros((len(self.observables), n))
        if spins is None:
            if self.reversible_spins:
                rng = rng if rng is not None else np.random
                state[0, :] = 2 * rng.randint(2, size=n) - 1
            else:
                state[0, :] = -1
        else:
            state[0, :] = self._signed(spins)
        s = state[0, :]
        qm = sc.qmask(s, J)
        # the observables are written BEFORE set_invalidity_normalizer (:216 vs :219): the validity
        # difference uses the normaliser left by the previous reset (1 at construction)
        for idx, obs in self.observables:
            if obs == IMMEDIATE_QUALITY_CHANGE:
                state[idx, :] = qm / sc.mlr
            elif obs == IMMEDIATE_VALIDITY_DIFFERENCE:
                state[idx, :] = sc.imask(s, J) / sc.inorm
            elif obs == IMMEDIATE_VALIDITY_CHANGE:
                state[idx, :] = sc.vmask(s, J)
            elif obs == NUMBER_OF_QUALITY_IMPROVEMENTS:
                state[idx, :] = np.sum(qm > 0) / n
            elif obs == NUMBER_OF_VALIDITY_IMPROVEMENTS:
                state[idx, :] = np.sum(sc.imask(s, J) > 0) / n   # '> 0' at reset, '< 0' in step
            elif obs == VALIDITY_BIT:
                state[idx, :] = sc.valid(s, J)
        self.state = state
        sc.set_normalisers(J)                                     # :219-221
        self.score = sc.score(s, J)
        self.normalized_score = sc.nscore(s, J)
        self.solution = sc.solution(s, J)
        self.best_score = self.score
        self.best_score_normalized = self.normalized_score
        self.best_obs_score = self.score
        self.best_obs_score_normalized = self.normalized_score
        self.best_solution = self.solution
        self.best_spins = s.copy()
        self.best_obs_spins = s.copy()
        self.history = HistoryBuffer() if (self.stag_punishment is not None or
                                           self.basin_reward is not None) else None
        return self.get_observation()

    def step(self, action):
        """spinsystem.py:355-559."""
        n, J, sc = self.n_spins, self.matrix, self.scorer
        done = False
        rew = 0
        self.current_step += 1
        self.early_stopping += 1
        if self.current_step > self.max_steps:
            raise NotImplementedError("The environment has already returned done.")
        new_state = np.copy(self.state)
        delta = sc.score_mask(self.state[0, :], J)[action]
        delta_n = sc.nscore_mask(self.state[0, :], J)[action]
        new_state[0, action] = -self.state[0, action]
        self.score += delta
        self.normalized_score += delta_n
        self.state = new_state
        s = self.state[0, :]
        qm = sc.qmask(s, J)
        im = None if sc.cut_like else sc.imask(s, J)
        smask = sc.score_mask(s, J)
        if self.score > self.best_obs_score:
            self.early_stopping = 0
            if self.reward_signal == "BLS":
                rew = (self.normalized_score - self.best_obs_score_normalized
                       if self.norm_rewards else self.score - self.best_obs_score)
        if self.reward_signal == "DENSE":
            rew = delta_n if self.norm_rewards else delta
        new = True
        if self.history is not None:
            new = self.history.update(action)
        if self.stag_punishment is not None and not new:
            rew -= self.stag_punishment
        if self.basin_reward is not None and np.all(smask <= 0) and new:
            rew += self.basin_reward
        if self.score > self.best_score:
            self.best_score = self.score
            self.best_score_normalized = self.normalized_score
            self.best_spins = s.copy()
            self.best_solution = sc.solution(self.best_spins, J)
        self.best_obs_score = self.best_score
        self.best_obs_score_normalized = self.best_score_normalized
        self.best_obs_spins = self.best_spins.copy()
        for idx, obs in self.observables:
            if obs == IMMEDIATE_QUALITY_CHANGE:
                self.state[idx, :] = qm / sc.mlr
            elif obs == TIME_SINCE_FLIP:
                self.state[idx, :] += (1. / self.max_steps)
                self.state[idx, action] = 0
            elif obs == IMMEDIATE_VALIDITY_DIFFERENCE:
                self.state[idx, :] = im / sc.inorm
            elif obs == IMMEDIATE_VALIDITY_CHANGE:
                self.state[idx, :] = sc.vmask(s, J)
            elif obs == EPISODE_TIME:
                self.state[idx, :] += (1. / self.max_steps)
            elif obs == TERMINATION_IMMANENCY:
                self.state[idx, :] = max(0, ((self.current_step - self.max_steps) / self.horizon_length) + 1)
            elif obs == NUMBER_OF_QUALITY_IMPROVEMENTS:
                self.state[idx, :] = np.sum(qm > 0) / n
            elif obs == DISTANCE_FROM_BEST_SOLUTION:
                self.state[idx, :] = np.abs(sc.quality(s, J) - sc.quality(self.best_spins, J)) / sc.mlr
            elif obs == NUMBER_OF_VALIDITY_IMPROVEMENTS:
                self.state[idx, :] = np.sum(im < 0) / n
            elif obs == DISTANCE_FROM_BEST_STATE:
                self.state[idx, :] = np.count_nonzero(self.best_obs_spins - s)
            elif obs == GLOBAL_VALIDITY_DIFFERENCE:
                self.state[idx, :] = (sc.inv(s, J) - sc.inv(self.best_spins, J)) / sc.inorm
            elif obs == VALIDITY_BIT:
                self.state[idx, :] = sc.valid(s, J)
        if self.current_step == self.max_steps:
            done = True
        if self.stopping == "EARLY" and self.early_stopping == 15:
            done = True
        if self.stopping == "QUARTER" and self.current_step == self.max_steps // 4:
            done = True
        if not self.reversible_spins and not np.any(self.state[0, :] < 0):
            done = True
        return self.get_observation(), rew, done, None

    def get_observation(self):
        state = self.state.copy()
        if self.spin_basis == "BINARY":
            state[0, :] = (1 - state[0, :]) / 2
        return np.vstack((state, self.matrix))

    def state_rows(self):
        return self.get_observation()[:len(self.observables)]


def greedy_action(env):
    """Greedy.step's choice (src/agents/solver.py:110-127) on the env's scorer: argmax of the score mask
    (irreversible: over spins still at -1); None when that change is negative (the solver stops)."""
    m = np.asarray(env.scorer.score_mask(env.state[0, :], env.matrix), dtype=np.float64)
    if not env.reversible_spins:
        m = np.where(env.state[0, :] == -1, m, np.finfo(np.float64).min)
    a = int(m.argmax())
    return None if m[a] < 0 else a
