"""CPU restatement of the reference MaxCut SpinSystem env (TEST INFRASTRUCTURE ONLY).

This module is the parity oracle and the CPU baseline ("port") for the env step.
Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may import
it -- it is never on the product path (the product is the HIP kernel behind
`libecohip.so`).

It restates, op for op, the reference's per-step work so that its timing is a
faithful "reference-cost" baseline:
  * `calculate_cut`          = src/envs/utils.py:90-94   (dense 1/4 sum J*(1-s s^T))
  * `calculate_cut_changes`  = src/envs/utils.py:97-102  (s * (J @ s), numba-jitted upstream)
  * MaximumCutUnbiasedScorer = src/envs/score_solver.py:343-419 (+ MaximizationProblem :175-200)
  * HistoryBuffer            = src/envs/utils.py:438-464
  * SpinSystemBase.reset     = src/envs/spinsystem.py:183-259, _reset_state :283-330
  * SpinSystemBase.step      = src/envs/spinsystem.py:355-559
  * get_observation          = src/envs/spinsystem.py:561-574

Pinned against the reference itself: tests/golden/make_golden.py imports the
reference (identity numba.jit shim) and records trajectories; tests/test_oracle_golden.py
checks this file against them bit for bit.
"""
import numpy as np

# Observable enum values of the reference (src/envs/utils.py:48-65).
SPIN_STATE = 1
IMMEDIATE_QUALITY_CHANGE = 2
TIME_SINCE_FLIP = 5
TERMINATION_IMMANENCY = 7
NUMBER_OF_QUALITY_IMPROVEMENTS = 8
DISTANCE_FROM_BEST_SOLUTION = 10
DISTANCE_FROM_BEST_STATE = 11

# src/envs/utils.py:68-74
DEFAULT_OBSERVABLES = [SPIN_STATE, IMMEDIATE_QUALITY_CHANGE, TIME_SINCE_FLIP,
                       DISTANCE_FROM_BEST_SOLUTION, DISTANCE_FROM_BEST_STATE,
                       NUMBER_OF_QUALITY_IMPROVEMENTS, TERMINATION_IMMANENCY]
S2V_OBSERVABLES = [SPIN_STATE]          # experiments/train_eco.py:311-315


def calculate_cut(spins, matrix):
    """src/envs/utils.py:90-94"""
    return (1 / 4) * np.sum(np.multiply(matrix, 1 - np.outer(spins, spins)))


def calculate_cut_changes(spins, matrix):
    """src/envs/utils.py:97-102 (numba @jit upstream; identical values for integer weights)."""
    return spins * (matrix @ spins)


class HistoryBuffer:
    """src/envs/utils.py:438-464: set of flipped-vertex sets, bucketed by size.
    The initial (empty) set is never inserted, so the first return to the start
    state counts as new."""

    def __init__(self):
        self.buffer = {}
        self.cur = frozenset()

    def update(self, action):
        nxt = set(self.cur)
        if action in nxt:
            nxt.remove(action)
        else:
            nxt.add(action)
        nxt = frozenset(nxt)
        bucket = self.buffer.setdefault(len(nxt), set())
        self.cur = nxt
        if nxt in bucket:
            return False
        bucket.add(nxt)
        return True


class SpinSystemOracle:
    """MaxCut (OptimisationTarget.CUT, unbiased, ExtraAction.NONE) SpinSystem."""

    def __init__(self, matrix, max_steps, observables=DEFAULT_OBSERVABLES,
                 reward_signal="BLS", norm_rewards=True, basin_reward=None,
                 stag_punishment=None, reversible_spins=True, spin_basis="SIGNED",
                 horizon_length=None, stopping="NORMAL"):
        # spinsystem.py:116 -- first observable must be the spin state
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

    # ---- MaximumCutUnbiasedScorer (score_solver.py:343-419) ----
    def _set_normalisers(self):
        J = self.matrix
        self.qn = max(1, np.sum(np.multiply(J, (J > 0))) / 2)          # :353-357
        self.lb = min(0, np.sum(np.multiply(J, (J < 0))) / 2)          # :359-365

    def _quality(self, spins):                                          # :196-200, :377-387
        return calculate_cut(spins, self.matrix) + abs(min(0, self.lb))

    def _format_spins_to_signed(self, spins):                           # spinsystem.py:595-606
        spins = np.asarray(spins)
        if self.spin_basis == "BINARY":
            if not np.isin(spins, [0, 1]).all():
                raise Exception("SpinSystem is configured for binary spins ([0,1]).")
            return 2 * spins - 1
        if not np.isin(spins, [-1, 1]).all():
            raise Exception("SpinSystem is configured for signed spins ([-1,1]).")
        return spins

    def reset(self, spins=None, rng=None):
        """spinsystem.py:183-259. `rng` stands in for the global np.random stream
        (spins at :292-294 are `2*np.random.randint(2, size=N) - 1`)."""
        n = self.n_spins
        self.current_step = 0
        self.early_stopping = 0
        empty = np.array([-1] * n, dtype=np.float64)
        lra = calculate_cut_changes(empty, self.matrix)
        lra = lra[np.nonzero(lra)]
        if lra.size == 0:
            # The reference recurses into reset() to draw another graph (:208-211);
            # a fixed graph can never become valid, so this is an error here.
            raise ValueError("graph has no edges with nonzero local reward")
        self.mlr = np.max(lra)                                           # score_solver.py:367-375
        state = np.zeros((len(self.observables), n))
        if spins is None:
            if self.reversible_spins:
                rng = rng if rng is not None else np.random
                state[0, :] = 2 * rng.randint(2, size=n) - 1
            else:
                state[0, :] = -1
        else:
            state[0, :] = self._format_spins_to_signed(spins)
        state = state.astype("float")
        g = calculate_cut_changes(state[0, :], self.matrix)
        for idx, obs in self.observables:                                # :308-328
            if obs == IMMEDIATE_QUALITY_CHANGE:
                state[idx, :] = g / self.mlr
            elif obs == NUMBER_OF_QUALITY_IMPROVEMENTS:
                state[idx, :] = np.sum(g > 0) / n
        self.state = state
        self._set_normalisers()                                          # :219-221
        self.score = self._quality(state[0, :])                          # :224
        self.normalized_score = self.score / self.qn                     # :225, :190-194
        self.solution = calculate_cut(state[0, :], self.matrix)          # :226
        self.best_score = self.score
        self.best_score_normalized = self.normalized_score
        self.best_obs_score = self.score
        self.best_obs_score_normalized = self.normalized_score
        self.best_solution = self.solution
        self.best_spins = state[0, :].copy()
        self.best_obs_spins = state[0, :].copy()
        self.history = HistoryBuffer() if (self.stag_punishment is not None or
                                           self.basin_reward is not None) else None
        return self.get_observation()

    def step(self, action):
        """spinsystem.py:355-559 (ExtraAction.NONE, memory_length None)."""
        n = self.n_spins
        done = False
        rew = 0
        self.current_step += 1
        self.early_stopping += 1
        if self.current_step > self.max_steps:                          # :365-367
            raise NotImplementedError("The environment has already returned done.")
        new_state = np.copy(self.state)
        delta = calculate_cut_changes(self.state[0, :], self.matrix)[action]               # :393
        delta_n = (calculate_cut_changes(self.state[0, :], self.matrix) / self.qn)[action]  # :394
        new_state[0, action] = -self.state[0, action]
        self.score += delta
        self.normalized_score += delta_n                                 # :400 accumulated
        self.state = new_state
        g = calculate_cut_changes(self.state[0, :], self.matrix)         # :414
        g_score = calculate_cut_changes(self.state[0, :], self.matrix)   # :416
        if self.score > self.best_obs_score:                             # :418-424
            self.early_stopping = 0
            if self.reward_signal == "BLS":
                rew = (self.normalized_score - self.best_obs_score_normalized
                       if self.norm_rewards else self.score - self.best_obs_score)
        if self.reward_signal == "DENSE":                                # :437-438
            rew = delta_n if self.norm_rewards else delta
        if self.history is not None:
            new = self.history.update(action)                            # :443-444
        if self.stag_punishment is not None and not new:                 # :446-448
            rew -= self.stag_punishment
        if self.basin_reward is not None and np.all(g_score <= 0) and new:  # :450-457
            rew += self.basin_reward
        if self.score > self.best_score:                                 # :459-463
            self.best_score = self.score
            self.best_score_normalized = self.normalized_score
            self.best_spins = self.state[0, :].copy()
            self.best_solution = calculate_cut(self.best_spins, self.matrix)
        self.best_obs_score = self.best_score                            # :474-477
        self.best_obs_score_normalized = self.best_score_normalized
        self.best_obs_spins = self.best_spins.copy()
        for idx, obs in self.observables:                                # :486-535
            if obs == IMMEDIATE_QUALITY_CHANGE:
                self.state[idx, :] = g / self.mlr
            elif obs == TIME_SINCE_FLIP:
                self.state[idx, :] += (1. / self.max_steps)
                self.state[idx, action] = 0
            elif obs == TERMINATION_IMMANENCY:
                self.state[idx, :] = max(0, ((self.current_step - self.max_steps) / self.horizon_length) + 1)
            elif obs == NUMBER_OF_QUALITY_IMPROVEMENTS:
                self.state[idx, :] = np.sum(g > 0) / n
            elif obs == DISTANCE_FROM_BEST_SOLUTION:
                cq = self._quality(self.state[0, :])
                bq = self._quality(self.best_spins)
                self.state[idx, :] = np.abs(cq - bq) / self.mlr
            elif obs == DISTANCE_FROM_BEST_STATE:
                self.state[idx, :] = np.count_nonzero(self.best_obs_spins - self.state[0, :])
        if self.current_step == self.max_steps:                          # :541-556
            done = True
        if self.stopping == "EARLY" and self.early_stopping == 15:
            done = True
        if self.stopping == "QUARTER" and self.current_step == self.max_steps // 4:
            done = True
        if not self.reversible_spins and not np.any(self.state[0, :] < 0):
            done = True
        return self.get_observation(), rew, done, None

    def get_observation(self):
        """spinsystem.py:561-574"""
        state = self.state.copy()
        if self.spin_basis == "BINARY":
            state[0, :] = (1 - state[0, :]) / 2
        return np.vstack((state, self.matrix))

    def state_rows(self):
        """The observation without the appended adjacency rows (obs[:n_obs])."""
        return self.get_observation()[:len(self.observables)]


def greedy_solve(env):
    """Greedy solver rule (src/agents/solver.py:100-131) on an oracle env after reset:
    flip the vertex with the largest immediate cut change until that change is negative
    (or the episode ends).  Returns the list of actions taken."""
    acts = []
    done = False
    while not done:
        mask = calculate_cut_changes(env.state[0, :], env.matrix)
        if not env.reversible_spins:
            mask = np.where(env.state[0, :] < 0, mask, np.finfo(np.float64).min)
        a = int(mask.argmax())
        if mask[a] < 0:
            break
        _, _, done, _ = env.step(a)
        acts.append(a)
    return acts
