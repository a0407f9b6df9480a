"""Single-episode SpinSystem with the reference's interface (src/envs/spinsystem.py:29-607),
running on the batched HIP engine with B = 1.

For code written against `src.envs.core.make("SpinSystem", ...)`: same constructor
arguments, `reset(spins=None)` / `step(action)` returning the reference's float64
observation [n_obs + N, N] (state rows + adjacency), and the attributes callers read
(state, score, best_score, best_solution, best_spins, current_step, scorer, ...).
Each call synchronises with the device; batched callers use VecSpinSystem.
"""
from collections import namedtuple

import numpy as np
import torch

from ..graphs import GraphStore
from .batched import VecSpinSystem
from .utils import (DEFAULT_OBSERVABLES, EdgeType, ExtraAction, GraphGenerator, OptimisationTarget, RandomGraphGenerator,
                    RewardSignal, SpinBasis, Stopping)

ActionResult = namedtuple("action_result", ("snapshot", "observation", "reward", "is_done", "info"))


class DeviceScorer:
    """Host-side view of the env's ScoreSolver (score_solver.py:11-172): the normalisers the device computed
    for the current graph (read back after every call).  For the cut targets it also offers the numpy score
    helpers callers such as the reference's Greedy solver use; the set problems' masks live on the device
    only (VecSpinSystem.greedy_actions evaluates them there)."""

    def __init__(self, target, scalars):
        self.target = target
        self._max_local_reward = float(scalars["max_local_reward"])
        self._solution_quality_normalizer = float(scalars["quality_normalizer"])
        self._invalidity_normalizer = float(scalars["invalidity_normalizer"])
        self._lower_bound = float(scalars["lower_bound"])

    def _cut_only(self):
        if self.target not in (OptimisationTarget.CUT, OptimisationTarget.MIN_CUT):
            raise NotImplementedError(f"{self.target}: scorer masks are evaluated on the device "
                                      "(VecSpinSystem.greedy_actions / obs rows)")

    def get_solution(self, spins, matrix):
        self._cut_only()
        return (1 / 4) * np.sum(np.multiply(matrix, 1 - np.outer(spins, spins)))

    def get_solution_quality(self, spins, matrix):
        if self.target == OptimisationTarget.MIN_CUT:
            return max(0, self._solution_quality_normalizer) - self.get_solution(spins, matrix)
        return self.get_solution(spins, matrix) + abs(min(0, self._lower_bound))

    get_score = get_solution_quality

    def get_normalized_score(self, spins, matrix):
        return self.get_solution_quality(spins, matrix) / self._solution_quality_normalizer

    def get_score_mask(self, spins, matrix):
        self._cut_only()
        g = spins * (matrix @ spins)
        return g if self.target == OptimisationTarget.CUT else -g

    get_solution_quality_mask = get_score_mask

    def get_normalized_score_mask(self, spins, matrix):
        return self.get_score_mask(spins, matrix) / self._solution_quality_normalizer


class SpinSystemFactory:
    @staticmethod
    def get(graph_generator=None, max_steps=20, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.DENSE,
            extra_action=ExtraAction.PASS, optimisation_target=OptimisationTarget.ENERGY,
            spin_basis=SpinBasis.SIGNED, norm_rewards=False, memory_length=None, horizon_length=None,
            stag_punishment=None, basin_reward=None, reversible_spins=True, init_snap=None, seed=None,
            stopping=Stopping.NORMAL):
        """spinsystem.py:29-48 (same defaults)."""
        return SpinSystemBase(graph_generator, max_steps, observables, reward_signal, extra_action,
                              optimisation_target, spin_basis, norm_rewards, memory_length, horizon_length,
                              stag_punishment, basin_reward, reversible_spins, init_snap, seed, stopping)


class SpinSystemBase:
    class action_space:
        def __init__(self, n_actions):
            self.n = n_actions
            self.actions = np.arange(self.n)

        def sample(self, n=1):
            return np.random.choice(self.actions, n)

    class observation_space:
        def __init__(self, n_spins, n_observables):
            self.shape = [n_spins, n_observables]

    def __init__(self, graph_generator=None, max_steps=20, observables=DEFAULT_OBSERVABLES,
                 reward_signal=RewardSignal.DENSE, extra_action=ExtraAction.PASS,
                 optimisation_target=OptimisationTarget.ENERGY, spin_basis=SpinBasis.SIGNED, norm_rewards=False,
                 memory_length=None, horizon_length=None, stag_punishment=None, basin_reward=None,
                 reversible_spins=False, init_snap=None, seed=None, stopping=Stopping.NORMAL, device="cuda"):
        if seed is not None:
            np.random.seed(seed)
        if graph_generator is None:
            graph_generator = RandomGraphGenerator(n_spins=20, edge_type=EdgeType.DISCRETE)
        assert isinstance(graph_generator, GraphGenerator), "graph_generator must be a GraphGenerator implementation."
        self.gg = graph_generator
        self.n_spins = self.gg.n_spins
        self.max_steps = max_steps
        self.observables = list(enumerate(observables))
        self.extra_action = extra_action
        self.reward_signal = reward_signal
        self.norm_rewards = norm_rewards
        self.optimisation_target = optimisation_target
        self.spin_basis = spin_basis
        self.memory_length = memory_length
        self.horizon_length = horizon_length if horizon_length is not None else max_steps
        self.stag_punishment = stag_punishment
        self.basin_reward = basin_reward
        self.reversible_spins = reversible_spins
        self.stopping_type = stopping
        self.n_actions = self.n_spins
        self.action_space = self.action_space(self.n_actions)
        self.observation_space = self.observation_space(self.n_spins, len(self.observables))
        self.device = torch.device(device)
        self._env_args = dict(observables=observables, reward_signal=reward_signal, extra_action=extra_action,
                              optimisation_target=optimisation_target, spin_basis=spin_basis,
                              norm_rewards=norm_rewards, memory_length=memory_length,
                              horizon_length=horizon_length, stag_punishment=stag_punishment,
                              basin_reward=basin_reward, reversible_spins=reversible_spins, stopping=stopping)
        self._matrix_key = None
        self._vec = None
        self.reset()

    # ---- helpers ----
    def _bind_graph(self, matrix):
        key = id(matrix)
        if key != self._matrix_key or self._vec is None:
            store = GraphStore.from_dense([np.asarray(matrix, dtype=np.float64)], device=self.device)
            if self._vec is None:
                self._vec = VecSpinSystem(store, 1, self.max_steps, want_f64=True, **self._env_args)
            else:  # same episode state: the scorer's normalisers carry over like the reference's (:216-219)
                self._vec.graphs = store
            self._matrix_key = key
        self.matrix = matrix
        self.matrix_obs = matrix

    def _sync(self):
        st = self._vec.read(spins=True, best_spins=True)
        self.scorer = DeviceScorer(self.optimisation_target, {k: v[0].item() for k, v in st.items()
                                                              if k not in ("spins", "best_spins")})
        self.current_step = int(st["current_step"][0].item())
        self.score = float(st["score"][0].item())
        self.normalized_score = float(st["normalized_score"][0].item())
        self.best_score = float(st["best_score"][0].item())
        self.best_score_normalized = float(st["best_score_normalized"][0].item())
        self.best_solution = float(st["best_solution"][0].item())
        self.best_spins = st["best_spins"][0].cpu().numpy().astype(np.float64)
        self.best_obs_score = self.best_score
        self.best_obs_score_normalized = self.best_score_normalized
        self.best_obs_spins = self.best_spins.copy()
        rows = self._vec.obs_f64[0].cpu().numpy()
        self.state = rows.copy()
        if self.spin_basis == SpinBasis.BINARY:  # self.state keeps signed spins (spinsystem.py:561-569)
            self.state[0, :] = st["spins"][0].cpu().numpy().astype(np.float64)
        self._obs_rows = rows

    def _format_spins_to_signed(self, spins):
        """spinsystem.py:595-606"""
        spins = np.asarray(spins)
        if self.spin_basis == SpinBasis.BINARY:
            if not np.isin(spins, [0, 1]).all():
                raise Exception("SpinSystem is configured for binary spins ([0,1]).")
            spins = 2 * spins - 1
        elif self.spin_basis == SpinBasis.SIGNED:
            if not np.isin(spins, [-1, 1]).all():
                raise Exception("SpinSystem is configured for signed spins ([-1,1]).")
        return spins

    # ---- reference API ----
    def reset(self, spins=None):
        """spinsystem.py:183-259.  A graph with no nonzero local reward is redrawn (:203-211)."""
        for _ in range(1000):
            matrix = self.gg.get()
            self._bind_graph(matrix)
            cut_like = self.optimisation_target in (OptimisationTarget.CUT, OptimisationTarget.MIN_CUT)
            if not cut_like or int(self._vec.graphs.valid[0].item()):  # set problems: never redrawn
                break
        else:
            raise ValueError("graph generator keeps returning graphs with no nonzero local reward")
        if spins is None:
            if self.reversible_spins:
                sp = 2 * np.random.randint(2, size=self.n_spins) - 1   # spinsystem.py:294
            else:
                sp = -np.ones(self.n_spins, dtype=np.int64)
        else:
            sp = self._format_spins_to_signed(spins)
        self._vec.reset(graph_ids=[0], spins=np.asarray(sp)[None])
        self._vec.check_errors()
        self._sync()
        self.solution = self.best_solution
        return self.get_observation()

    def step(self, action):
        """spinsystem.py:355-559"""
        if self.current_step >= self.max_steps:
            print("The environment has already returned done. Stop it!")
            raise NotImplementedError
        a = torch.tensor([int(action)], dtype=torch.int32, device=self.device)
        _, rew, done = self._vec.step(a)
        self._vec.check_errors()
        rew = float(rew[0].item())
        done = bool(done[0].item())
        self._sync()
        return self.get_observation(), rew, done, None

    def get_observation(self):
        """spinsystem.py:561-574: vstack(state rows (basis-converted), adjacency)."""
        return np.vstack((self._obs_rows, self.matrix_obs))

    def get_allowed_action_states(self):
        """spinsystem.py:576-593"""
        if self.reversible_spins:
            return (0, 1) if self.spin_basis == SpinBasis.BINARY else (-1, 1)
        return 0 if self.spin_basis == SpinBasis.BINARY else -1

    def seed(self, seed):
        return self.seed

    def set_seed(self, seed):
        self.seed = seed
        np.random.seed(seed)
