"""Batched SpinSystem: B concurrent episodes on one GPU (libecohip env kernels).

The reference steps one `SpinSystemBase` at a time from a Python loop
(dqn.py:273-327, experiments/utils.py:169-201).  `VecSpinSystem` holds B episodes
in one device state buffer and advances all of them with one kernel launch; the
per-episode semantics are exactly spinsystem.py:183-559 (bit-exact f64 rewards and
observations, see tests/test_env_gpu.py).
"""
import ctypes

import numpy as np
import torch

from .. import _lib
from .utils import (DEFAULT_OBSERVABLES, ExtraAction, Observable, OptimisationTarget, RewardSignal,
                    SpinBasis, Stopping)


def make_config(n_spins, max_steps, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.DENSE,
                extra_action=ExtraAction.PASS, optimisation_target=OptimisationTarget.ENERGY,
                spin_basis=SpinBasis.SIGNED, norm_rewards=False, memory_length=None, horizon_length=None,
                stag_punishment=None, basin_reward=None, reversible_spins=True, stopping=Stopping.NORMAL,
                **_ignored):
    """env_args (spinsystem.py:29-48 defaults) -> eco_env_config."""
    if optimisation_target == OptimisationTarget.ENERGY:
        # the reference factory has no ENERGY branch (score_solver.py:866-885)
        raise NotImplementedError(f"Invalid optimization target: {optimisation_target} and biased False")
    if extra_action != ExtraAction.NONE:
        raise NotImplementedError("eco_hip runs ExtraAction.NONE only (PASS shape-breaks the reference "
                                  "score mask, spinsystem.py:141-142,393)")
    if memory_length is not None:
        raise NotImplementedError("finite memory_length is not on the hot path")
    obs = list(observables)
    assert obs[0] == Observable.SPIN_STATE, "First observable must be Observation.SPIN_STATE."
    if len(obs) > 13:
        raise ValueError("at most 13 observables")
    if optimisation_target in (OptimisationTarget.CUT, OptimisationTarget.MIN_CUT) and any(
            o in (Observable.IMMEDIATE_VALIDITY_DIFFERENCE, Observable.IMMEDIATE_VALIDITY_CHANGE,
                  Observable.NUMBER_OF_VALIDITY_IMPROVEMENTS) for o in obs):
        # the cut scorers return the invalidity mask as a python list (score_solver.py:403-407, :489-493)
        raise TypeError("unsupported operand type(s) for /: 'list' and 'int' (validity-mask observable "
                        "with a cut target)")
    if spin_basis not in (SpinBasis.SIGNED, SpinBasis.BINARY):
        raise Exception("Unrecognised SpinBasis")
    c = _lib.EnvConfig()
    c.n_spins = n_spins
    c.max_steps = max_steps
    c.n_obs = len(obs)
    for i, o in enumerate(obs):
        c.obs_ids[i] = o.value
    c.reward_signal = reward_signal.value
    c.norm_rewards = int(bool(norm_rewards))
    c.reversible_spins = int(bool(reversible_spins))
    c.spin_basis = spin_basis.value
    c.stopping = stopping.value
    c.has_basin_reward = int(basin_reward is not None)
    c.basin_reward = float(basin_reward) if basin_reward is not None else 0.0
    c.has_stag_punishment = int(stag_punishment is not None)
    c.stag_punishment = float(stag_punishment) if stag_punishment is not None else 0.0
    c.horizon_length = int(horizon_length if horizon_length is not None else max_steps)
    c.optimisation_target = optimisation_target.value
    return c


class VecSpinSystem:
    """B episodes over graphs of a GraphStore, for any OptimisationTarget scorer except ENERGY.

    reset(graph_ids, spins=None, mask=None, seed=0) and step(actions) return the
    fp32 node features obs_x [B, N, W] (W = 8, or 16 beyond 8 observables) that the MPNN
    consumes (obs.float() of the reference observation rows, dqn.py:282); pass want_f64=True
    to also fill obs_f64 [B, n_obs, N] (the reference's float64 rows, for parity checks)."""

    def __init__(self, graphs, n_envs, max_steps, want_f64=False, stream=None, **env_args):
        self.graphs = graphs
        self.n_envs = n_envs
        self.n_spins = graphs.n_spins
        self.max_steps = max_steps
        self.env_args = env_args
        self.cfg = make_config(graphs.n_spins, max_steps, **env_args)
        self.n_obs = self.cfg.n_obs
        self.reversible_spins = bool(self.cfg.reversible_spins)
        self.spin_basis = env_args.get("spin_basis", SpinBasis.SIGNED)
        dev = graphs.device
        nbytes = _lib.lib.eco_env_state_bytes(ctypes.byref(self.cfg), n_envs)
        if nbytes == 0:
            raise ValueError(_lib.last_error())
        self.state = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        self.obs_x = torch.zeros(n_envs, self.n_spins, _lib.obs_x_stride(self.n_obs), dtype=torch.float32,
                                 device=dev)
        self.obs_f64 = (torch.zeros(n_envs, self.n_obs, self.n_spins, dtype=torch.float64, device=dev)
                        if want_f64 else None)
        self.rewards = torch.zeros(n_envs, dtype=torch.float64, device=dev)
        self.dones = torch.zeros(n_envs, dtype=torch.uint8, device=dev)
        self.graph_ids = torch.zeros(n_envs, dtype=torch.int32, device=dev)
        self.scalars = torch.zeros(n_envs, _lib.ECO_ENV_SCALARS, dtype=torch.float64, device=dev)
        self.stream = stream

    def _s(self):
        return _lib.stream_ptr(self.stream)

    def _upload(self, a, dtype):
        """Host or device array -> contiguous device tensor of `dtype`, without a host synchronisation: host data
        goes through pinned memory (torch's caching host allocator keeps the block until the copy has run) and
        a non-blocking copy on the current stream."""
        dev = self.graphs.device
        if isinstance(a, torch.Tensor) and a.is_cuda:
            return a.to(device=dev, dtype=dtype).contiguous()
        t = torch.as_tensor(np.asarray(a.cpu() if isinstance(a, torch.Tensor) else a)).to(dtype).contiguous()
        return t.pin_memory().to(dev, non_blocking=True)

    def reset(self, graph_ids=None, spins=None, mask=None, seed=0, obs_out=None):
        mk = None
        if mask is not None:
            mk = self._upload(mask, torch.uint8)
        if graph_ids is not None:
            gi = self._upload(graph_ids, torch.int32)
            if mask is None:
                self.graph_ids.copy_(gi)
            else:  # graph_ids[mask] = gi[mask] without the host round trip of boolean indexing
                self.graph_ids.copy_(torch.where(mk.bool(), gi, self.graph_ids))
        sp = None
        if spins is not None:
            sp = self._upload(spins, torch.int8)
        if obs_out is not None:
            self.obs_x = obs_out
        _lib.check(_lib.lib.eco_env_reset(ctypes.byref(self.cfg), ctypes.byref(self.graphs.gs),
                                          _lib.ptr(self.state), self.n_envs, _lib.ptr(self.graph_ids),
                                          _lib.ptr(sp), _lib.ptr(mk), ctypes.c_uint64(seed),
                                          _lib.ptr(self.obs_x), _lib.ptr(self.obs_f64), self._s()))
        if mask is None:
            self.dones.zero_()
        else:
            self.dones.masked_fill_(mk.bool(), 0)
        return self.obs_x

    def step(self, actions, obs_out=None):
        """Advance every episode by its action.  obs_out: optional [B, N, 8] buffer that
        receives the new features (self.obs_x is then left untouched, so a caller can
        keep s and s' without a copy); it becomes self.obs_x afterwards."""
        a = actions if actions.dtype == torch.int32 else actions.to(torch.int32)
        out = self.obs_x if obs_out is None else obs_out
        _lib.check(_lib.lib.eco_env_step(ctypes.byref(self.cfg), ctypes.byref(self.graphs.gs),
                                         _lib.ptr(self.state), self.n_envs, _lib.ptr(a.contiguous()),
                                         _lib.ptr(self.rewards), _lib.ptr(self.dones), _lib.ptr(out),
                                         _lib.ptr(self.obs_f64), self._s()))
        self.obs_x = out
        return self.obs_x, self.rewards, self.dones

    def greedy_actions(self, actions_out=None):
        """Greedy solver step (solver.py:100-131): argmax of the scorer's score mask per episode;
        episodes without a non-negative change are marked done."""
        out = actions_out if actions_out is not None else torch.empty(self.n_envs, dtype=torch.int32,
                                                                      device=self.graphs.device)
        _lib.check(_lib.lib.eco_env_greedy_actions(ctypes.byref(self.cfg), ctypes.byref(self.graphs.gs),
                                                   _lib.ptr(self.state), self.n_envs, _lib.ptr(out), self._s()))
        return out

    def check_errors(self):
        _lib.check(_lib.lib.eco_check_errors(self._s()))

    def read(self, spins=False, best_spins=False):
        """-> dict of per-episode attributes (dqn.py:564-566 BEST metric reads best_score/best_solution)."""
        dev = self.graphs.device
        sp = torch.zeros(self.n_envs, self.n_spins, dtype=torch.int8, device=dev) if spins else None
        bs = torch.zeros(self.n_envs, self.n_spins, dtype=torch.int8, device=dev) if best_spins else None
        _lib.check(_lib.lib.eco_env_read(ctypes.byref(self.cfg), _lib.ptr(self.state), self.n_envs,
                                         _lib.ptr(self.scalars), _lib.ptr(sp), _lib.ptr(bs), self._s()))
        out = self.scalar_fields(self.scalars)
        if spins:
            out["spins"] = sp
        if best_spins:
            out["best_spins"] = bs
        return out

    @staticmethod
    def scalar_fields(s):
        """The named columns of an [n_envs, ECO_ENV_SCALARS] float64 scalar block (eco_env_read), device or host."""
        return dict(current_step=s[:, 0], score=s[:, 1], normalized_score=s[:, 2], best_score=s[:, 3],
                    best_score_normalized=s[:, 4], best_solution=s[:, 5], hamming=s[:, 6], done=s[:, 7],
                    max_local_reward=s[:, 8], quality_normalizer=s[:, 9], invalidity_normalizer=s[:, 10],
                    lower_bound=s[:, 11], set_size=s[:, 12], invalidity=s[:, 13])

    def allowed_action_value(self):
        """get_allowed_action_states (spinsystem.py:576-593) for irreversible envs: the
        feature-0 value of still-flippable vertices."""
        return 0.0 if self.spin_basis == SpinBasis.BINARY else -1.0
