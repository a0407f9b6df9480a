"""Replay buffer, seeding and test-metric enum of the DQN agent
(src/agents/dqn/utils.py:11-83 in the reference).

The reference's ReplayBuffer is a Python dict of full float64 observations (adjacency
included, ~662 KB per transition at N=200) sampled by a background thread
(dqn/utils.py:28-83).  Here the ring lives on the device and stores compact
transitions: fp32 node features of s and s' ([N][8]), graph id (the adjacency stays
resident in the GraphStore), action, reward, done.  add/sample are HIP kernels.
"""
import ctypes
import random
from collections import namedtuple
from enum import Enum

import numpy as np
import torch

from ... import _lib

Transition = namedtuple('Transition', ('state', 'action', 'reward', 'state_next', 'done'))


class TestMetric(Enum):
    FINAL = 1
    BEST = 2
    CUMULATIVE_REWARD = 3
    ENERGY_ERROR = 4


def set_global_seed(seed, env=None):
    """dqn/utils.py:22-26"""
    torch.manual_seed(seed)
    if env is not None and hasattr(env, "set_seed"):
        env.set_seed(seed)
    np.random.seed(seed)
    random.seed(seed)


class ReplayBuffer:
    """Device ring of compact transitions (eco_replay, include/eco_hip.h)."""

    def __init__(self, capacity, n_spins, device="cuda", seed=0, n_obs=7):
        self._capacity = int(capacity)
        self.n_spins = n_spins
        self.x_stride = _lib.obs_x_stride(n_obs)
        dev = torch.device(device)
        self.device = dev
        self.xs = torch.zeros(capacity, n_spins, self.x_stride, dtype=torch.float32, device=dev)
        self.xn = torch.zeros(capacity, n_spins, self.x_stride, dtype=torch.float32, device=dev)
        self.gid = torch.zeros(capacity, dtype=torch.int32, device=dev)
        self.act = torch.zeros(capacity, dtype=torch.int32, device=dev)
        self.rew = torch.zeros(capacity, dtype=torch.float32, device=dev)
        self.done = torch.zeros(capacity, dtype=torch.float32, device=dev)
        self.rb = _lib.Replay(self._capacity, n_spins, self.x_stride, self.xs.data_ptr(), self.xn.data_ptr(), self.gid.data_ptr(),
                              self.act.data_ptr(), self.rew.data_ptr(), self.done.data_ptr())
        self._position = 0
        self._size = 0
        self.seed = seed
        self._counter = 0
        self._out = {}

    def add_batch(self, xs, xn, graph_ids, actions, rewards, dones, stream=None):
        """ReplayBuffer.add (dqn/utils.py:39-47) for B transitions at once."""
        B = xs.shape[0]
        _lib.check(_lib.lib.eco_replay_push(ctypes.byref(self.rb), self._position, B, _lib.ptr(xs), _lib.ptr(xn),
                                            _lib.ptr(graph_ids), _lib.ptr(actions), _lib.ptr(rewards),
                                            _lib.ptr(dones), _lib.stream_ptr(stream)))
        self._position = (self._position + B) % self._capacity
        self._size = min(self._capacity, self._size + B)

    def _buffers(self, m):
        if m not in self._out:
            dev = self.device
            self._out[m] = (torch.empty(m, self.n_spins, self.x_stride, device=dev),
                            torch.empty(m, self.n_spins, self.x_stride, device=dev),
                            torch.empty(m, dtype=torch.int32, device=dev), torch.empty(m, dtype=torch.int32, device=dev),
                            torch.empty(m, device=dev), torch.empty(m, device=dev))
        return self._out[m]

    def sample(self, batch_size, device=None, stream=None):
        """ReplayBuffer.sample (dqn/utils.py:62-80): `batch_size` distinct uniform transitions
        -> (states_x, actions, rewards, states_next_x, dones, graph_ids), all on the device.
        The returned tensors are reused by the next sample of the same size."""
        xs, xn, gid, act, rew, done = self._buffers(batch_size)
        self._counter += 1
        _lib.check(_lib.lib.eco_replay_sample(ctypes.byref(self.rb), self._size, batch_size,
                                              ctypes.c_uint64(self.seed), ctypes.c_uint64(self._counter),
                                              _lib.ptr(xs), _lib.ptr(xn), _lib.ptr(gid), _lib.ptr(act),
                                              _lib.ptr(rew), _lib.ptr(done), _lib.stream_ptr(stream)))
        return xs, act, rew, xn, done, gid

    def __len__(self):
        return self._size


class CompactReplayBuffer:
    """ReplayBuffer (dqn/utils.py:28-83) for MaxCut envs that stores each transition as the env's integer
    state (include/eco_hip.h eco_replay_compact_*): ONE state per transition -- per vertex spin,
    time-since-flip count and local field in 4 B -- plus four float64 observation scalars for s and s'
    (4N + 80 B per transition, 880 B at N=200, against 64N B of fp32 feature rows for s and s').  s' is
    rebuilt from s, the action and the graph on sample, and both feature rows bit-exactly; sample() returns
    the same tuple as ReplayBuffer.sample.  Driven by the env: snapshot() after every reset, add_step()
    after every step."""

    def __init__(self, capacity, env, seed=0):
        self.env = env
        self._capacity = int(capacity)
        self.n_spins = env.n_spins
        self.x_stride = _lib.obs_x_stride(env.n_obs)
        self.device = env.graphs.device
        if env.n_envs > self._capacity:
            raise ValueError("compact replay: capacity must hold at least one batch of transitions")
        nbytes = _lib.lib.eco_replay_compact_bytes(self.n_spins, self._capacity, env.n_envs)
        if nbytes == 0:
            raise ValueError("bad compact replay size")
        self.ring = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
        self._pushed = 0  # transitions added over the buffer's life (the k-th lives in slot k % (capacity + B))
        self._size = 0
        self.seed = seed
        self._counter = 0
        self._out = {}

    def snapshot(self, mask=None, stream=None):
        """Record the env's current states (after env.reset; mask: only those episodes)."""
        mk = None if mask is None else torch.as_tensor(mask, dtype=torch.uint8, device=self.device).contiguous()
        _lib.check(_lib.lib.eco_replay_compact_snapshot(ctypes.byref(self.env.cfg), _lib.ptr(self.env.state),
                                                        self.env.n_envs, _lib.ptr(self.ring), self._capacity,
                                                        self._pushed, _lib.ptr(mk), _lib.stream_ptr(stream)))

    def add_step(self, actions, rewards, dones, stream=None):
        """ReplayBuffer.add (dqn/utils.py:39-47) of the transitions of the env step just taken."""
        B = self.env.n_envs
        _lib.check(_lib.lib.eco_replay_compact_push(ctypes.byref(self.env.cfg), _lib.ptr(self.env.state), B,
                                                    _lib.ptr(self.ring), self._capacity, self._pushed,
                                                    _lib.ptr(actions), _lib.ptr(rewards), _lib.ptr(dones),
                                                    _lib.stream_ptr(stream)))
        self._pushed += B
        self._size = min(self._capacity, self._size + B)

    def _buffers(self, m):
        if m not in self._out:
            dev = self.device
            self._out[m] = (torch.empty(m, self.n_spins, self.x_stride, device=dev),
                            torch.empty(m, self.n_spins, self.x_stride, device=dev),
                            torch.empty(m, dtype=torch.int32, device=dev), torch.empty(m, dtype=torch.int32, device=dev),
                            torch.empty(m, device=dev), torch.empty(m, device=dev))
        return self._out[m]

    def sample(self, batch_size, device=None, stream=None):
        """ReplayBuffer.sample (dqn/utils.py:62-80): (states_x, actions, rewards, states_next_x, dones,
        graph_ids) of `batch_size` distinct uniform transitions, features rebuilt on the device."""
        xs, xn, gid, act, rew, done = self._buffers(batch_size)
        self._counter += 1
        _lib.check(_lib.lib.eco_replay_compact_sample(
            ctypes.byref(self.env.cfg), _lib.ptr(self.env.state), ctypes.byref(self.env.graphs.gs), self.env.n_envs,
            _lib.ptr(self.ring), self._capacity, self._size, self._pushed, batch_size, ctypes.c_uint64(self.seed),
            ctypes.c_uint64(self._counter), _lib.ptr(xs), _lib.ptr(xn), _lib.ptr(gid), _lib.ptr(act), _lib.ptr(rew),
            _lib.ptr(done), _lib.stream_ptr(stream)))
        return xs, act, rew, xn, done, gid

    @property
    def bytes_per_transition(self):
        return self.ring.numel() / (self._capacity + self.env.n_envs)

    def __len__(self):
        return self._size


class PrioritisedReplayBuffer:
    """PrioritisedReplayBuffer (dqn/utils.py:86-277): rank-based prioritised replay with the reference's API
    (add, sample, update_priorities, rebalance, configure_beta_anneal_time, __len__, alpha / beta / full).

    The binary max-heap of (buffer position, td error) is the native host heap of libecohip.so (eco_per_*;
    every add / priority update is a sequential heap walk, which has no parallel form to put on the GPU),
    following the reference's comparisons exactly; the transitions stay on the device, at slot = buffer
    position - 1:
      * add(state, action, reward, state_next, done): one transition of any tensors, as the reference
        (device rings [capacity, *shape] allocated on the first add);
      * add_batch(xs, xn, graph_ids, actions, rewards, dones): B transitions of the vector env into an fp32
        feature ring (eco_replay, the layout ReplayBuffer uses), sampled with the eco_replay_gather kernel.
    sample() draws one rank per partition with np.random.randint(low, high) exactly like the reference, so
    under the same numpy seed it picks the same transitions; it returns (batch, weights [B, 1] on the
    device, buffer positions), batch being the stacked fields for add() rings or (xs, actions, rewards, xn,
    dones, graph_ids) for add_batch() rings.
    """

    def __init__(self, capacity=10000, alpha=0.7, beta0=0.5, device="cuda"):
        self._capacity = int(capacity)
        self.alpha = alpha
        self.device = torch.device(device)
        h = _lib.lib.eco_per_create(self._capacity, float(alpha), float(beta0))
        if not h:
            raise ValueError(_lib.last_error())
        self._h = ctypes.c_void_p(h)
        self._rings = None      # add(): per-field device rings
        self._fring = None      # add_batch(): eco_replay feature ring
        self._out = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.lib.eco_per_destroy(h)
            self._h = None

    @property
    def beta(self):
        return _lib.lib.eco_per_beta(self._h)

    @property
    def full(self):
        return bool(_lib.lib.eco_per_full(self._h))

    def __len__(self):
        return _lib.lib.eco_per_len(self._h)

    def configure_beta_anneal_time(self, beta_max_at_samples):
        _lib.check(_lib.lib.eco_per_configure_beta_anneal_time(self._h, float(beta_max_at_samples)))

    def _add_positions(self, n):
        pos = np.zeros(n, np.int32)
        _lib.check(_lib.lib.eco_per_add(self._h, n, pos.ctypes.data_as(ctypes.c_void_p)))
        return pos

    def add(self, *args):
        """add (utils.py:120-142): one (state, action, reward, state_next, done) transition."""
        if self._fring is not None:
            raise ValueError("prioritised replay: add() on a buffer filled with add_batch()")
        t = Transition(*args)
        if self._rings is None:
            self._rings = [torch.zeros((self._capacity,) + tuple(torch.as_tensor(f).shape),
                                       dtype=torch.as_tensor(f).dtype, device=self.device) for f in t]
        slot = int(self._add_positions(1)[0]) - 1
        for ring, f in zip(self._rings, t):
            ring[slot].copy_(torch.as_tensor(f), non_blocking=True)

    def add_batch(self, xs, xn, graph_ids, actions, rewards, dones, stream=None):
        """B consecutive add() calls of vector-env transitions (the ReplayBuffer.add_batch arguments)."""
        if self._rings is not None:
            raise ValueError("prioritised replay: add_batch() on a buffer filled with add()")
        B, n_spins, x_stride = xs.shape
        if B > self._capacity:
            raise ValueError("prioritised replay: batch larger than the buffer (slots would collide)")
        if self._fring is None:
            dev = self.device
            c = self._capacity
            self._fring = (torch.zeros(c, n_spins, x_stride, device=dev), torch.zeros(c, n_spins, x_stride, device=dev),
                           torch.zeros(c, dtype=torch.int32, device=dev), torch.zeros(c, dtype=torch.int32, device=dev),
                           torch.zeros(c, device=dev), torch.zeros(c, device=dev))
            f = self._fring
            self._rb = _lib.Replay(c, n_spins, x_stride, *(t.data_ptr() for t in f))
        pos = self._add_positions(B)
        # consecutive buffer positions: one ring run starting at slot pos[0] - 1 (wrapping at capacity)
        _lib.check(_lib.lib.eco_replay_push(ctypes.byref(self._rb), int(pos[0]) - 1, B, _lib.ptr(xs), _lib.ptr(xn),
                                            _lib.ptr(graph_ids), _lib.ptr(actions), _lib.ptr(rewards), _lib.ptr(dones),
                                            _lib.stream_ptr(stream)))

    def update_priorities(self, buffer_positions, td_error):
        """update_priorities (utils.py:234-240)."""
        b = np.ascontiguousarray(np.asarray(buffer_positions), np.int32)
        t = td_error.detach().double().cpu().numpy() if torch.is_tensor(td_error) else np.asarray(td_error, np.float64)
        t = np.ascontiguousarray(t.reshape(-1), np.float64)
        if len(t) != len(b):
            raise ValueError("prioritised replay: one td error per buffer position")
        _lib.check(_lib.lib.eco_per_update_priorities(self._h, len(b), b.ctypes.data_as(ctypes.c_void_p),
                                                      t.ctypes.data_as(ctypes.c_void_p)))

    def rebalance(self):
        """rebalance (utils.py:185-202)."""
        _lib.check(_lib.lib.eco_per_rebalance(self._h))

    @property
    def partitions(self):
        n = _lib.lib.eco_per_partitions(self._h, None, None)
        bounds = np.zeros(n + 1, np.int32)
        _lib.lib.eco_per_partitions(self._h, bounds.ctypes.data_as(ctypes.c_void_p), None)
        return [(int(a), int(b)) for a, b in zip(bounds[:-1], bounds[1:])]

    def sample(self, batch_size, device=None, stream=None):
        """sample (utils.py:242-273) -> (batch, weights [B, 1], buffer positions)."""
        if self._rings is None and self._fring is None:
            raise KeyError("prioritised replay: sample from an empty buffer")
        bounds = np.zeros(batch_size + 1, np.int32)
        _lib.check(_lib.lib.eco_per_sample_begin(self._h, batch_size, bounds.ctypes.data_as(ctypes.c_void_p)))
        ranks = np.array([np.random.randint(lo, hi) for lo, hi in zip(bounds[:-1], bounds[1:])], np.int64)
        bps = np.zeros(batch_size, np.int32)
        w = np.zeros(batch_size, np.float32)
        _lib.check(_lib.lib.eco_per_sample_finish(self._h, batch_size, ranks.ctypes.data_as(ctypes.c_void_p),
                                                  ctypes.c_uint64(0), bps.ctypes.data_as(ctypes.c_void_p),
                                                  w.ctypes.data_as(ctypes.c_void_p), None))
        dev = self.device if device is None else torch.device(device)
        slots = torch.from_numpy(bps - 1).to(self.device, non_blocking=True)
        weights = torch.from_numpy(w).reshape(-1, 1).to(dev)
        if self._rings is not None:
            batch = [ring.index_select(0, slots.long()).to(dev) for ring in self._rings]
        else:
            m = batch_size
            if m not in self._out:
                d = self.device
                n_spins, x_stride = self._fring[0].shape[1:]
                self._out[m] = (torch.empty(m, n_spins, x_stride, device=d), torch.empty(m, n_spins, x_stride, device=d),
                                torch.empty(m, dtype=torch.int32, device=d), torch.empty(m, dtype=torch.int32, device=d),
                                torch.empty(m, device=d), torch.empty(m, device=d))
            xs, xn, gid, act, rew, done = self._out[m]
            _lib.check(_lib.lib.eco_replay_gather(ctypes.byref(self._rb), m, _lib.ptr(slots), _lib.ptr(xs), _lib.ptr(xn),
                                                  _lib.ptr(gid), _lib.ptr(act), _lib.ptr(rew), _lib.ptr(done),
                                                  _lib.stream_ptr(stream)))
            batch = (xs, act, rew, xn, done, gid)
        return batch, weights, tuple(int(b) for b in bps)
