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
