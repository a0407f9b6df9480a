"""Batched DQN agent (src/agents/dqn/dqn.py) on the HIP engine.

Same constructor keywords and public methods as the reference DQN
(`learn`, `train_step`, `act`, `predict`, `update_epsilon`, `update_lr`,
`evaluate_agent`, `save`, `load`), but `envs` is a VecSpinSystem: every call
advances B episodes.  Everything on the step path runs in libecohip:
  act       -> MPNN forward with the fused epsilon-greedy argmax (dqn.py:453-465)
  env.step  -> batched SpinSystem kernel (spinsystem.py:355-559)
  replay    -> device ring push / distinct-index sample (dqn/utils.py:28-83)
  train     -> online(s') argmax, target(s') gather, online(s) forward with saved
               activations, TD + MSE gradient, MPNN backward, Adam (dqn.py:403-451)
Schedules are per env-step as in the reference; a vector step advances the
counter by B.  The replay ratio of the reference (minibatch_size/update_frequency
samples per env-step, 64/32 = 2 in train_eco.py:136-137) is kept by running
K = B*ratio/M gradient steps of minibatch M per vector step.  Multi-GPU: one
process per GPU, episodes sharded, gradients summed over RCCL (torch.distributed)
and averaged inside the Adam kernel; parameters stay bit-identical across ranks.
"""
import ctypes
import math
import os
import random

import numpy as np
import torch

from ... import _lib
from ...parallel import allreduce_gradients_async, broadcast_parameters
from .utils import CompactReplayBuffer, ReplayBuffer, TestMetric, set_global_seed


def graph_slots_needed(n_envs, max_steps, replay_buffer_size):
    """GraphStore slots for fresh graphs per episode with lockstep episodes (each ends at max_steps):
    a batch of n_envs episodes pushes n_envs * max_steps transitions, and a batch's slots may only be
    regenerated once replay_buffer_size pushes have passed since it ended, so
    ceil(replay_buffer_size / (n_envs * max_steps)) + 1 batches of n_envs slots rotate."""
    per_batch = n_envs * max_steps
    return n_envs * (-(-int(replay_buffer_size) // per_batch) + 1)


class DQN:
    def __init__(self, envs, network, init_network_params=None, init_weight_std=None, double_dqn=True,
                 update_target_frequency=10000, gamma=0.99, clip_Q_targets=False, replay_start_size=50000,
                 replay_buffer_size=1000000, minibatch_size=32, update_frequency=1, update_learning_rate=True,
                 initial_learning_rate=0, peak_learning_rate=1e-3, peak_learning_rate_step=10000,
                 final_learning_rate=5e-5, final_learning_rate_step=200000, max_grad_norm=None, weight_decay=0,
                 update_exploration=True, initial_exploration_rate=1, final_exploration_rate=0.1,
                 final_exploration_step=1000000, adam_epsilon=1e-8, loss="mse", save_network_frequency=10000,
                 network_save_path='network', evaluate=True, test_envs=None, test_episodes=20,
                 test_frequency=10000, test_save_path='test_scores', test_metric=TestMetric.ENERGY_ERROR,
                 logging=True, seed=None, train_minibatch=None, graph_pool_ids=None, regenerate_graphs=None,
                 compact_replay=None, target_sync="grad_steps", overlap_evaluation=True):
        if isinstance(envs, (list, tuple)):
            if len(envs) != 1:
                raise NotImplementedError("pass one VecSpinSystem (it already holds B episodes)")
            envs = envs[0]
        if loss != "mse":
            raise NotImplementedError("eco_hip implements the reference's training loss 'mse' (train_eco.py:148)")
        if max_grad_norm is not None:
            raise NotImplementedError("gradient clipping is not on the hot path (train_eco.py:138 uses None)")
        self.env = envs
        self.graphs = envs.graphs
        self.device = envs.graphs.device
        self.double_dqn = double_dqn
        self.replay_start_size = replay_start_size
        self.replay_buffer_size = replay_buffer_size
        self.gamma = gamma
        self.clip_Q_targets = clip_Q_targets
        self.update_target_frequency = update_target_frequency
        self.minibatch_size = minibatch_size
        self.update_learning_rate = update_learning_rate
        self.initial_learning_rate = initial_learning_rate
        self.peak_learning_rate = peak_learning_rate
        self.peak_learning_rate_step = peak_learning_rate_step
        self.final_learning_rate = final_learning_rate
        self.final_learning_rate_step = final_learning_rate_step
        self.weight_decay = weight_decay
        self.update_frequency = update_frequency
        # dqn.py:161 stores a one-tuple (`self.update_exploration = update_exploration,`), which is always
        # truthy: the reference decays epsilon whatever is passed, and so does this class
        self.update_exploration = update_exploration,
        self.initial_exploration_rate = initial_exploration_rate
        self.epsilon = initial_exploration_rate
        self.final_exploration_rate = final_exploration_rate
        self.final_exploration_step = final_exploration_step
        self.adam_epsilon = adam_epsilon
        self.lr = initial_learning_rate
        self.logging = logging
        self.seed = random.randint(0, 10 ** 6) if seed is None else seed
        set_global_seed(self.seed)
        self.acting_in_reversible_spin_env = envs.reversible_spins
        self.allowed_value = envs.allowed_action_value()

        self.network = network()
        self.target_network = network()
        self._network_factory = network
        self._eval_net = None
        if init_network_params is not None:
            self.load(init_network_params)
        elif init_weight_std is not None:
            self.network.init_normal_(init_weight_std, generator=torch.Generator().manual_seed(self.seed))
        self.dist = torch.distributed.is_available() and torch.distributed.is_initialized()
        self.world = torch.distributed.get_world_size() if self.dist else 1
        broadcast_parameters(self.network.flat)  # every rank starts from rank 0's weights
        # evaluations use rank 0's seed on every rank (learn() runs each evaluation of the job on one rank: its
        # episodes' initial spins must not depend on which rank that is); = seed in one process
        self.eval_seed = self.seed
        if self.dist and self.world > 1:
            t = torch.tensor([self.seed], dtype=torch.int64,
                             device=self.device if torch.distributed.get_backend() == "nccl" else "cpu")
            torch.distributed.broadcast(t, src=0)
            self.eval_seed = int(t.item())
        self.target_network.load_state_dict(self.network.state_dict())
        n = self.network.flat.numel()
        self.grad = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.exp_avg = torch.zeros_like(self.grad)
        self.exp_avg_sq = torch.zeros_like(self.grad)
        self.adam_step = 0
        self.grad_steps = 0

        self.B = envs.n_envs
        self.N = envs.n_spins
        self.M = int(train_minibatch or minibatch_size)
        # compact replay (one integer env state per transition, 4 B per vertex) for MaxCut envs on +-1
        # graphs; else fp32 features
        eligible = (envs.cfg.optimisation_target == _lib.ECO_TARGET_CUT and envs.graphs.unit_weights
                    and envs.max_steps < 32768 and self.N <= _lib.ECO_COMPACT_MAX_SPINS)
        self.compact_replay = eligible if compact_replay is None else bool(compact_replay)
        if self.compact_replay and not eligible:
            raise ValueError("compact replay needs OptimisationTarget.CUT, +-1 weights, max_steps < 32768 and "
                             f"n_spins <= {_lib.ECO_COMPACT_MAX_SPINS}")
        if self.compact_replay:
            self.replay_buffer = CompactReplayBuffer(replay_buffer_size, envs, seed=self.seed)
        else:
            self.replay_buffer = ReplayBuffer(replay_buffer_size, self.N, device=self.device, seed=self.seed,
                                              n_obs=envs.n_obs)
        self.replay_ratio = minibatch_size / float(update_frequency)
        # reference (dqn.py:332-347): one train_step every update_frequency env-steps and one target sync every
        # update_target_frequency env-steps, i.e. a sync every update_target_frequency / update_frequency gradient
        # steps.  target_sync="grad_steps" (default) keeps that count of optimiser steps between syncs whatever
        # the minibatch ("count sync in gradient steps"); "samples" syncs every
        # update_target_frequency env-steps' worth of replayed samples instead (the two agree at M = minibatch_size).
        if target_sync not in ("grad_steps", "samples"):
            raise ValueError("target_sync must be 'grad_steps' or 'samples'")
        self.target_sync = target_sync
        self.target_sync_grad_steps = max(1, int(round(update_target_frequency / float(update_frequency))))
        self.target_sync_samples = update_target_frequency * self.replay_ratio
        self._samples_since_sync = 0.0
        self.graph_pool_ids = (np.arange(self.graphs.n_graphs) if graph_pool_ids is None
                               else np.asarray(graph_pool_ids))
        # Fresh graphs per episode like the reference's generators (utils.py:165-236): every reset
        # takes the next slots of the store in ring order and regenerates them on the device first.
        # Replay entries reference graph ids, so a slot is only regenerated once no live episode uses
        # it and `replay_buffer_size` pushes have passed since its last episode ended (every entry
        # that could reference it has been overwritten); otherwise its graph is reused as it is
        # (still correct, not fresh) and a warning is issued once.
        self.regenerate_graphs = regenerate_graphs
        self._pushed = 0
        if regenerate_graphs is not None:
            if not hasattr(self.graphs, "cap"):
                raise ValueError("regenerate_graphs needs a GraphStore.slots(...) store")
            need = graph_slots_needed(envs.n_envs, envs.max_steps, replay_buffer_size)
            if envs.reversible_spins and envs.cfg.stopping == 1 and self.graphs.n_graphs < need:
                # lockstep episodes (every one ends at max_steps): B * max_steps pushes per episode batch,
                # so ceil(capacity / (B * max_steps)) + 1 batches of B slots must rotate
                raise ValueError(f"regenerate_graphs with n_envs={envs.n_envs}, max_steps={envs.max_steps} and "
                                 f"replay_buffer_size={replay_buffer_size} needs GraphStore.slots(>= {need}, ...) "
                                 f"(has {self.graphs.n_graphs}): a slot may only be regenerated once no stored "
                                 "transition references it")
            n_slots = self.graphs.n_graphs
            self._slot_users = np.zeros(n_slots, np.int64)
            self._slot_free_at = np.full(n_slots, -(1 << 62), np.int64)
            self._slot_cursor = 0
            self._slot_warned = False
            self.graphs_regenerated = 0      # slots regenerated so far (fresh graphs handed out)
            self.graphs_reused = 0           # slots handed out without regeneration (not yet safe)
        self._rng = np.random.default_rng(self.seed)

        self.evaluate = evaluate
        self.test_envs = test_envs
        self.test_episodes = int(test_episodes)
        self.test_frequency = test_frequency
        self.test_save_path = test_save_path
        self.test_metric = test_metric
        self.save_network_frequency = save_network_frequency
        self.network_save_path = network_save_path
        # learn(): evaluations that take the one-fill path run on a side stream on a snapshot of the weights while
        # training continues (same results: the snapshot is the network at the evaluation's timestep)
        self.overlap_evaluation = overlap_evaluation
        self._eval_stream = None
        # one-fill evaluations replay their rollout from a HIP graph captured at the second evaluation of an
        # (env, network) pair (_capture_eval_rollout); False keeps every evaluation's launches eager
        self.eval_graphs = True
        self._eval_graphs = {}
        # learn(): spread the B lockstep episodes over the T phases of an episode (start(); False: all B episodes
        # start together and end together every T vector steps)
        self.stagger_episodes = False

        self._act_counter = 0
        self._alloc_train_buffers(self.M)

    # ---------------------------------------------------------------- buffers
    def _alloc_train_buffers(self, m):
        dev = self.device
        self.q_s = torch.empty(m, self.N, device=dev)
        self.q_tn = torch.empty(m, self.N, device=dev)
        self.a_star = torch.empty(m, dtype=torch.int32, device=dev)
        self.dq = torch.empty(m, self.N, device=dev)
        self.sqerr = torch.empty(m, device=dev)
        self.loss_dev = torch.zeros(1, device=dev)
        self.saved = torch.empty(self.network.saved_bytes(self.N, m), dtype=torch.uint8, device=dev)
        self.bw_ws = torch.empty(_lib.lib.eco_mpnn_backward_workspace_bytes(self.N, m), dtype=torch.uint8,
                                 device=dev)
        self._train_m = m
        self._actions = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self._obs = [self.env.obs_x, torch.zeros_like(self.env.obs_x)]

    # -------------------------------------------------------------- schedules
    def update_epsilon(self, timestep):
        """dqn.py:467-471"""
        eps = self.initial_exploration_rate - (self.initial_exploration_rate - self.final_exploration_rate) * (
            timestep / self.final_exploration_step)
        self.epsilon = max(eps, self.final_exploration_rate)

    def update_lr(self, timestep):
        """dqn.py:473-488"""
        if timestep <= self.peak_learning_rate_step:
            lr = self.initial_learning_rate - (self.initial_learning_rate - self.peak_learning_rate) * (
                timestep / self.peak_learning_rate_step)
        elif timestep <= self.final_learning_rate_step:
            lr = self.peak_learning_rate - (self.peak_learning_rate - self.final_learning_rate) * (
                (timestep - self.peak_learning_rate_step) /
                (self.final_learning_rate_step - self.peak_learning_rate_step))
        else:
            lr = None
        if lr is not None:
            self.lr = lr

    # ------------------------------------------------------------------- act
    def _act_config(self, epsilon):
        self._act_counter += 1
        return _lib.ActConfig(float(epsilon), int(self.acting_in_reversible_spin_env), float(self.allowed_value),
                              self.seed, self._act_counter)

    def act(self, obs_x, graph_ids, is_training_ready=True, actions_out=None):
        """dqn.py:453-465 for every episode: epsilon-greedy over the MPNN (B=1 norm semantics, :282)."""
        eps = self.epsilon if is_training_ready else 1.0
        out = actions_out if actions_out is not None else torch.empty(obs_x.shape[0], dtype=torch.int32,
                                                                       device=self.device)
        self.network.forward_graphs(obs_x, self.graphs, graph_ids, norm_scope=_lib.ECO_NORM_PER_GRAPH,
                                    act=self._act_config(eps), actions_out=out)
        return out

    @torch.no_grad()
    def predict(self, obs_x, graph_ids, graphs=None, norm_scope=_lib.ECO_NORM_PER_CALL):
        """dqn.py:490-512: greedy actions (allowed vertices only for irreversible envs)."""
        out = torch.empty(obs_x.shape[0], dtype=torch.int32, device=self.device)
        self.network.forward_graphs(obs_x, graphs or self.graphs, graph_ids, norm_scope=norm_scope,
                                    act=self._act_config(0.0), actions_out=out)
        return out

    # ----------------------------------------------------------------- train
    def train_step(self, transitions, sync_loss=True, loss_out=None, overlap=None):
        """dqn.py:403-451.  transitions = (states_x, actions, rewards, states_next_x, dones, graph_ids)
        as returned by ReplayBuffer.sample.  Returns the loss: a float if sync_loss, else the one-element
        device tensor it was written to (`loss_out`, or a copy of the agent's loss slot).
        overlap: optional callable issued while the gradient all-reduce is in flight (multi-GPU): work that does
        not read the gradient or the online weights, e.g. the next minibatch's replay sample."""
        xs, act, rew, xn, done, gid = transitions
        loss_dev = self.loss_dev if loss_out is None else loss_out
        m = xs.shape[0]
        if m != self._train_m:
            self._alloc_train_buffers(m)
        net, tgt = self.network, self.target_network
        greedy = _lib.ActConfig(0.0, int(self.acting_in_reversible_spin_env), float(self.allowed_value), 0, 0)
        if self.double_dqn:
            # greedy_actions = network(s').argmax (masked for irreversible envs), q_t = target(s')[a*]
            net.forward_pair_graphs(tgt, xn, self.graphs, gid, norm_scope=_lib.ECO_NORM_PER_CALL, act=greedy,
                                    actions_out=self.a_star, q_out_other=self.q_tn)
            # same graph ids, same workspace: the per-call max degree the pair left there
            scope_s = _lib.ECO_NORM_PER_CALL_REUSE
        else:
            tgt.forward_graphs(xn, self.graphs, gid, norm_scope=_lib.ECO_NORM_PER_CALL, q_out=self.q_tn,
                               act=greedy, actions_out=self.a_star)
            scope_s = _lib.ECO_NORM_PER_CALL
        net.forward_graphs(xs, self.graphs, gid, norm_scope=scope_s, q_out=self.q_s, saved=self.saved)
        _lib.check(_lib.lib.eco_dqn_td(_lib.ptr(self.q_s), _lib.ptr(self.q_tn), _lib.ptr(self.a_star),
                                       _lib.ptr(act), _lib.ptr(rew), _lib.ptr(done), m, self.N,
                                       ctypes.c_float(self.gamma), int(bool(self.clip_Q_targets)), _lib.ptr(self.dq),
                                       _lib.ptr(self.sqerr), _lib.ptr(loss_dev), _lib.stream_ptr()))
        net.backward_graphs(xs, self.graphs, gid, self.saved, self.dq, self.grad, workspace=self.bw_ws)
        # RCCL sum over xGMI (233.7 KB) on the collective's stream, the mean folded into Adam; independent work
        # (the caller's `overlap`) is issued on this stream meanwhile
        work, scale = allreduce_gradients_async(self.grad)
        if overlap is not None:
            overlap()
        if work is not None:
            work.wait()
        self.adam_step += 1
        _lib.check(_lib.lib.eco_adam(_lib.ptr(net.flat), _lib.ptr(self.grad), _lib.ptr(self.exp_avg),
                                     _lib.ptr(self.exp_avg_sq), net.flat.numel(), self.lr, 0.9, 0.999,
                                     self.adam_epsilon, float(self.weight_decay), scale, self.adam_step,
                                     _lib.stream_ptr()))
        net.repack()
        self.grad_steps += 1
        self._samples_since_sync += m * self.world
        if sync_loss:
            return loss_dev.item()
        return loss_dev if loss_out is not None else loss_dev.clone()

    def sync_target(self):
        """dqn.py:346-347: target <- online."""
        self.target_network.flat.copy_(self.network.flat)

    def _take_graph_slots(self, episodes):
        """Graph ids for the episodes being reset (a bool mask over B, or None = all).  Without
        regenerate_graphs: random graphs of the pool.  With it: the next slots of the store in ring
        order, each regenerated on the device when it is safe (no live user, `replay_buffer_size`
        pushes since its last episode ended), reused otherwise (warned once)."""
        k = self.B if episodes is None else int(episodes.sum())
        if self.regenerate_graphs is None:
            ids = self.graph_pool_ids[self._rng.integers(0, len(self.graph_pool_ids), k)]
            if episodes is None:
                return ids
            out = np.zeros(self.B, np.int64)   # VecSpinSystem.reset reads graph_ids[mask]: B-long
            out[episodes] = ids
            return out
        kind, param = self.regenerate_graphs[:2]
        weights = self.regenerate_graphs[2] if len(self.regenerate_graphs) > 2 else "discrete"
        n_slots = len(self._slot_users)
        if self._started:   # release the slots of the episodes being reset (host mirror: no device read)
            old = self._host_graph_ids
            old = old if episodes is None else old[episodes]
            np.subtract.at(self._slot_users, old, 1)
            self._slot_free_at[old[self._slot_users[old] == 0]] = self._pushed
        ids = (self._slot_cursor + np.arange(k)) % n_slots
        self._slot_cursor = int((self._slot_cursor + k) % n_slots)
        safe = (self._slot_users[ids] == 0) & (self._pushed - self._slot_free_at[ids] >= self.replay_buffer_size)
        fresh = ids[safe]
        for run in np.split(fresh, np.nonzero(np.diff(fresh) != 1)[0] + 1) if len(fresh) else []:
            self.graphs.generate(int(run[0]), len(run), kind, param, seed=int(self._rng.integers(1 << 62)),
                                 weights=weights, check=False)
        self.graphs_regenerated += len(fresh)
        self.graphs_reused += k - len(fresh)
        if len(fresh) < k and not self._slot_warned:
            import warnings
            warnings.warn(f"regenerate_graphs: {k - len(fresh)} of {k} episodes reset onto graphs that stored "
                          f"transitions may still reference (store of {n_slots} slots); they reuse those graphs. "
                          "Allocate more GraphStore.slots for a fresh graph per episode.", RuntimeWarning)
            self._slot_warned = True
        np.add.at(self._slot_users, ids, 1)
        if episodes is None:
            return ids
        out = np.zeros(self.B, np.int64)
        out[episodes] = ids
        return out

    def vector_step(self, is_training_ready):
        """One act -> env.step -> replay.add over all B episodes; returns the new obs buffer.
        Every episode is live here: finished ones are reset by iteration() right after the step
        that ended them (the reference resets on done, dqn.py:306-327)."""
        x = self.env.obs_x
        nxt = self._obs[1] if x.data_ptr() == self._obs[0].data_ptr() else self._obs[0]
        self.act(x, self.env.graph_ids, is_training_ready, actions_out=self._actions)
        _, rew, done = self.env.step(self._actions, obs_out=nxt)
        if self.compact_replay:
            self.replay_buffer.add_step(self._actions, rew, done)
        else:
            self.replay_buffer.add_batch(x, nxt, self.env.graph_ids, self._actions, rew, done)
        self._pushed += self.B
        return nxt

    def _reset_env(self, graph_ids, seed, mask=None):
        """env.reset (all episodes, or the masked ones) and, for the compact replay, record the new states.
        The episodes' graph ids are mirrored on the host for the slot bookkeeping of _take_graph_slots."""
        ids = np.asarray(graph_ids, np.int64)
        if mask is None or not hasattr(self, "_host_graph_ids"):
            self._host_graph_ids = ids.copy()
        else:
            m = np.asarray(mask.cpu() if torch.is_tensor(mask) else mask).astype(bool)
            self._host_graph_ids[m] = ids[m]
            mask = self.env._upload(mask, torch.uint8)  # one non-blocking upload for the env and the replay
        self.env.reset(graph_ids=graph_ids, mask=mask, seed=seed)
        if self.compact_replay:
            self.replay_buffer.snapshot(mask)

    def start(self):
        """Reset every episode on fresh pool graphs (start of learn).  The replay buffer and the push
        count persist across learn() calls (as the reference's replay buffer does), so graph slots that
        stored transitions reference are not regenerated by a second learn()."""
        self._started = getattr(self, "_started", False)
        self._reset_env(self._take_graph_slots(None), self.seed)
        self._started = True
        self._steps_in_episode = 0
        self._timestep = 0
        self._ready = False
        self._k_per_vec = max(1, int(round(self.B * self.replay_ratio / self.M)))
        self._last_loss = None
        if not hasattr(self, "_loss_buf"):   # every gradient step's loss, kept on the device (dqn.py:339)
            self._loss_buf = torch.zeros(4096, dtype=torch.float32, device=self.device)
            self._loss_t = np.zeros(4096, np.int64)
            self._loss_n = 0
        # the reference's `losses` list is local to one learn() call (dqn.py:269): report from here on
        self._loss_start = self._loss_n
        # every episode ends exactly at max_steps only for reversible spins with Stopping.NORMAL
        # (spinsystem.py:539-554); otherwise dones are read back after each vector step
        self._lockstep = self.env.reversible_spins and self.env.cfg.stopping == 1
        # staggered episodes (stagger_episodes, lockstep envs only): episode b's first episode is cut after
        # T - (b T // B) steps (its last transition stored with the env's done = 0: a truncation, not a terminal),
        # so from then on the B episodes sit at B / T evenly spread phases and ~B / T of them end and are reset on
        # fresh graphs every vector step, as a single reference env's consecutive episodes pass through every phase
        self._stagger = bool(self.stagger_episodes and self._lockstep)
        if self._stagger:
            T = self.env.max_steps
            self._ep_left = T - (np.arange(self.B, dtype=np.int64) * T) // self.B

    def iteration(self):
        """One vector step of DQN.learn (dqn.py:273-347): act/step/add for all B episodes, reset
        finished episodes, then K gradient steps (replay ratio preserved) with target syncs.
        Schedules count global env-steps: B per rank per vector step, times the world size."""
        B, T = self.B, self.env.max_steps
        if not self._ready and len(self.replay_buffer) >= max(self.replay_start_size, self.M):
            self._ready = True
        self.vector_step(self._ready)
        self._timestep += B * self.world
        self._steps_in_episode += 1
        # dqn.py:284-290 run after each act with that env-step's 0-based index: a vector step ends with
        # the index of its last env-step (B = 1 reproduces the reference's sequence exactly)
        if self.update_exploration:
            self.update_epsilon(self._timestep - 1)
        if self.update_learning_rate:
            self.update_lr(self._timestep - 1)
        if self._stagger:
            self._ep_left -= 1
            ending = self._ep_left == 0
            if ending.any():
                self._reset_env(self._take_graph_slots(ending), self.seed + self._timestep, mask=ending)
                self._ep_left[ending] = T
        elif self._lockstep:
            if self._steps_in_episode == T:
                self._reset_env(self._take_graph_slots(None), self.seed + self._timestep)
                self._steps_in_episode = 0
        else:
            done = self.env.dones.bool()
            n_done = int(done.sum())
            if n_done == B:
                self._reset_env(self._take_graph_slots(None), self.seed + self._timestep)
                self._steps_in_episode = 0
            elif n_done:
                mask = done.cpu().numpy()
                self._reset_env(self._take_graph_slots(mask), self.seed + self._timestep, mask=done)
        if self._ready:
            # gradient step k's all-reduce overlaps step k+1's replay sample (stream order: the sample rewrites
            # the minibatch buffers after step k's forwards and backward have read them)
            nxt = [self.replay_buffer.sample(self.M)]
            for k in range(self._k_per_vec):
                tr = nxt.pop()
                more = k + 1 < self._k_per_vec

                def prefetch():
                    nxt.append(self.replay_buffer.sample(self.M))
                self._last_loss = self.train_step(tr, sync_loss=False, loss_out=self._loss_slot(self._timestep),
                                                  overlap=prefetch if more else None)
                if (self.grad_steps % self.target_sync_grad_steps == 0 if self.target_sync == "grad_steps"
                        else self._samples_since_sync >= self.target_sync_samples):
                    self.sync_target()
                    self._samples_since_sync = 0.0
        return self._last_loss

    def _loss_slot(self, timestep):
        """One-element view of the device loss log for the next gradient step (grown by doubling, so
        the log costs no allocation per step and one host copy in losses())."""
        if self._loss_n == len(self._loss_t):
            self._loss_buf = torch.cat([self._loss_buf, torch.zeros_like(self._loss_buf)])
            self._loss_t = np.concatenate([self._loss_t, np.zeros_like(self._loss_t)])
        self._loss_t[self._loss_n] = timestep
        self._loss_n += 1
        return self._loss_buf[self._loss_n - 1:self._loss_n]

    def learn(self, timesteps, verbose=False, on_vector_step=None):
        """dqn.py:256-395 with B episodes per vector step on each rank (timesteps counts global
        env-steps).  As in the reference, once training is ready: every `test_frequency` env-steps
        evaluate_agent() and save `<network_save_path>_best` when the score beats every earlier one
        (:349-364); every `save_network_frequency` env-steps save `<network_save_path><t>` (:366-372);
        at the end pickle test_scores / losses / solutions (:377-394).  A vector step that crosses
        k * frequency counts as reaching timestep k * frequency.  Files are written by rank 0.

        Multi-GPU: each crossing is ONE evaluation of the job, run by one rank (evaluation e by rank e mod world,
        on its test env: the same episodes and test graphs as a single-process evaluation at that timestep); its
        scores reach every rank through a small all-reduce to which only the owner contributes, issued by every
        rank at the same point (when evaluation e + world starts, or at the end of learn()), so the evaluation
        work per rank per vector step does not grow with the world size.  Nothing here waits for the training
        stream: the all-reduce is asynchronous and its result is read back into pinned memory behind an event,
        recorded (scores, `_best`) once that event has fired -- a few vector steps later -- or at the end; the
        owner's scores come from pinned copies behind the side stream's event; the regenerated graphs' error word
        is peeked the same way (eco_error_word_copy).  Rank 0 snapshots the weights of every evaluation into
        pinned host memory at its timestep for `_best` (the parameters are bit-identical across ranks).
        Returns the last 100 (timestep, loss) pairs."""
        import pickle
        from collections import deque
        self.start()
        rank = torch.distributed.get_rank() if self.dist else 0
        world = self.world
        nccl = world > 1 and torch.distributed.get_backend() == "nccl"
        test_scores, test_solutions = [], []
        inflight = deque()   # evaluations launched, scores not yet taken (index order)
        reducing = deque()   # scores taken, all-reduce / read-back in flight, not yet recorded (index order)
        err_checks = deque()  # (event, pinned word) peeks at the device error word
        saves = deque()      # (event, pinned weights, path) periodic checkpoints not yet written
        n_eval = 0           # evaluations launched by the job so far (every rank counts the same)
        test_env0 = self._test_env() if self.evaluate else None
        cursor0 = getattr(test_env0, "_eval_next_graph", 0) if test_env0 is not None else 0
        # rank 0's weight snapshots for _best, one pinned slot per evaluation that can be unrecorded at once
        depth = 3 * world
        snaps = ([torch.empty(self.network.flat.numel(), dtype=torch.float32).pin_memory() for _ in range(depth)]
                 if rank == 0 and self.evaluate else None)

        def record(e, test_score, test_solution):
            if verbose and rank == 0:
                print('\nTest score: {}\nTest solution: {}\n'.format(np.round(test_score, 3),
                                                                    np.round(test_solution, 3)))
            if all(test_score > sc for _, sc in test_scores) and rank == 0:
                main, ext = os.path.splitext(self.network_save_path)
                e["snap_ev"].synchronize()  # the snapshot copy (issued at the evaluation's timestep) has landed
                self._save_flat(main + "_best" + (ext or ".pth"), e["snap"])
            test_scores.append([e["tk"], test_score])
            test_solutions.append([e["tk"], test_solution])

        def take(e):
            """Evaluation e's scores on every rank (the same call order everywhere: the all-reduce is collective):
            the owner's from its pinned results, all-reduced without waiting; recorded by flush()."""
            if e["owner"] == rank:
                sc, so = self._eval_one_fill_finish(e["p"]) if "p" in e else e["result"]
            else:
                sc, so = 0.0, 0.0
            if world == 1:
                record(e, sc, so)
                return
            src = torch.tensor([sc, so], dtype=torch.float64).pin_memory()
            if nccl:
                t = torch.empty(2, dtype=torch.float64, device=self.device)
                t.copy_(src, non_blocking=True)
            else:
                t = src
            work = torch.distributed.all_reduce(t, async_op=True)  # only the owner contributes: the sum is its result
            e["red"] = (src, t, work)
            if nccl:
                work.wait()  # the current stream waits for the collective; the host does not
                e["res"] = torch.empty(2, dtype=torch.float64).pin_memory()
                e["res"].copy_(t, non_blocking=True)
                e["res_ev"] = torch.cuda.Event()
                e["res_ev"].record()
            reducing.append(e)

        def flush(upto):
            """Record, in order, the reduced evaluations whose results have arrived, waiting for those with
            index <= upto (None: wait for none)."""
            while reducing:
                e = reducing[0]
                src, t, work = e["red"]
                must = upto is not None and e["idx"] <= upto
                if nccl:
                    if not (must or e["res_ev"].query()):
                        return
                    e["res_ev"].synchronize()
                    res = e["res"]
                else:
                    if not (must or work.is_completed()):
                        return
                    work.wait()
                    res = t
                reducing.popleft()
                record(e, float(res[0]), float(res[1]))

        def save_deferred(path, block):
            """Periodic checkpoints: the weights copied into pinned memory at their timestep, written once the
            copy has landed (no wait on the training stream)."""
            if path is not None:
                host = torch.empty(self.network.flat.numel(), dtype=torch.float32).pin_memory()
                host.copy_(self.network.flat, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                saves.append((ev, host, path))
            while saves and (block or saves[0][0].query()):
                ev, host, p_ = saves.popleft()
                ev.synchronize()
                self._save_flat(p_, host)

        def peek_errors(block):
            """Raise a device error flagged since the last peek (regenerated graphs: edge-slot overflow)."""
            while err_checks and (block or err_checks[0][0].query()):
                ev, word = err_checks.popleft()
                ev.synchronize()
                if int(word[0]) != 0:
                    self.graphs.check_errors()

        def launch(tk):
            nonlocal n_eval
            owner = n_eval % world
            e = {"tk": tk, "owner": owner, "idx": n_eval}
            n_eval += 1
            if rank == 0:
                # slot idx % depth is free once evaluation idx - depth is recorded (launched >= 2 world earlier)
                flush(e["idx"] - depth)
                e["snap"] = snaps[e["idx"] % depth]
                e["snap"].copy_(self.network.flat, non_blocking=True)  # the weights at tk, for _best
                e["snap_ev"] = torch.cuda.Event()
                e["snap_ev"].record()
            if owner == rank:
                env = self._test_env()
                n_graphs = env.graphs.n_graphs
                env._eval_next_graph = (cursor0 + e["idx"] * self.test_episodes) % n_graphs  # job-wide order
                if self._overlap_ok(env):
                    e["p"] = self._evaluate_overlapped(tk)
                else:
                    e["result"] = self.evaluate_agent()
            inflight.append(e)

        while self._timestep < timesteps:
            t_prev = self._timestep
            self.iteration()
            t = self._timestep
            if on_vector_step is not None:
                on_vector_step(t)
            if not self._ready:
                continue
            crossed_test = t // self.test_frequency > t_prev // self.test_frequency
            if crossed_test and self.regenerate_graphs is not None:
                # graphs regenerated with check=False since the last peek: an edge-slot overflow sets the device
                # error word (the slot becomes an empty graph); peeked without waiting, raised when seen
                word = torch.zeros(1, dtype=torch.int32).pin_memory()
                _lib.check(_lib.lib.eco_error_word_copy(_lib.ptr(word), _lib.stream_ptr()))
                ev = torch.cuda.Event()
                ev.record()
                err_checks.append((ev, word))
            peek_errors(False)
            flush(None)
            save_deferred(None, False)
            if world == 1 and inflight and "p" in inflight[0] and inflight[0]["p"]["done"].query():
                take(inflight.popleft())  # finished early (one process: no collective to keep in step)
            if self.evaluate and crossed_test:
                tk = (t // self.test_frequency) * self.test_frequency
                while len(inflight) >= world:  # this evaluation's owner runs one evaluation at a time
                    take(inflight.popleft())
                launch(tk)
            if t // self.save_network_frequency > t_prev // self.save_network_frequency and rank == 0:
                tk = (t // self.save_network_frequency) * self.save_network_frequency
                main, ext = os.path.splitext(self.network_save_path)
                save_deferred(main + str(tk) + (ext or ".pth"), False)
        while inflight:
            take(inflight.popleft())
        flush(n_eval)
        peek_errors(True)
        save_deferred(None, True)
        if self.regenerate_graphs is not None:
            self.graphs.check_errors()
        losses = self.losses()
        if rank == 0 and self.test_save_path is not None:
            path = self.test_save_path
            if os.path.splitext(path)[-1] == '':
                path += '.pkl'
            folder = os.path.split(self.test_save_path)[0]
            for p_, arr in ((path, test_scores), (os.path.join(folder, "losses.pkl"), losses),
                            (os.path.join(folder, "solution.pkl"), test_solutions)):
                with open(p_, 'wb+') as output:
                    pickle.dump(np.array(arr), output, pickle.HIGHEST_PROTOCOL)
                if verbose:
                    print('saved to {}'.format(p_))
        self.test_scores, self.test_solutions = test_scores, test_solutions
        self.evaluations_run = sum(1 for i in range(n_eval) if i % world == rank)  # by this rank
        return losses[-100:]

    def _overlap_ok(self, env):
        """learn() overlaps an evaluation with training (side stream, weight snapshot) when it takes the one-fill
        path, the test env runs on the default stream (its kernels are then ordered by the side stream alone), and
        training cannot rewrite the test env's graphs meanwhile (regenerate_graphs on the store the test env reads,
        i.e. test_envs=None): otherwise the evaluation runs synchronously."""
        if not (self.overlap_evaluation and self._one_fill_ok(env, None)):
            return False
        if getattr(env, "stream", None) is not None:
            return False
        return not (self.regenerate_graphs is not None and env.graphs is self.graphs)

    def losses(self):
        """[[timestep, loss], ...] of every gradient step of the current (or last) learn() call
        (dqn.py:269,339; one host copy)."""
        n = getattr(self, "_loss_n", 0)
        s = getattr(self, "_loss_start", 0)
        if n <= s:
            return []
        vals = self._loss_buf[s:n].cpu().tolist()
        return [[int(t), v] for t, v in zip(self._loss_t[s:n], vals)]

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate_agent(self, batch_size=None, test_env=None):
        """dqn.py:514-602: greedy rollouts of `test_episodes` episodes, at most `batch_size`
        (default minibatch_size) at a time, on the test VecSpinSystem whose n_envs slots hold the
        concurrent episodes.  Episodes take the test graphs in order, continuing across calls (the
        ordered SetGraphGenerator of train_eco.py:69).  A finished episode's slot is refilled before
        the next prediction, and each prediction couples norm.max() over the active episodes only
        (predict on obs_batch, :546-547).  test_metric:
          BEST              -> (best_score, best_solution)  (:564-566)
          FINAL             -> (score, solution) of the final spins (:567-569)
          CUMULATIVE_REWARD -> (sum of rewards, 0)          (:560-561, :580-581)
          ENERGY_ERROR      -> (0, 0), as in the reference whose branch is commented out (:571-583)
        Returns (mean score, mean solution)."""
        env = self._test_env(test_env, batch_size)
        slots = min(int(batch_size or self.minibatch_size), env.n_envs)
        dev = self.device
        act_cfg = self._act_config(0.0)
        act_cfg.reversible = int(env.reversible_spins)
        act_cfg.allowed_value = float(env.allowed_action_value())
        if self._one_fill_ok(env, batch_size):
            return self._eval_one_fill_finish(self._eval_one_fill_launch(env, act_cfg, self.network))
        if not hasattr(env, "_eval_next_graph"):
            env._eval_next_graph = 0
        n_graphs = env.graphs.n_graphs
        # every slot holds a valid episode (unused ones run to their end and stay masked)
        env.reset(graph_ids=np.arange(env.n_envs) % n_graphs, seed=self.eval_seed)
        active = torch.zeros(env.n_envs, dtype=torch.bool, device=dev)
        cum = torch.zeros(env.n_envs, dtype=torch.float64, device=dev)
        acts = torch.zeros(env.n_envs, dtype=torch.int32, device=dev)
        scores, solutions = [], []
        started = 0
        metric = self.test_metric
        while len(scores) < self.test_episodes:
            free = (~active[:slots]).nonzero().flatten().cpu().numpy()
            take = free[:max(0, self.test_episodes - started)]
            if len(take):
                mask = np.zeros(env.n_envs, dtype=np.uint8)
                mask[take] = 1
                gids = np.zeros(env.n_envs, dtype=np.int64)
                gids[take] = (env._eval_next_graph + np.arange(len(take))) % n_graphs
                env._eval_next_graph = (env._eval_next_graph + len(take)) % n_graphs
                env.reset(graph_ids=gids, mask=mask, seed=self.eval_seed + started)
                active[torch.as_tensor(take, device=dev)] = True
                cum[torch.as_tensor(take, device=dev)] = 0.0
                started += len(take)
            idx = active.nonzero().flatten()
            act_cfg.counter = 0
            if len(idx) == env.n_envs:
                self.network.forward_graphs(env.obs_x, env.graphs, env.graph_ids, norm_scope=_lib.ECO_NORM_PER_CALL,
                                            act=act_cfg, actions_out=acts)
            else:
                sub = torch.empty(len(idx), dtype=torch.int32, device=dev)
                self.network.forward_graphs(env.obs_x[idx].contiguous(), env.graphs, env.graph_ids[idx],
                                            norm_scope=_lib.ECO_NORM_PER_CALL, act=act_cfg, actions_out=sub)
                acts.zero_()
                acts[idx] = sub
            _, rew, done = env.step(acts)
            cum[active] += rew[active]
            fin = active & done.bool()
            if bool(fin.any()):
                st = env.read()
                for i in fin.nonzero().flatten().cpu().tolist():
                    if metric == TestMetric.BEST:
                        sc, so = float(st["best_score"][i]), float(st["best_solution"][i])
                    elif metric == TestMetric.FINAL:
                        sc, so = float(st["score"][i]), self._final_solution(env, st, i)
                    elif metric == TestMetric.CUMULATIVE_REWARD:
                        sc, so = float(cum[i]), 0.0
                    else:
                        sc, so = 0.0, 0.0
                    scores.append(sc)
                    solutions.append(so)
                active &= ~fin
        if metric == TestMetric.ENERGY_ERROR:
            print("\n{}/{} graphs solved optimally".format(np.count_nonzero(np.array(scores) == 0),
                                                          self.test_episodes), end="")
        self.last_evaluation = (scores, solutions)  # per episode, in completion order
        return float(np.mean(scores)), float(np.mean(solutions))

    def _test_env(self, test_env=None, batch_size=None):
        env = test_env or self.test_envs
        if env is None:
            # dqn.py:225-227: test on the training environment(s) -- here a separate batch of episodes
            # over the training graph pool (the training episodes keep running untouched)
            from ...envs.batched import VecSpinSystem
            env = self.test_envs = VecSpinSystem(self.graphs, max(1, int(batch_size or self.minibatch_size)),
                                                 self.env.max_steps, **self.env.env_args)
        if isinstance(env, (list, tuple)):
            env = env[0]
        return env

    def _one_fill_ok(self, env, batch_size):
        """Every test episode fits the slots at once and ends exactly at max_steps (reversible spins,
        Stopping.NORMAL, spinsystem.py:539-554)."""
        slots = min(int(batch_size or self.minibatch_size), env.n_envs)
        return self.test_episodes <= slots and env.reversible_spins and env.cfg.stopping == 1

    def _eval_one_fill_launch(self, env, act_cfg, net):
        """evaluate_agent when every test episode fits the slots at once (the reference's 50 ER-200 test graphs
        in 64 slots) and every episode ends exactly at max_steps: the same resets, predictions and steps as the
        refill loop, issued with no host synchronisation (on the current stream).  The k episodes take slots
        0..k-1, so each prediction's batch (its norm.max() coupling, dqn.py:546-547) is the contiguous prefix
        obs_x[:k] -- all of them are active until the last step, as in the refill loop."""
        k = self.test_episodes
        n_graphs = env.graphs.n_graphs
        if not hasattr(env, "_eval_next_graph"):
            env._eval_next_graph = 0
        keep_cum = self.test_metric == TestMetric.CUMULATIVE_REWARD
        act_cfg.counter = 0
        net._ensure_packed()
        rec = self._eval_rollout_record(env, act_cfg, net, k, keep_cum)
        # the resets' graph ids and mask are formed on the device (no host upload, no synchronisation): every slot
        # holds a valid episode (unused ones run to their end and stay masked), as evaluate_agent, then slots
        # 0..k-1 take the next k test graphs
        slot = rec["slot"]
        env.reset(graph_ids=slot % n_graphs, seed=self.eval_seed)
        env.reset(graph_ids=(slot + env._eval_next_graph) % n_graphs, mask=rec["mask"], seed=self.eval_seed)
        env._eval_next_graph = (env._eval_next_graph + k) % n_graphs
        if keep_cum:
            rec["cum"].zero_()
        if rec["graph"] is not None:
            rec["graph"].replay()
        else:
            self._eval_rollout(env, act_cfg, net, k, rec)
            rec["eager_runs"] += 1
            if self.eval_graphs and net.timer is None:
                self._capture_eval_rollout(env, act_cfg, net, k, rec)
        env.read()
        # the results into pinned host memory behind the rollout (read by _eval_one_fill_finish once the stream's
        # event has fired: no device read on the training stream)
        rec["host_scalars"].copy_(env.scalars, non_blocking=True)
        if keep_cum:
            rec["host_cum"].copy_(rec["cum"], non_blocking=True)
        return {"env": env, "k": k, "cum": rec["host_cum"], "st": env.scalar_fields(rec["host_scalars"]),
                "metric": self.test_metric}

    def _eval_rollout(self, env, act_cfg, net, k, rec):
        """The one-fill evaluation's max_steps greedy steps: forward + fused greedy act over the k episodes, then
        the env step of every slot (dqn.py:536-558 without the host round trips)."""
        acts, cum = rec["acts"], rec["cum"]
        sub = acts[:k]
        scope = _lib.ECO_NORM_PER_CALL  # the batch obs_x[:k] never changes: its max degree once, then reused
        for _ in range(env.max_steps):
            net.forward_graphs(env.obs_x[:k], env.graphs, env.graph_ids[:k], norm_scope=scope,
                               act=act_cfg, actions_out=sub)
            _, rew, _ = env.step(acts)
            scope = _lib.ECO_NORM_PER_CALL_REUSE
            if rec["keep_cum"]:  # only the cumulative-reward metric reads it: one elementwise launch fewer per step
                cum += rew

    @staticmethod
    def _eval_rollout_key(env, act_cfg, net, k, keep_cum):
        """Everything the captured rollout's kernel arguments depend on: the buffers' device addresses (a
        reallocated workspace or feature buffer needs a new capture) and the act / env configuration."""
        ws = net._workspace(env.n_spins, k)
        ptrs = tuple(int(t.data_ptr()) if t is not None else 0 for t in
                     (env.obs_x, env.obs_f64, env.state, env.rewards, env.dones, env.graph_ids, net.packed, ws))
        return (ptrs, bytes(env.graphs.gs), bytes(env.cfg), env.n_envs, k, keep_cum, float(act_cfg.epsilon),
                int(act_cfg.reversible), float(act_cfg.allowed_value), int(act_cfg.seed))

    def _eval_rollout_record(self, env, act_cfg, net, k, keep_cum):
        """The (env, network) pair's rollout record: persistent action / cumulative-reward buffers and, from the
        second evaluation on, the HIP graph of the rollout's 2 x max_steps launches.  The record holds the env and
        the network (so every address the graph names stays allocated); a changed key drops the old graph."""
        key = self._eval_rollout_key(env, act_cfg, net, k, keep_cum)
        pair = (id(env), id(net))
        rec = self._eval_graphs.get(pair)
        if rec is None or rec["key"] != key:
            dev = self.device
            slot = torch.arange(env.n_envs, dtype=torch.int32, device=dev)
            rec = {"key": key, "env": env, "net": net, "graph": None, "eager_runs": 0, "keep_cum": keep_cum,
                   "acts": torch.zeros(env.n_envs, dtype=torch.int32, device=dev),
                   "cum": torch.zeros(env.n_envs, dtype=torch.float64, device=dev),
                   "slot": slot, "mask": (slot < k).to(torch.uint8),
                   "host_scalars": torch.zeros(env.scalars.shape, dtype=torch.float64).pin_memory(),
                   "host_cum": torch.zeros(env.n_envs, dtype=torch.float64).pin_memory()}
            self._eval_graphs[pair] = rec
        return rec

    def _capture_eval_rollout(self, env, act_cfg, net, k, rec):
        """Capture the rollout (2 x max_steps launches) into a HIP graph, replayed by the next evaluations of this
        (env, network) pair: one graph launch instead of ~800 host launches of ~20-30 us each, which otherwise
        leave the training stream without queued work while an overlapped evaluation is issued.  Captured after an
        eager run (workspaces allocated, kernels loaded); the capture itself executes nothing."""
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._eval_rollout(env, act_cfg, net, k, rec)
        rec["graph"] = g

    def _eval_one_fill_finish(self, p):
        """Scores of a launched one-fill evaluation, listed in completion order (end step, then slot), as the
        refill loop appends them."""
        env, k, cum, st, metric = p["env"], p["k"], p["cum"], p["st"], p["metric"]
        if p.get("done") is None:  # a synchronous evaluation: its copies were issued on the current stream
            p["done"] = torch.cuda.Event()
            p["done"].record()
        p["done"].synchronize()  # the host copies have landed (the side stream's work only)
        ends = st["current_step"][:k].numpy()
        order = np.lexsort((np.arange(k), ends))
        scores, solutions = [], []
        for i in order.tolist():
            if metric == TestMetric.BEST:
                sc, so = float(st["best_score"][i]), float(st["best_solution"][i])
            elif metric == TestMetric.FINAL:
                sc, so = float(st["score"][i]), self._final_solution(env, st, i)
            elif metric == TestMetric.CUMULATIVE_REWARD:
                sc, so = float(cum[i]), 0.0
            else:
                sc, so = 0.0, 0.0
            scores.append(sc)
            solutions.append(so)
        if metric == TestMetric.ENERGY_ERROR:
            print("\n{}/{} graphs solved optimally".format(np.count_nonzero(np.array(scores) == 0),
                                                          self.test_episodes), end="")
        self.last_evaluation = (scores, solutions)
        return float(np.mean(scores)), float(np.mean(solutions))

    @torch.no_grad()
    def _evaluate_overlapped(self, tk):
        """learn()'s evaluation at timestep tk without stopping training: the online weights are copied into a
        snapshot network on the training stream, and the one-fill evaluation runs on a side stream that waits
        for that copy only; training kernels keep going.  The evaluation's kernels and inputs are those of
        evaluate_agent() at tk, so its scores are identical; learn() records them (and saves the snapshot as
        `_best`) once the side stream's completion event has fired, or at the next evaluation / the end."""
        if self._eval_net is None:
            self._eval_net = self._network_factory()
        if self._eval_stream is None:
            self._eval_stream = torch.cuda.Stream(device=self.device)
        main = torch.cuda.current_stream(self.device)
        self._eval_net.flat.copy_(self.network.flat)
        snap = torch.cuda.Event()
        snap.record(main)
        env = self._test_env()
        act_cfg = self._act_config(0.0)
        act_cfg.reversible = int(env.reversible_spins)
        act_cfg.allowed_value = float(env.allowed_action_value())
        with torch.cuda.stream(self._eval_stream):
            self._eval_stream.wait_event(snap)
            p = self._eval_one_fill_launch(env, act_cfg, self._eval_net)
            p["done"] = torch.cuda.Event()
            p["done"].record(self._eval_stream)
        p["tk"], p["net"] = tk, self._eval_net
        return p

    @staticmethod
    def _final_solution(env, st, i):
        """scorer.get_solution of the episode's current spins (score_solver.py:263-271, 377-381,
        463-467, 537-544, 649-656, 776-783) from the env's integer state."""
        t = env.cfg.optimisation_target
        score, lb, qn = float(st["score"][i]), float(st["lower_bound"][i]), float(st["quality_normalizer"][i])
        invalid = float(st["invalidity"][i]) != 0
        size = float(st["set_size"][i])
        if t == _lib.ECO_TARGET_CUT:
            return score - abs(min(0.0, lb))
        if t == _lib.ECO_TARGET_MIN_CUT:
            return max(0.0, qn) - score
        if t in (_lib.ECO_TARGET_MIN_COVER, _lib.ECO_TARGET_MIN_DOM_SET):
            return float(env.n_spins) if invalid else size
        return 0.0 if invalid else size

    # ------------------------------------------------------------ checkpoint
    def _save_flat(self, path, flat):
        """save() of a parameter vector in state_dict order (a host copy of MPNN.flat): the same keys and
        tensors as the network's state_dict (mpnn.MPNN.flat views)."""
        from ...networks.mpnn import param_layout
        sd, off = {}, 0
        for name, shape in param_layout(self.network.n_obs_in):
            cnt = int(np.prod(shape))
            sd[name] = flat[off:off + cnt].view(shape).clone()
            off += cnt
        assert off == flat.numel()
        torch.save(sd, path)

    def save(self, path='network.pth', network=None):
        """dqn.py:604-607: torch.save(state_dict) -- loadable by the reference MPNN.  The reference's
        extension fix-up is a no-op expression (`path + '.pth'`, :606), so `path` is used as given.
        network: another network to save (learn()'s evaluation snapshot); default the online network."""
        net = self.network if network is None else network
        torch.save({k: v.detach().cpu().clone() for k, v in net.state_dict().items()}, path)

    def load(self, path):
        """dqn.py:609-610 (weights_only: state_dicts are plain tensors)."""
        self.network.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
