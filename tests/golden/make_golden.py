"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference; never on the GPU box):
    python tests/golden/make_golden.py

How the reference is imported: `/root/reference` is put on sys.path and
`tests/golden/_shim` supplies an identity `numba.jit` (numba is not installed in
this image: an ordinary ModuleNotFoundError at src/envs/utils.py:8).  For integer
edge weights `calculate_cut_changes` (src/envs/utils.py:97-102) is integer-valued,
so jitting cannot change any result.  The pretrained `.pth` state_dicts are read
with `torch.load(..., weights_only=True)`.  Graph pickles under `_graphs/` are NOT
loaded (no unpickling of reference files): graphs come from oracle/graphs.py.

Every fixture is data (inputs + the reference's outputs) -- no reference source.
"""
import hashlib
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(HERE, "_shim"))

import src.envs.core as ising_env                       # noqa: E402
from src.envs.utils import (SingleGraphGenerator, RewardSignal, ExtraAction,   # noqa: E402
                            OptimisationTarget, SpinBasis, DEFAULT_OBSERVABLES, Observable)
from src.networks.mpnn import MPNN                      # noqa: E402
from src.agents.dqn.dqn import DQN                      # noqa: E402
from oracle import graphs                               # noqa: E402


def env_args(mode, n, basis="SIGNED"):
    """experiments/train_eco.py:40-50,255-264 (eco) and :311-315 (s2v)."""
    a = {'observables': DEFAULT_OBSERVABLES,
         'reward_signal': RewardSignal.BLS,
         'extra_action': ExtraAction.NONE,
         'optimisation_target': OptimisationTarget.CUT,
         'spin_basis': SpinBasis.SIGNED if basis == "SIGNED" else SpinBasis.BINARY,
         'norm_rewards': True,
         'memory_length': None,
         'horizon_length': None,
         'stag_punishment': None,
         'basin_reward': 1. / n,
         'reversible_spins': True}
    if mode == "s2v":
        a.update(observables=[Observable.SPIN_STATE], reversible_spins=False,
                 basin_reward=None, reward_signal=RewardSignal.DENSE)
    if mode == "pretrained":          # experiments/pretrained_agent/test_eco.py:57-67
        a.update(basin_reward=None, spin_basis=SpinBasis.BINARY)
    return a


def digest(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.uint64)[0]


def run_episode(J, T, mode, spins, actions, basis="SIGNED", full_steps=None):
    """Drive the reference env; return per-step records."""
    n = J.shape[0]
    env = ising_env.make("SpinSystem", SingleGraphGenerator(J), T, **env_args(mode, n, basis))
    n_obs = len(env.observables)
    obs = env.reset(spins=spins)
    rec = dict(obs=[obs[:n_obs].copy()], rew=[], done=[], score=[env.score], nscore=[env.normalized_score],
               best_score=[env.best_score], best_nscore=[env.best_score_normalized],
               best_solution=[env.best_solution], mlr=env.scorer._max_local_reward,
               qn=env.scorer._solution_quality_normalizer, lb=env.scorer._lower_bound)
    for a in actions:
        obs, rew, done, _ = env.step(int(a))
        rec["obs"].append(obs[:n_obs].copy())
        rec["rew"].append(float(rew))
        rec["done"].append(bool(done))
        rec["score"].append(env.score)
        rec["nscore"].append(env.normalized_score)
        rec["best_score"].append(env.best_score)
        rec["best_nscore"].append(env.best_score_normalized)
        rec["best_solution"].append(env.best_solution)
        if done:
            break
    # step past the end must raise NotImplementedError (spinsystem.py:365-367)
    raised = False
    if rec["done"] and rec["done"][-1] and env.current_step == env.max_steps:
        try:
            env.step(0)
        except NotImplementedError:
            raised = True
    rec["raised_past_end"] = raised
    return rec


def pack_env_cases(cases, full=True, full_steps=()):
    out = {}
    for ci, c in enumerate(cases):
        p = f"c{ci}_"
        rec = c["rec"]
        out[p + "J"] = c["J"].astype(np.int8)
        out[p + "T"] = np.int64(c["T"])
        out[p + "mode"] = np.array(c["mode"])
        out[p + "basis"] = np.array(c["basis"])
        out[p + "spins"] = np.asarray(c["spins"], dtype=np.int8)
        out[p + "actions"] = np.asarray(c["actions"], dtype=np.int32)
        obs = np.stack(rec["obs"])
        if full:
            out[p + "obs"] = obs
        else:
            out[p + "obs_digest"] = np.array([digest(o) for o in obs], dtype=np.uint64)
            steps = [s for s in full_steps if s < len(obs)]
            out[p + "obs_steps"] = np.array(steps, dtype=np.int64)
            out[p + "obs_at"] = obs[steps]
        for k in ("rew", "score", "nscore", "best_score", "best_nscore", "best_solution"):
            out[p + k] = np.asarray(rec[k], dtype=np.float64)
        out[p + "done"] = np.asarray(rec["done"], dtype=bool)
        out[p + "mlr"] = np.float64(rec["mlr"])
        out[p + "qn"] = np.float64(rec["qn"])
        out[p + "lb"] = np.float64(rec["lb"])
        out[p + "raised_past_end"] = np.bool_(rec["raised_past_end"])
    out["n_cases"] = np.int64(len(cases))
    return out


def make_env_er20():
    rng = np.random.default_rng(20)
    cases = []
    for gi in range(8):
        n = 20
        if gi == 6:
            J = graphs.negative_mlr_graph(n, rng)            # mlr <= 0 trap
        elif gi == 7:
            J = graphs.er_graph(n, 0.15, rng, "uniform")     # EdgeType.UNIFORM
        else:
            J = graphs.er_graph(n, 0.15, rng)                # isolated vertices common at p=.15
        T = 2 * n
        mode = "s2v" if gi == 5 else "eco"
        basis = "BINARY" if gi == 4 else "SIGNED"
        if mode == "s2v":
            spins = -np.ones(n, dtype=np.int64)
            actions = rng.permutation(n)                      # irreversible: each spin once
            T = n
        else:
            spins = 2 * rng.integers(0, 2, n) - 1
            actions = rng.integers(0, n, T)
        if gi == 3:
            # revisit pattern: flip back and forth to exercise the visited-set quirk
            actions = np.array([int(a) for a in rng.integers(0, n, T // 2) for _ in (0, 1)])
        sp = (1 - spins) // 2 if basis == "BINARY" else spins
        rec = run_episode(J, T, mode, sp, actions, basis)
        cases.append(dict(J=J, T=T, mode=mode, basis=basis, spins=sp, actions=actions, rec=rec))
    np.savez_compressed(os.path.join(HERE, "env_er20.npz"), **pack_env_cases(cases))


def make_env_large():
    rng = np.random.default_rng(200)
    cases = []
    for kind, n, extra in (("ER", 200, 0.15), ("ER", 200, 0.15), ("BA", 500, 4)):
        J = graphs.er_graph(n, extra, rng) if kind == "ER" else graphs.ba_graph(n, extra, rng)
        T = 2 * n
        spins = 2 * rng.integers(0, 2, n) - 1
        actions = rng.integers(0, n, T)
        rec = run_episode(J, T, "eco", spins, actions)
        cases.append(dict(J=J, T=T, mode="eco", basis="SIGNED", spins=spins, actions=actions, rec=rec))
    np.savez_compressed(os.path.join(HERE, "env_large.npz"),
                        **pack_env_cases(cases, full=False, full_steps=(0, 1, 2, 3, 5, 100, 200, 399, 400, 999, 1000)))


def obs_after_random_steps(J, T, n_steps, rng, basis="SIGNED", mode="eco"):
    n = J.shape[0]
    env = ising_env.make("SpinSystem", SingleGraphGenerator(J), T, **env_args(mode, n, basis))
    spins = 2 * rng.integers(0, 2, n) - 1
    obs = env.reset(spins=(1 - spins) // 2 if basis == "BINARY" else spins)
    for a in rng.integers(0, n, n_steps):
        obs, _, _, _ = env.step(int(a))
    return obs


def state_dict_np(net):
    return {k: v.detach().cpu().numpy().copy() for k, v in net.state_dict().items()}


def make_mpnn():
    rng = np.random.default_rng(7)
    out = {}
    # (i) pretrained ECO ER-200 weights (MIT, experiments/pretrained_agent/networks/eco)
    sd = torch.load(os.path.join(REF, "experiments/pretrained_agent/networks/eco/network_best_ER_200spin.pth"),
                    map_location="cpu", weights_only=True)
    net = MPNN(n_obs_in=7, n_layers=3, n_features=64, n_hid_readout=[], tied_weights=False)
    net.load_state_dict(sd)
    net.eval()
    for k, v in state_dict_np(net).items():
        out["er200/" + k] = v
    Js = [graphs.er_graph(200, 0.15, rng) for _ in range(2)]
    obs = [obs_after_random_steps(J, 400, 37, rng) for J in Js]
    with torch.no_grad():
        q_b1 = [net(torch.FloatTensor(o.copy())).numpy() for o in obs]
        q_b2 = net(torch.FloatTensor(np.array(obs))).numpy()
    out["er200/obs"] = np.array(obs)
    out["er200/q_b1"] = np.array(q_b1)
    out["er200/q_b2"] = q_b2
    # (iii) BINARY-basis observation for the same net (pretrained script's env args)
    ob = obs_after_random_steps(Js[0], 400, 11, rng, basis="BINARY", mode="pretrained")
    with torch.no_grad():
        out["er200/obs_binary"] = ob
        out["er200/q_binary"] = net(torch.FloatTensor(ob.copy())).numpy()
    # (ii) ER-20, seeded normal(0, 0.01) init (dqn.py:199-205), batch of 8 incl. isolated vertices
    torch.manual_seed(1234)
    net20 = MPNN(n_obs_in=7, n_layers=3, n_features=64, n_hid_readout=[], tied_weights=False)
    with torch.no_grad():
        for m in net20.modules():
            if type(m) == torch.nn.Linear:
                m.weight.normal_(0, 0.01)
    for k, v in state_dict_np(net20).items():
        out["er20/" + k] = v
    Js20 = [graphs.er_graph(20, 0.15, rng) for _ in range(8)]
    obs20 = np.array([obs_after_random_steps(J, 40, 9, rng) for J in Js20])
    with torch.no_grad():
        out["er20/q_b8"] = net20(torch.FloatTensor(obs20)).numpy()
        out["er20/q_b1"] = np.array([net20(torch.FloatTensor(o.copy())).numpy() for o in obs20])
    out["er20/obs"] = obs20
    # in-place transpose quirk (mpnn.py:44): a float32 3-D input is mutated to [B, N, 7+N]
    t = torch.FloatTensor(obs20.copy())
    with torch.no_grad():
        net20(t)
    out["er20/input_after_forward"] = t.numpy()
    np.savez_compressed(os.path.join(HERE, "mpnn_fwd.npz"), **out)


def make_dqn_step():
    """Three consecutive DQN.train_step calls (dqn.py:403-451) on ER-20 transitions."""
    rng = np.random.default_rng(99)
    n, M = 20, 16
    J = graphs.er_graph(n, 0.15, rng)
    env = ising_env.make("SpinSystem", SingleGraphGenerator(J), 2 * n, **env_args("eco", n))
    net_fn = lambda: MPNN(n_obs_in=7, n_layers=3, n_features=64, n_hid_readout=[], tied_weights=False)  # noqa: E731
    agent = DQN([env], net_fn, init_weight_std=0.01, double_dqn=True, clip_Q_targets=False,
                replay_start_size=10, replay_buffer_size=100, gamma=0.95, update_target_frequency=1000,
                update_learning_rate=False, initial_learning_rate=1e-4, peak_learning_rate=1e-4,
                final_learning_rate=1e-4, update_frequency=32, minibatch_size=M, max_grad_norm=None,
                weight_decay=0, update_exploration=True, initial_exploration_rate=1,
                final_exploration_rate=0.05, final_exploration_step=150000, adam_epsilon=1e-8,
                logging=False, loss="mse", save_network_frequency=10**9, network_save_path="/tmp/n.pth",
                evaluate=False, test_envs=None, test_episodes=1, test_frequency=10**9,
                test_save_path="/tmp/ts.pkl", seed=5)
    # perturb the target net so double-DQN's argmax(online) != argmax(target) matters
    with torch.no_grad():
        for p in agent.target_network.parameters():
            p.add_(torch.randn_like(p) * 0.01)
    out = {}
    for k, v in state_dict_np(agent.network).items():
        out["w0/" + k] = v
    for k, v in state_dict_np(agent.target_network).items():
        out["target/" + k] = v
    steps = 3
    for s in range(steps):
        sts, acts, rews, nxt, dns = [], [], [], [], []
        for _ in range(M):
            Jg = graphs.er_graph(n, 0.15, rng)
            e = ising_env.make("SpinSystem", SingleGraphGenerator(Jg), 2 * n, **env_args("eco", n))
            o = e.reset(spins=2 * rng.integers(0, 2, n) - 1)
            for a in rng.integers(0, n, int(rng.integers(0, 2 * n - 1))):
                o, _, _, _ = e.step(int(a))
            a = int(rng.integers(0, n))
            o2, r, d, _ = e.step(a)
            sts.append(o); acts.append([a]); rews.append([r]); nxt.append(o2); dns.append([float(d)])
        tr = [torch.as_tensor(np.array(sts)), torch.as_tensor(np.array(acts), dtype=torch.long),
              torch.as_tensor(np.array(rews), dtype=torch.float), torch.as_tensor(np.array(nxt)),
              torch.as_tensor(np.array(dns), dtype=torch.float)]
        out[f"s{s}/states"] = np.array(sts)
        out[f"s{s}/actions"] = np.array(acts)
        out[f"s{s}/rewards"] = np.array(rews, dtype=np.float32)
        out[f"s{s}/states_next"] = np.array(nxt)
        out[f"s{s}/dones"] = np.array(dns, dtype=np.float32)
        loss = agent.train_step(tr)
        out[f"s{s}/loss"] = np.float64(loss)
        for k, v in state_dict_np(agent.network).items():
            out[f"s{s}/w/" + k] = v
    out["steps"] = np.int64(steps)
    np.savez_compressed(os.path.join(HERE, "dqn_step.npz"), **out)


def make_dqn_step_s2v():
    """Three DQN.train_step calls on IRREVERSIBLE (S2V) ER-20 transitions: the -10000 masking of
    disallowed actions before the double-DQN argmax (dqn.py:414-428), including terminal next
    states where every spin is flipped (all actions masked: argmax 0, (1 - done) zeroes the term)."""
    rng = np.random.default_rng(1999)
    n, M = 20, 16
    J = graphs.er_graph(n, 0.15, rng)
    env = ising_env.make("SpinSystem", SingleGraphGenerator(J), n, **env_args("s2v", n))
    net_fn = lambda: MPNN(n_obs_in=1, n_layers=3, n_features=64, n_hid_readout=[], tied_weights=False)  # noqa: E731
    agent = DQN([env], net_fn, init_weight_std=0.01, double_dqn=True, clip_Q_targets=False,
                replay_start_size=10, replay_buffer_size=100, gamma=0.95, update_target_frequency=1000,
                update_learning_rate=False, initial_learning_rate=1e-4, peak_learning_rate=1e-4,
                final_learning_rate=1e-4, update_frequency=32, minibatch_size=M, max_grad_norm=None,
                weight_decay=0, update_exploration=True, initial_exploration_rate=1,
                final_exploration_rate=0.05, final_exploration_step=150000, adam_epsilon=1e-8,
                logging=False, loss="mse", save_network_frequency=10**9, network_save_path="/tmp/n.pth",
                evaluate=False, test_envs=None, test_episodes=1, test_frequency=10**9,
                test_save_path="/tmp/ts.pkl", seed=6)
    with torch.no_grad():
        for p in agent.target_network.parameters():
            p.add_(torch.randn_like(p) * 0.01)
    out = {"allowed_action_state": np.float64(agent.allowed_action_state)}
    for k, v in state_dict_np(agent.network).items():
        out["w0/" + k] = v
    for k, v in state_dict_np(agent.target_network).items():
        out["target/" + k] = v
    steps = 3
    for s in range(steps):
        sts, acts, rews, nxt, dns = [], [], [], [], []
        for i in range(M):
            Jg = graphs.er_graph(n, 0.15, rng)
            e = ising_env.make("SpinSystem", SingleGraphGenerator(Jg), n, **env_args("s2v", n))
            o = e.reset()
            order = rng.permutation(n)
            # every 4th transition is the episode's last flip (terminal s')
            k = n - 1 if i % 4 == 0 else int(rng.integers(0, n - 1))
            for a in order[:k]:
                o, _, _, _ = e.step(int(a))
            a = int(order[k])
            o2, r, d, _ = e.step(a)
            sts.append(o); acts.append([a]); rews.append([r]); nxt.append(o2); dns.append([float(d)])
        tr = [torch.as_tensor(np.array(sts)), torch.as_tensor(np.array(acts), dtype=torch.long),
              torch.as_tensor(np.array(rews), dtype=torch.float), torch.as_tensor(np.array(nxt)),
              torch.as_tensor(np.array(dns), dtype=torch.float)]
        out[f"s{s}/states"] = np.array(sts)
        out[f"s{s}/actions"] = np.array(acts)
        out[f"s{s}/rewards"] = np.array(rews, dtype=np.float32)
        out[f"s{s}/states_next"] = np.array(nxt)
        out[f"s{s}/dones"] = np.array(dns, dtype=np.float32)
        loss = agent.train_step(tr)
        out[f"s{s}/loss"] = np.float64(loss)
        for k2, v in state_dict_np(agent.network).items():
            out[f"s{s}/w/" + k2] = v
    out["steps"] = np.int64(steps)
    np.savez_compressed(os.path.join(HERE, "dqn_step_s2v.npz"), **out)


def make_schedules():
    """DQN.update_epsilon / update_lr (dqn.py:467-488) over a range of timesteps for two
    hyper-parameter sets (train_eco.py:136-146 and a warm-up/decay learning-rate schedule)."""
    n = 20
    J = graphs.er_graph(n, 0.15, np.random.default_rng(5))
    env = ising_env.make("SpinSystem", SingleGraphGenerator(J), 2 * n, **env_args("eco", n))
    net_fn = lambda: MPNN(n_obs_in=7, n_layers=3, n_features=64, n_hid_readout=[], tied_weights=False)  # noqa: E731
    sets = [dict(initial_exploration_rate=1, final_exploration_rate=0.05, final_exploration_step=800000,
                 initial_learning_rate=1e-4, peak_learning_rate=1e-4, peak_learning_rate_step=20000,
                 final_learning_rate=1e-4, final_learning_rate_step=200000),
            dict(initial_exploration_rate=0.9, final_exploration_rate=0.1, final_exploration_step=12345,
                 initial_learning_rate=0, peak_learning_rate=1e-3, peak_learning_rate_step=10000,
                 final_learning_rate=5e-5, final_learning_rate_step=200000)]
    ts = np.array([0, 1, 7, 999, 5000, 10000, 10001, 12345, 12346, 20000, 100000, 199999, 200000, 200001,
                   799999, 800000, 10 ** 7], dtype=np.int64)
    out = {"timesteps": ts}
    for i, hp in enumerate(sets):
        agent = DQN([env], net_fn, replay_start_size=10, replay_buffer_size=100, logging=False,
                    evaluate=False, seed=1, network_save_path="/tmp/n.pth", test_save_path="/tmp/ts.pkl", **hp)
        eps, lrs = [], []
        for t in ts:
            agent.update_epsilon(int(t))
            agent.update_lr(int(t))
            eps.append(agent.epsilon)
            lrs.append(agent.optimizer.param_groups[0]["lr"])
        out[f"h{i}/eps"] = np.array(eps, dtype=np.float64)
        out[f"h{i}/lr"] = np.array(lrs, dtype=np.float64)
        for k, v in hp.items():
            out[f"h{i}/{k}"] = np.float64(v)
    np.savez_compressed(os.path.join(HERE, "schedules.npz"), **out)


def make_exploration():
    """DQN.learn's epsilon trace (dqn.py:284-286) with update_exploration False and True: dqn.py:161 stores
    a one-tuple, so epsilon decays either way.  update_epsilon is wrapped to record (timestep, epsilon)
    after every call; replay_start_size > timesteps, so no train_step runs."""
    n, T = 20, 60
    J = graphs.er_graph(n, 0.15, np.random.default_rng(8))
    net_fn = lambda: MPNN(n_obs_in=7, n_layers=3, n_features=64, n_hid_readout=[], tied_weights=False)  # noqa: E731
    out = {}
    for flag in (False, True):
        env = ising_env.make("SpinSystem", SingleGraphGenerator(J), 2 * n, **env_args("eco", n))
        agent = DQN([env], net_fn, replay_start_size=10 ** 6, replay_buffer_size=1000, logging=False,
                    evaluate=False, seed=1, network_save_path="/tmp/n.pth", test_save_path="/tmp/ts.pkl",
                    update_exploration=flag, initial_exploration_rate=1, final_exploration_rate=0.1,
                    final_exploration_step=40, update_learning_rate=False, initial_learning_rate=1e-4)
        trace = []
        orig = agent.update_epsilon

        def rec(t, orig=orig, trace=trace):
            orig(t)
            trace.append((t, agent.epsilon))
        agent.update_epsilon = rec
        agent.learn(T)
        out[f"{int(flag)}/attr_truthy"] = np.bool_(bool(agent.update_exploration))
        out[f"{int(flag)}/timesteps"] = np.array([t for t, _ in trace], dtype=np.int64)
        out[f"{int(flag)}/eps"] = np.array([e for _, e in trace], dtype=np.float64)
        out[f"{int(flag)}/final_eps"] = np.float64(agent.epsilon)
    np.savez_compressed(os.path.join(HERE, "exploration.npz"), **out)


def make_greedy_rollout():
    """Pretrained-net greedy rollout (dqn.py:490-512 predict) on one ER-200 graph:
    actions plus the top-1/top-2 Q margin per step (argmax-tie robustness)."""
    rng = np.random.default_rng(4242)
    n = 200
    J = graphs.er_graph(n, 0.15, rng)
    sd = torch.load(os.path.join(REF, "experiments/pretrained_agent/networks/eco/network_best_ER_200spin.pth"),
                    map_location="cpu", weights_only=True)
    net = MPNN(n_obs_in=7, n_layers=3, n_features=64, n_hid_readout=[], tied_weights=False)
    net.load_state_dict(sd)
    net.eval()
    env = ising_env.make("SpinSystem", SingleGraphGenerator(J), 2 * n, **env_args("eco", n))
    spins = 2 * rng.integers(0, 2, n) - 1
    obs = env.reset(spins=spins)
    acts, margins, rews = [], [], []
    done = False
    with torch.no_grad():
        while not done:
            q = net(torch.FloatTensor(obs.copy()))
            top = torch.topk(q, 2).values
            a = int(q.argmax().item())
            acts.append(a)
            margins.append(float(top[0] - top[1]))
            obs, r, done, _ = env.step(a)
            rews.append(float(r))
    np.savez_compressed(os.path.join(HERE, "greedy_er200.npz"), J=J.astype(np.int8), spins=spins.astype(np.int8),
                        actions=np.array(acts, np.int32), margins=np.array(margins), rewards=np.array(rews),
                        best_solution=np.float64(env.best_solution), best_score=np.float64(env.best_score))


def make_greedy_solver():
    """The reference Greedy solver rule (src/agents/solver.py:100-131) driven on the reference env:
    action = argmax(env.scorer.get_score_mask(state)); stop when that change is negative.
    (solver.py itself imports docplex, which is absent here, so its 10-line rule is applied
    directly to the reference env/scorer objects.)"""
    rng = np.random.default_rng(31)
    out = {}
    cases = []
    for kind, n in (("ER", 20), ("ER", 20), ("ER", 200), ("BA", 60)):
        J = graphs.er_graph(n, 0.15, rng) if kind == "ER" else graphs.ba_graph(n, 4, rng)
        for init in ("minus", "random"):
            spins = -np.ones(n, dtype=np.int64) if init == "minus" else 2 * rng.integers(0, 2, n) - 1
            env = ising_env.make("SpinSystem", SingleGraphGenerator(J), 2 * n, **env_args("eco", n))
            env.reset(spins=spins)
            acts = []
            done = False
            while not done:
                mask = env.scorer.get_score_mask(env.state[0, :env.n_spins], env.matrix)
                a = int(mask.argmax())
                if mask[a] < 0:
                    break
                _, _, done, _ = env.step(a)
                acts.append(a)
            cases.append((J, spins, acts, env.best_solution, env.best_score))
    for i, (J, spins, acts, bsol, bsc) in enumerate(cases):
        out[f"c{i}_J"] = J.astype(np.int8)
        out[f"c{i}_spins"] = spins.astype(np.int8)
        out[f"c{i}_actions"] = np.array(acts, dtype=np.int32)
        out[f"c{i}_best_solution"] = np.float64(bsol)
        out[f"c{i}_best_score"] = np.float64(bsc)
    out["n_cases"] = np.int64(len(cases))
    np.savez_compressed(os.path.join(HERE, "greedy_solver.npz"), **out)


PROBLEMS = (("MIN_COVER", "uniform"), ("MAX_IND_SET", "uniform"), ("MAX_CLIQUE", "uniform"),
            ("MIN_DOM_SET", "uniform"), ("MIN_CUT", "discrete"), ("CUT", "uniform"))
MAIN_OBS = [Observable(v) for v in range(1, 14)]   # src/envs/utils.py:76-88


def problem_args(target, mode, n):
    """experiments/train_eco.py:244-315: MAIN_OBSERVABLES for the set problems, DEFAULT_OBSERVABLES for the
    cut problems (the validity-mask observables raise TypeError with a cut scorer); s2v as :311-315."""
    a = env_args("eco", n)
    a["optimisation_target"] = OptimisationTarget[target]
    if target not in ("CUT", "MIN_CUT"):
        a["observables"] = MAIN_OBS
    if mode == "s2v":
        a.update(observables=[Observable.SPIN_STATE], reversible_spins=False, basin_reward=None,
                 reward_signal=RewardSignal.DENSE)
    return a


def make_env_problems():
    """Every OptimisationTarget scorer (score_solver.py:232-858) through the reference env.  Each case's env
    is built on graph J0 (the constructor draws once, :154, and resets once, :168) and then reset onto graph J with
    the recorded spins, so the stale invalidity normaliser of the first observation (set only after
    _reset_state, :216-219) comes from J0.  A greedy rollout (solver.py:110-127 rule on the scorer's score
    mask) from the same start is recorded as well."""
    from src.envs.utils import SetGraphGenerator
    rng = np.random.default_rng(77)
    out = {}
    ci = 0
    for target, w in PROBLEMS:
        for mode in ("eco", "s2v"):
            for n, p in ((20, 0.15), (24, 0.35)):
                J0 = graphs.er_graph(n, p, rng, w)
                J = graphs.er_graph(n, p, rng, w)
                T = 2 * n if mode == "eco" else n
                env = ising_env.make("SpinSystem", SetGraphGenerator([J0, J0, J], ordered=True), T,
                                     **problem_args(target, mode, n))
                if mode == "s2v":
                    spins = -np.ones(n, dtype=np.int64)
                    actions = rng.permutation(n)
                else:
                    spins = 2 * rng.integers(0, 2, n) - 1
                    actions = rng.integers(0, n, T)
                n_obs = len(env.observables)
                obs = env.reset(spins=spins)
                assert np.array_equal(env.matrix, J)
                sc = env.scorer
                rec = dict(obs=[obs[:n_obs].copy()], rew=[], done=[], score=[env.score], nscore=[env.normalized_score],
                           best_score=[env.best_score], best_nscore=[env.best_score_normalized],
                           best_solution=[env.best_solution])
                norms = [sc._max_local_reward, sc._solution_quality_normalizer, sc._invalidity_normalizer,
                         sc._lower_bound]
                for a in actions:
                    obs, rew, done, _ = env.step(int(a))
                    rec["obs"].append(obs[:n_obs].copy())
                    rec["rew"].append(float(rew))
                    rec["done"].append(bool(done))
                    for k, v in (("score", env.score), ("nscore", env.normalized_score),
                                 ("best_score", env.best_score), ("best_nscore", env.best_score_normalized),
                                 ("best_solution", env.best_solution)):
                        rec[k].append(v)
                    if done:
                        break
                # greedy rollout from the same start on the same graph
                genv = ising_env.make("SpinSystem", SingleGraphGenerator(J), T, **problem_args(target, mode, n))
                genv.reset(spins=spins)
                gacts, gdone = [], False
                while not gdone:
                    mask = genv.scorer.get_score_mask(genv.state[0, :genv.n_spins], genv.matrix)
                    m = np.array(mask, dtype=np.float64)
                    if not genv.reversible_spins:
                        np.putmask(m, genv.state[0, :genv.n_spins] != -1, np.finfo(np.float64).min)
                    a = int(m.argmax())
                    if m[a] < 0:
                        break
                    _, _, gdone, _ = genv.step(a)
                    gacts.append(a)
                q = f"c{ci}_"
                out[q + "target"] = np.array(target)
                out[q + "mode"] = np.array(mode)
                out[q + "J0"] = J0.astype(np.int8)
                out[q + "J"] = J.astype(np.int8)
                out[q + "T"] = np.int64(T)
                out[q + "spins"] = spins.astype(np.int8)
                out[q + "actions"] = np.asarray(actions, dtype=np.int32)
                out[q + "obs"] = np.stack(rec["obs"])
                for k in ("rew", "score", "nscore", "best_score", "best_nscore", "best_solution"):
                    out[q + k] = np.asarray(rec[k], dtype=np.float64)
                out[q + "done"] = np.asarray(rec["done"], dtype=bool)
                out[q + "norms"] = np.asarray(norms, dtype=np.float64)   # mlr, qn, invalidity normaliser, lb
                out[q + "greedy_actions"] = np.asarray(gacts, dtype=np.int32)
                out[q + "greedy_best_solution"] = np.float64(genv.best_solution)
                out[q + "greedy_best_score"] = np.float64(genv.best_score)
                ci += 1
    out["n_cases"] = np.int64(ci)
    np.savez_compressed(os.path.join(HERE, "env_problems.npz"), **out)


if __name__ == "__main__":
    random.seed(0)
    np.random.seed(0)
    which = sys.argv[1:] or ["env_er20", "env_large", "mpnn", "dqn_step", "dqn_step_s2v", "schedules", "exploration",
                              "greedy_rollout", "greedy_solver",
                              "env_problems"]
    for w in which:
        globals()["make_" + w]()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
