#!/usr/bin/env python
"""Benchmark: env-steps/sec (batched episodes) on ER-200 MaxCut (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload train|rollout] [--envs B] [--n N]

Default workload = BASELINE.json configs[2]: ER_200spin, 8192 parallel episodes per
GPU (each on its own graph), the FULL ECO-DQN train loop:
  one step = one vector step of DQN.learn over all B episodes:
     MPNN forward + fused eps-greedy act, batched env step, replay add,
     then K = B * (64/32) / M gradient steps of minibatch M (replay ratio of
     train_eco.py:136-137): replay sample, online(s') argmax, target(s') gather,
     online(s) forward, TD + MSE grad, MPNN backward, Adam, target sync.
  "rollout" = the act + env step part only.
value = B * K * world / max-over-ranks(time): episodes shard across ranks; the
train loop all-reduces gradients over RCCL (weak scaling, B fixed per GPU).

Prints ONE JSON line on rank 0 with
  roofline: dominant kernel measured live with HIP events (on the launch stream),
            algorithmic FLOPs from SURVEY.md 8d: forward F = 1392*nnz + 107,648*N + 8,192
            per graph, backward = 2F; peak = the dense peak of the MFMA dtype the kernel ISSUES
            (f16 / bf16, 2.5 PFLOP/s: the fp16x2 split kernels; bf16x3 in the per-episode N > 512 one), frac <= 1 by construction;
            the f32-MFMA figure (157.3) is kept as a separately named field.
  env_step_roofline: the env step kernel alone (same B, N), SURVEY.md 8d incremental algorithmic bytes
            per env-step (N + 14.25 N + 28 N) x rate / HBM peak (8 TB/s).
  cpu_baseline: the oracle ('port') env + torch-CPU MPNN act loop on this host.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "eco-dqn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32-input MFMA peak
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E peak ~8 TB/s


def envstep_alg_bytes(n):
    """SURVEY.md 8d algorithmic HBM bytes of one incremental env-step: one column of J (N), the episode
    state read + written (spins N, h 4N, tsf 2N, best bitset N/8: 14.25N) and the fp32 observation rows
    (7 x 4 B = 28N)."""
    return n + 14.25 * n + 28.0 * n


def envstep_roofline(rate, ms, n, B=None):
    """env_step_roofline object from a measured env-step rate (env-steps/s) and mean launch time; traffic = the
    PMC HBM bytes per launch of the committed train profile (ER-200 x 8192 only)."""
    bpe = envstep_alg_bytes(n)
    achieved = bpe * rate / 1e9
    traffic = None
    if n == 200 and B == 8192:
        try:
            with open(PMC_SUMMARY) as f:
                k = json.load(f)["kernels"]
            traffic = k["env_step_fast_kernel"][str(B // 4)]["hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            traffic = None
    return {"bound": "hbm", "kernel": "env_step_fast_kernel" if n <= 256 else "env_step_kernel",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC, %s)" % os.path.relpath(PMC_SUMMARY, REPO),
            "alg_bytes_per_launch": bpe * B if B else None, "alg_bytes_per_env_step": bpe, "env_steps_per_s": rate,
            "avg_launch_ms": ms, "source": "SURVEY.md 8d incremental bytes x the env step kernel's rate (launches "
                                          "replayed from a HIP graph, HIP events, random actions, same B and N)"}


def mpnn_flops(nnz, n):
    """algorithmic forward FLOPs of one graph."""
    return 1392.0 * nnz + 107648.0 * n + 8192.0


def cpu_baseline(n=200, seconds=12.0, train=True):
    """Oracle (CPU 'port'): SpinSystem.step restatement + torch-CPU MPNN forward, B=1
    epsilon-greedy act (dqn.py:282 path); with train=True also one oracle train_step of
    minibatch 64 every 32 env-steps (train_eco.py:136-137), i.e. the reference's learn loop."""
    sys.path.insert(0, REPO)
    from oracle import spinsystem_oracle as so
    from oracle import mpnn_oracle as mo
    from oracle import graphs as og
    rng = np.random.default_rng(0)
    w = mo.init_weights(torch.Generator().manual_seed(0), std=0.01)
    adam = {"step": 0, "m": {}, "v": {}}
    buf = []
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        J = og.er_graph(n, 0.15, rng)
        env = so.SpinSystemOracle(J, 2 * n, basin_reward=1. / n)
        obs = env.reset(rng=np.random.RandomState(int(rng.integers(1 << 31))))
        done = False
        while not done and time.perf_counter() - t0 < seconds:
            with torch.no_grad():
                q = mo.forward(w, torch.from_numpy(obs).float())
            a = int(q.argmax()) if rng.random() >= 0.05 else int(rng.integers(n))
            obs2, r, done, _ = env.step(a)
            steps += 1
            if train:
                buf.append((obs, a, r, obs2, float(done)))
                buf = buf[-2000:]
                if steps % 32 == 0 and len(buf) >= 64:
                    idx = rng.choice(len(buf), 64, replace=False)
                    tr = [buf[i] for i in idx]
                    w, _ = mo.train_step(w, adam, torch.from_numpy(np.array([t[0] for t in tr])).float(),
                                         torch.tensor([[t[1]] for t in tr]), torch.tensor([[t[2]] for t in tr],
                                                                                         dtype=torch.float32),
                                         torch.from_numpy(np.array([t[3] for t in tr])).float(),
                                         torch.tensor([[t[4]] for t in tr], dtype=torch.float32))
            obs = obs2
    dt = time.perf_counter() - t0
    what = "learn loop: act + env.step + train_step(64) every 32 steps" if train else "act + env.step"
    return dict(value=steps / dt, unit="env-steps/s", cores=torch.get_num_threads(), kind="port",
                sample=f"{steps} ER-200 env-steps in {dt:.1f}s of the oracle {what} "
                       f"(numpy SpinSystem restatement + torch-CPU MPNN, B=1)")


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            return next(ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name"))
    except (OSError, StopIteration):
        import platform
        return platform.processor() or platform.machine()


def cgroup_cpu_quota():
    """CPUs granted by this process's cgroup CPU quota (cgroup v2 cpu.max 'quota period', or v1
    cfs_quota_us / cfs_period_us), rounded up; None when unlimited or unreadable."""
    import math
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max" and int(p) > 0:
            return max(1, math.ceil(int(q) / int(p)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return max(1, math.ceil(q / p)) if q > 0 and p > 0 else None
    except (OSError, ValueError):
        return None


def cpu_refcost_baseline(n=200, seconds=10.0, gpus_on_node=1):
    """SURVEY.md 8d CPU side-by-side: the reference-cost restatement of env.step (oracle/refcost.py:
    the reference's per-step op mix -- 4 dense J@s matvecs, 2 dense np.outer cuts, the observables
    loop, the list-of-sets visited buffer and the vstack observation; bit-exact with the reference
    and calibrated against it in the build container, oracle/refcost_calibration.json) with a
    uniform random policy (configs[0]'s plumbing loop) on fresh ER(n, 0.15) graphs, one single-
    threaded process per CPU of this process's affinity set (every host core it may use), all at
    once.  value = the sum of the per-process rates (each timed over its own env.step loops in wall
    time, so an oversubscribed share is not overstated); per_gpu_share = value / the node's GPUs (the
    host cores split evenly over them).  ECO_CPU_BASELINE_PROCS caps the process count (testing)."""
    import subprocess
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    # the CPUs this job may actually use: its affinity set, capped by its cgroup CPU quota (on the GPU box the
    # affinity set names all 256 host CPUs while the quota grants 16: 256 processes on 16 CPUs measured 0.44x
    # the rate of 16 processes)
    share = max(1, min(affinity, quota)) if quota else affinity
    cap = int(os.environ.get("ECO_CPU_BASELINE_PROCS", "0")) or share
    procs = max(1, min(share, cap))
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, "-m", "oracle.refcost", str(n), str(seconds), str(100 + i)], cwd=REPO,
                           env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
          for i in range(procs)]
    rates, steps = [], 0
    for p in ps:
        out, _ = p.communicate(timeout=seconds * 6 + 120)
        st, busy = out.split()
        steps += int(st)
        rates.append(int(st) / float(busy))
    cal = None
    try:
        with open(os.path.join(REPO, "oracle", "refcost_calibration.json")) as fh:
            cal = {c["workload"]: round(c["ratio"], 3) for c in json.load(fh)["cases"]}
    except (OSError, ValueError, KeyError):
        pass
    return dict(value=float(sum(rates)), unit="env-steps/s", cores=procs, kind="port",
                nproc=os.cpu_count(), cpu_share=share, cpu_affinity=affinity, cgroup_cpu_quota=quota,
                cpu_model=_cpu_model(),
                per_core=float(np.mean(rates)), gpus_on_node=gpus_on_node,
                per_gpu_share=float(sum(rates)) / max(1, gpus_on_node),
                sample=f"{steps} ER-{n} env.step calls (random actions, T=2N episodes) in {procs} single-threaded "
                       f"processes x {seconds:.0f}s of oracle/refcost.py, the reference-cost restatement of "
                       "spinsystem.py:355-574",
                calibration_ratio_vs_reference=cal)


PMC_SUMMARY = os.path.join(REPO, "profiles", "r06", "final", "train", "pmc_hbm.json")
PMC_SQ = os.path.join(REPO, "profiles", "r06", "final", "train", "pmc_sq_dense.json")
PMC_PAIRED = True  # the committed train PMC pass ran the paired s' forward (eco_mpnn_forward_pair)
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16 / bf16 MFMA peak (~2.5 PF)


def forward_kernel_name(n, graph, n_graphs=None):
    """The forward kernel the dispatcher runs for 8-feature rows and +-1 / unit weights (eco_mpnn_forward):
    blocks of <= 224 rows -> the fp16x2 dense kernels; one graph of 224 < N <= 512 -> the fp16x2 DL kernels;
    N > 512 on one shared graph -> the shared-graph kernels (fp16x2 Linears).  All issue f16/bf16 MFMAs."""
    if n <= 224:
        return ("mpnn_forward_dense2_kernel" if int(os.environ.get("ECO_BENCH_KERNEL_PATHS", "0") or 0) & 16
                else "mpnn_forward_dense3_kernel")
    if n <= 512:
        return "mpnn_forward_dl_kernel"
    return "shared_agg_kernel+shared_lin_kernel" if n_graphs == 1 else "mpnn_forward_large_kernel"


def mfma_roofline(achieved_tflops, kernel):
    """roofline fields for an MPNN kernel: frac against the dense peak of the MFMA dtype it issues (f16 for
    the fp16x2 dense / DL kernels and the shared-graph Linears, 2.5 PF; f32 157.3 TF is not used for the
    per-episode large kernel either: it runs bf16x3 fragments, the bf16 peak being the same 2.5 PF)."""
    peak = F16_MFMA_PEAK_TFLOPS
    return {"bound": "mfma", "kernel": kernel, "achieved": achieved_tflops, "peak": peak, "unit": "TFLOP/s",
            "frac": achieved_tflops / peak, "peak_dtype": "f16/bf16 dense MFMA (the issued dtype)",
            "frac_vs_f32_mfma_peak": achieved_tflops / FP32_MFMA_PEAK_TFLOPS}
# kernel names of the dense path, newest first (the PMC summaries of earlier rounds carry the older ones)
FWD_NAMES = ("mpnn_forward_dense3_kernel", "mpnn_forward_dense2_kernel", "mpnn_forward_dense_kernel")
BWD_NAMES = ("mpnn_backward_dense3_kernel", "mpnn_backward_dense2_kernel", "mpnn_backward_dense_kernel")
WGRAD_NAMES = ("wgrad_fh_kernel", "wgrad_bf3_kernel", "wgrad_kernel")


def _first(d, names):
    return next(d[k] for k in names if k in d)
PMC_GSET = os.path.join(REPO, "profiles", "r04", "final", "gset_pmc", "pmc_hbm.json")


def pmc_mfma(dom, B, M, n, graph, flops_per_graph):
    """MFMA evidence of the dominant kernel from the committed SQ PMC pass (PMC_SQ, ER-200 M=2048): MFMA-busy fraction (launch mix of the train loop: inference forwards
    of act and of s', training forwards with saved activations) and the ratio of ISSUED f16 MFMA FLOPs
    (fp16x2 splits, dense N^2 aggregations) to the algorithmic FLOPs, so the issued rate can be priced
    against the f16 peak beside the f32-algorithmic fraction."""
    if (graph, n, M) != ("ER", 200, 2048) or dom != "mpnn_forward_kernel":
        return None
    try:
        with open(PMC_SQ) as f:
            k = json.load(f)["kernels"]
        inf = _first(k, [n + t for n in FWD_NAMES for t in ("<false, 1, true>", "<false, 1>", "<false>")])
        trn = _first(k, [n + t for n in FWD_NAMES for t in ("<true, 1, true>", "<true, 1>", "<true>")])
    except (OSError, ValueError, KeyError):
        return None
    n_inf, n_trn = 1 + 2 * (B * 2 // M), B * 2 // M  # act + online/target(s') per grad step (their work, paired
    # or not); online(s) saves
    busy = (n_inf * inf["mfma_busy"] + n_trn * trn["mfma_busy"]) / (n_inf + n_trn)
    ratio = inf.get("issued_mfma_flop", inf.get("issued_bf16_flop")) / (flops_per_graph * M)
    return {"mfma_busy": busy, "issued_per_algorithmic_flop": ratio, "source": os.path.relpath(PMC_SQ, REPO)}


def pmc_gset_traffic():
    """HBM bytes of one configs[4] forward (shared-graph prep + edge + 3 layer launches) from the committed
    PMC summary (2 x FETCH_SIZE + WRITE_SIZE, KB = 1024 B), or None."""
    try:
        with open(PMC_GSET) as f:
            k = json.load(f)["kernels"]
        return sum(v["hbm_bytes_per_launch"] * v["launches_per_forward"] for name, v in k.items()
                   if name.startswith("shared_"))
    except (OSError, ValueError, KeyError):
        return None


def pmc_traffic(dom, B, M, n, graph="ER"):
    """HBM bytes per launch of the dominant kernel, from the committed rocprofv3 PMC pass of this
    workload (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md gfx950 correction), averaged over the
    launch mix the live timing averages over; None when no matching measurement is committed."""
    if (graph, n, B, M) != ("ER", 200, 8192, 2048):  # the profiled configuration only
        return None
    try:
        with open(PMC_SUMMARY) as f:
            k = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    gpb = 1 if n >= 208 else 208 // n
    try:
        if dom == "mpnn_forward_kernel":
            fw = _first(k, FWD_NAMES)
            act, tr = fw[str((B + gpb - 1) // gpb)], fw[str((M + gpb - 1) // gpb)]
            # per vector step: one act forward over B graphs, and per gradient step the s' pair (one launch when
            # paired) + the training forward; tr averages the M-graph launches of the profiled run
            k = B * 2 // M
            per_k = 2 if PMC_PAIRED else 3
            return (act["hbm_bytes_per_launch"] + per_k * k * tr["hbm_bytes_per_launch"]) / (1 + per_k * k)
        bw = _first(k, BWD_NAMES)[str((M + gpb - 1) // gpb)]
        wg = next(iter(_first(k, WGRAD_NAMES).values()))
        return bw["hbm_bytes_per_launch"] + wg["hbm_bytes_per_launch"]
    except (KeyError, StopIteration):
        return None


def envstep_rate(dev, B, n, steps=200, warmup=5, seed=1234, store=None):
    """The batched MaxCut env step kernel alone (spinsystem.py:355-559, ER(n, 0.15) +-1 graphs -- or the
    given store's graphs -- one per episode, uniform random actions drawn beforehand): env-steps/s over
    `steps` launches replayed from a HIP graph and timed with HIP events, and the mean launch time (ms)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget
    if store is None:
        store = GraphStore.random("ER", B, n, 0.15, seed=seed, device=dev)
    T = 2 * n
    env = VecSpinSystem(store, B, T, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        norm_rewards=True, basin_reward=1. / n)
    steps = min(steps, T - warmup)
    g = torch.Generator(device=dev).manual_seed(7)
    acts = torch.randint(0, n, (warmup + steps, B), generator=g, device=dev, dtype=torch.int32)
    env.reset(graph_ids=np.arange(B), seed=seed)
    for i in range(warmup):
        env.step(acts[i])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the launches are replayed from a HIP graph: a Python loop of ctypes launches (~20-30 us of host time each)
    # cannot keep a ~20 us kernel busy, and the events would time the host.  Graph replay issues them back to back
    # (one kernel boundary each, ~1.5 us), which is what the kernel's rate is.
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):
        with torch.cuda.graph(graph, stream=cap):
            for i in range(steps):
                env.step(acts[warmup + i])
    torch.cuda.current_stream(dev).wait_stream(cap)
    torch.cuda.synchronize()
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize()
    env.check_errors()
    ms = e0.elapsed_time(e1) / steps
    return B / (ms * 1e-3), ms


def make_test_env(agent, dev, test_graphs=50, graph="ER", gparam=0.15):
    """The reference's ER-200 test setting (train_eco.py:59-69, 166-169): a VecSpinSystem of 64 slots over
    `test_graphs` seeded test graphs with the training env's arguments."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    return VecSpinSystem(GraphStore.random(graph, test_graphs, agent.N, gparam, seed=4321, device=dev), 64,
                         agent.env.max_steps, **agent.env.env_args)


def untimed_costs(agent, B, world, dev, test, test_frequency=50000):
    """What the timed vector steps never contain (T = 2N steps per episode, 20 timed steps): the full reset of
    all B episodes at an episode boundary (the agent's own path: fresh graph slots regenerated on the device,
    fresh spins, compact-replay snapshot; dqn.py:306-327), and one evaluate_agent() at the reference's ER-200
    test settings (`test`: train_eco.py:59-69,166-169,368-377: 50 test graphs, BEST metric, every 50k env-steps).
    Both measured here with HIP-synchronised wall time and amortised per vector step.  Evaluations: learn() runs
    ONE evaluation per test_frequency crossing for the whole job (round-robin over the ranks) and at most one
    per vector step, so a rank runs min(1, B x world / test_frequency) / world evaluations per vector step."""
    from eco_hip.agents.dqn.utils import TestMetric
    T = agent.env.max_steps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent._reset_env(agent._take_graph_slots(None), agent.seed + 99)
    torch.cuda.synchronize()
    reset_ms = (time.perf_counter() - t0) * 1e3
    saved = (agent.test_envs, agent.test_episodes, agent.test_metric)
    agent.test_envs, agent.test_episodes, agent.test_metric = test, test.graphs.n_graphs, TestMetric.BEST
    agent.eval_graphs = False
    agent.evaluate_agent()  # first call: allocations
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent.evaluate_agent()
    torch.cuda.synchronize()
    eval_eager_ms = (time.perf_counter() - t0) * 1e3
    agent.eval_graphs = True
    agent.evaluate_agent()  # eager once more, then the rollout is captured into a HIP graph
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent.evaluate_agent()
    torch.cuda.synchronize()
    eval_ms = (time.perf_counter() - t0) * 1e3
    # learn()'s default: the evaluation overlapped with training (DQN._evaluate_overlapped, side stream on a
    # snapshot of the weights, the rollout replayed from its HIP graph).  Its cost = the wall time it adds to the
    # vector steps it runs beside.
    k = 8
    for _ in range(2):  # allocations, capture
        agent._eval_one_fill_finish(agent._evaluate_overlapped(0))
    ts = []
    for ov in (False, True, False, True):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = agent._evaluate_overlapped(0) if ov else None
        for _ in range(k):
            agent.iteration()
        if p is not None:
            agent._eval_one_fill_finish(p)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ov_ms = max(0.0, (ts[1] + ts[3] - ts[0] - ts[2]) / 2)
    agent.test_envs, agent.test_episodes, agent.test_metric = saved
    per_vec_evals = min(1.0, B * world / test_frequency) / world
    per_vec_sync = reset_ms / T + eval_ms * per_vec_evals
    per_vec = reset_ms / T + ov_ms * per_vec_evals
    return {"episode_reset_ms": reset_ms, "reset_every_vector_steps": T,
            "reset_path": "DQN._take_graph_slots + DQN._reset_env (graph slots regenerated when free)",
            "evaluate_agent_ms": eval_ms, "evaluate_agent_eager_launches_ms": eval_eager_ms,
            "evaluate_overlapped_ms": ov_ms,
            "evaluate_overlapped_note": f"wall time one overlapped evaluation adds to {k} vector steps of training "
                                        "(learn()'s default; evaluate_agent_ms is the synchronous call replaying the "
                                        "rollout's HIP graph, evaluate_agent_eager_launches_ms the same call with "
                                        "~800 host launches)",
            "evaluate_every_env_steps": test_frequency,
            "evaluate_setting": f"{test.graphs.n_graphs} test graphs, BEST metric, {T} greedy steps each",
            "evaluations_per_vector_step_per_rank": per_vec_evals,
            "amortised_ms_per_vector_step": per_vec, "amortised_ms_per_vector_step_sync_eval": per_vec_sync,
            "amortised_formula": "reset_ms / T + evaluate_overlapped_ms * min(1, B * world / test_frequency) / world: "
                                 "one evaluation per crossing for the whole job, at most one per vector step, dealt "
                                 "round-robin to the ranks (DQN.learn)",
            "note": "not in the timed region: amortised, these would add this many ms to ms_per_step; the learn_loop "
                    "figure measures them end to end"}


def learn_loop(agent, B, world, dev, test, vector_steps=60, test_frequency=50000, save_network_frequency=400000):
    """The reference's whole training loop on the record: DQN.learn() (dqn.py:256-395) end to end, with the
    evaluation every test_frequency env-steps on `test` (50 ER-200 graphs, BEST metric, overlapped, `_best`
    saved; train_eco.py:368-377 cadence) and the periodic checkpoints, over `vector_steps` vector steps of all
    ranks' B episodes.  Returns the job's env-steps/s (max wall time over ranks) and what ran."""
    import tempfile
    from eco_hip.agents.dqn.utils import TestMetric
    from eco_hip.parallel import max_over_ranks
    saved = (agent.test_envs, agent.test_episodes, agent.test_metric, agent.test_frequency, agent.evaluate,
             agent.save_network_frequency, agent.network_save_path, agent.test_save_path)
    timesteps = vector_steps * B * world
    with tempfile.TemporaryDirectory() as d:
        agent.test_envs, agent.test_episodes, agent.test_metric = test, test.graphs.n_graphs, TestMetric.BEST
        agent.test_frequency, agent.evaluate = test_frequency, True
        agent.save_network_frequency = save_network_frequency
        agent.network_save_path, agent.test_save_path = os.path.join(d, "network.pth"), None
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        regen0, reuse0 = getattr(agent, "graphs_regenerated", 0), getattr(agent, "graphs_reused", 0)
        t0 = time.perf_counter()
        agent.learn(timesteps)
        torch.cuda.synchronize()
        dt_rank = time.perf_counter() - t0
        n_eval = len(agent.test_scores)
    (agent.test_envs, agent.test_episodes, agent.test_metric, agent.test_frequency, agent.evaluate,
     agent.save_network_frequency, agent.network_save_path, agent.test_save_path) = saved
    dt = max_over_ranks(dt_rank, device=dev)
    return {"value": agent._timestep / dt, "unit": "env-steps/s", "env_steps": agent._timestep, "seconds": dt,
            "vector_steps": vector_steps, "evaluations": n_eval, "test_frequency": test_frequency,
            "graphs_regenerated": getattr(agent, "graphs_regenerated", 0) - regen0,
            "graphs_reused": getattr(agent, "graphs_reused", 0) - reuse0,
            "save_network_frequency": save_network_frequency,
            "what": "DQN.learn() end to end: start() (every episode reset on fresh graphs), act + env step + replay "
                    "add + gradient steps per vector step, one evaluation per test_frequency crossing (50 test "
                    "graphs, BEST, overlapped on a side stream, `_best` saved), periodic checkpoints, final "
                    "collection of the scores and losses"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(nproc):
    """`bench.py --gpus N` without a torch.distributed.run environment: start N fresh child
    processes of this script, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT set (one process per GPU, episodes sharded).  The parent never
    touches the GPU (no torch.cuda call before or after the children start; nothing is exec'd);
    children inherit stdout, and only rank 0 prints the JSON line.  A failing rank stops the
    others; the parent exits with the first non-zero code."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:  # one rank failed: the collective would hang the rest
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        time.sleep(0.05)
    return rc


def dry_run_bench(args, world, rank, local):
    """--dry-run: the launcher / rendezvous / timing harness on CPU over gloo (no GPU).  A step is a
    small numpy reduction; rank 0 reports the world size the process group observed and every rank's
    local rank, so a CPU test can check that N distinct ranks ran and exactly one line was printed."""
    import torch.distributed as tdist
    if world > 1:
        tdist.init_process_group("gloo")
    if os.environ.get("ECO_BENCH_DRY_FAIL_RANK") == str(rank):
        raise SystemExit(3)  # failure-propagation check of the launcher
    x = np.random.default_rng(rank).random(1 << 16)
    for _ in range(args.warmup):
        float(x.sum())
    if world > 1:
        tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        float(x.sum())
    if world > 1:
        tdist.barrier()
    dt = time.perf_counter() - t0
    per_rank = _gather_floats([dt, float(local)], world)
    if rank == 0:
        print(json.dumps({"metric": "dry-run (launcher check)", "value": 0.0, "unit": "steps/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": max(p[0] for p in per_rank) / max(args.steps, 1) * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                          "data": "synthetic", "config": {"workload": "dry-run"},
                          "process_group": {"backend": "gloo" if world > 1 else None, "world_size": world,
                                            "local_ranks": [int(p[1]) for p in per_rank]}}))
    if world > 1:
        tdist.destroy_process_group()


def _gather_floats(vals, world, device=None):
    """All-gather a short list of floats from every rank (rank-ordered list of lists)."""
    if world == 1:
        return [list(vals)]
    import torch.distributed as tdist
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    tdist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def process_group_info(world, per_rank_s, steps, local, device):
    """What the collective backend saw: its name and world size, and every rank's own timed-region
    ms per step (the headline ms_per_step is the max over ranks)."""
    import torch.distributed as tdist
    ranks = _gather_floats([per_rank_s / max(steps, 1) * 1e3, float(local)], world, device)
    ms = [r[0] for r in ranks]
    return {"backend": tdist.get_backend() if world > 1 else None,
            "rccl_world_size": tdist.get_world_size() if world > 1 else 1,
            "local_ranks": [int(r[1]) for r in ranks],
            "ms_per_step_min": min(ms), "ms_per_step_max": max(ms)}


TARGET_SYNC_GRAD_STEPS = 16
REPLAY_EPISODES = 1.0     # replay ring in episode batches of B x T transitions
STAGGER_EPISODES = False  # DQN.stagger_episodes: episodes spread over the T phases of an episode


def build_train_agent(dev, B, n, graph="ER", gparam=0.15, minibatch=2048, seed=1234, replay_episodes=None,
                      n_graphs=None, regenerate=True, spare_batches=0):
    """The benched configs[2] / configs[3] agent: B episodes on a pool of B seeded graphs (one per episode),
    experiments/train_eco.py:114-169 hyper-parameters (N=200: :368-377) batched, with the large-batch recipe of
    tests/test_training_quality_gpu.py (lr 1e-4 x sqrt(M / 64); target sync every TARGET_SYNC_GRAD_STEPS gradient
    steps) and a replay ring of `replay_episodes` x B x T transitions: the B lockstep
    episodes push B per vector step, so a ring of one episode's worth holds every time step of the episodes
    (the reference's 15,000 transitions span ~19 whole ER-200 episodes); B x 16 (round 3) held only the last 16
    steps and measured 0.935 of the pretrained network's single-attempt cut against 0.974-0.991 with B x T
    (profiles/r04/quality/; round 5: profiles/r05/quality/).  tests/test_training_quality_er200_gpu.py trains this
    exact agent.
    regenerate (default): a fresh ER / BA graph for every episode, as the reference's env.reset() draws one
    (src/agents/dqn/dqn.py:306-327 -> src/envs/spinsystem.py:191-196 -> src/envs/utils.py:192-236): the store holds
    graph_slots_needed(B, T, ring) slots (two batches of B at one episode's ring), generated on the device, and
    DQN(regenerate_graphs=) regenerates a batch's slots at each reset once no stored transition references them.
    regenerate=False: a fixed pool of n_graphs (default B) seeded graphs that episodes draw from at each reset.
    spare_batches: extra batches of B slots for resets outside episode boundaries (the bench's untimed reset and
    learn_loop's start() follow the timed steps mid-episode, while the replay still references the first batch),
    so that those resets, too, draw freshly generated graphs.
    Returns (agent, store, env, lr)."""
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.agents.dqn.dqn import DQN, graph_slots_needed
    T = 2 * n
    cap = int(B * T * (REPLAY_EPISODES if replay_episodes is None else replay_episodes))
    if regenerate:
        store = GraphStore.generated(graph, graph_slots_needed(B, T, cap) + spare_batches * B, n, gparam, seed=seed,
                                     device=dev)
    else:
        store = GraphStore.random(graph, n_graphs or B, n, gparam, seed=seed, device=dev)
    env = VecSpinSystem(store, B, T, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    lr = 1e-4 * (minibatch / 64.0) ** 0.5
    agent = DQN(env, lambda: MPNN(device=dev), init_weight_std=0.01, double_dqn=True, clip_Q_targets=False,
                replay_start_size=3000, replay_buffer_size=cap, gamma=0.95, update_target_frequency=4000,
                update_learning_rate=False, initial_learning_rate=lr, peak_learning_rate=lr,
                final_learning_rate=lr, update_frequency=32, minibatch_size=64, train_minibatch=minibatch,
                initial_exploration_rate=1, final_exploration_rate=0.05, final_exploration_step=800000,
                adam_epsilon=1e-8, seed=seed, target_sync="grad_steps",
                regenerate_graphs=(graph, gparam) if regenerate else None)
    # target sync every TARGET_SYNC_GRAD_STEPS gradient steps (16,384 env-steps) instead of the reference's
    # update_target_frequency / update_frequency = 125: round-5 sweeps (profiles/r05/quality/) measured ER-200
    # single-attempt 0.989 (nine seeds) against 0.983 at 125, BA-200 1.010 against 1.012; one copy of the parameter
    # vector, no throughput cost
    agent.target_sync_grad_steps = TARGET_SYNC_GRAD_STEPS
    agent.stagger_episodes = STAGGER_EPISODES
    return agent, store, env, lr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node; N > 1 without a torch.distributed.run environment starts N ranks")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU-only launcher/rendezvous check over gloo (no GPU work)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--minibatch", type=int, default=2048, help="M graphs per gradient step")
    ap.add_argument("--graph", default="ER", choices=["ER", "BA"],
                    help="training graphs: ER(n, p=--param) (configs[2]) or BA(n, m=--param) (configs[3])")
    ap.add_argument("--param", type=float, default=None, help="ER p (default 0.15) / BA m (default 4)")
    ap.add_argument("--workload", default="train", choices=["train", "rollout", "gset", "er20", "envstep"],
                    help="train = configs[2] (default); rollout = its act + env step half; "
                         "gset = configs[4] per GPU: 1024 episodes of greedy best-cut search on one "
                         "G22-like ER(2000, p=0.01) unit-weight graph; er20 = configs[1]: 4096 ER-20 "
                         "episodes, MPNN forward + greedy act + env step; envstep = the env step kernel "
                         "alone (SURVEY.md 8d sub-bench) for --target")
    ap.add_argument("--target", default="CUT",
                    choices=["CUT", "MIN_COVER", "MIN_CUT", "MAX_IND_SET", "MAX_CLIQUE", "MIN_DOM_SET"],
                    help="envstep: OptimisationTarget (set problems use MAIN_OBSERVABLES and unit weights)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run_bench(args, world, rank, local)
    dist = world > 1
    # rehearsal knobs for a one-GPU box (never set by the driver): every rank on GPU 0, gloo collectives
    gpu = 0 if os.environ.get("ECO_BENCH_SHARED_DEVICE") == "1" else local
    if dist:
        torch.cuda.set_device(gpu)
        torch.distributed.init_process_group(os.environ.get("ECO_BENCH_BACKEND", "nccl"))
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    if os.environ.get("ECO_BENCH_KERNEL_PATHS"):  # A/B knob (never set by the driver): eco_set_kernel_paths bits
        from eco_hip import _lib
        _lib.lib.eco_set_kernel_paths(int(os.environ["ECO_BENCH_KERNEL_PATHS"]))

    if args.workload in ("gset", "er20"):
        return inference_bench(args, world, rank, local, dev, dist)
    if args.workload == "envstep":
        return envstep_bench(args, world, rank, local, dev, dist)

    B, n = args.envs, args.n
    T = 2 * n
    seed = 1234 + rank
    gparam = args.param if args.param is not None else (0.15 if args.graph == "ER" else 4)
    agent, store, env, lr = build_train_agent(dev, B, n, args.graph, gparam, args.minibatch, seed,
                                              spare_batches=1 if args.workload == "train" else 0)
    nnz = np.diff(store.row_ptr.cpu().numpy(), axis=1).sum(axis=1)
    gflops = np.array([mpnn_flops(z, n) for z in nnz])
    agent.start()
    train = args.workload == "train"

    def one_step():
        if train:
            agent.iteration()
        else:
            agent.vector_step(True)

    # warmup: fills the replay past replay_start_size, so every timed step trains
    for _ in range(max(args.warmup, 1)):
        one_step()
    torch.cuda.synchronize()
    timers = []
    agent.network.timer = timers
    agent.target_network.timer = timers
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt_rank = time.perf_counter() - t0
    agent.network.timer = None
    agent.target_network.timer = None
    from eco_hip.parallel import max_over_ranks
    dt = max_over_ranks(dt_rank, device=dev)
    pg = process_group_info(world, dt_rank, args.steps, local, dev)

    fixed = loop = None
    if train:
        test = make_test_env(agent, dev, graph=args.graph, gparam=gparam)
        fixed = untimed_costs(agent, B, world, dev, test)
        loop = learn_loop(agent, B, world, dev, test)

    # per-kernel roofline from the live events: forward launches vs backward launches
    kern = {"mpnn_forward_kernel": [0.0, 0.0, 0], "mpnn_backward(+wgrad)": [0.0, 0.0, 0]}
    mean_gf = float(gflops.mean())  # sampled minibatches draw from this pool: use its mean per graph
    for e0, e1, b, _ in timers:
        ms = e0.elapsed_time(e1)
        fl = mean_gf * abs(b)
        key = "mpnn_forward_kernel" if b > 0 else "mpnn_backward(+wgrad)"
        kern[key][0] += ms
        kern[key][1] += fl * (1 if b > 0 else 2)
        kern[key][2] += 1
    dom = max(kern, key=lambda k: kern[k][0])
    ms, fl, cnt = kern[dom]
    avg_ms = ms / max(cnt, 1)
    achieved = fl / max(ms, 1e-9) / 1e9  # TFLOP/s
    value = B * args.steps * world / dt
    if rank == 0:
        wl = (f"{args.graph}_{n}spin" + " x%d envs/GPU: full ECO-DQN train loop per vector step (act + env step + replay add "
              "+ %d grad steps of M=%d: sample, double-DQN TD, MPNN fwd/bwd, Adam)"
              % (B, agent._k_per_vec, args.minibatch)) if train else \
             (f"{args.graph}_{n}spin" + " x%d envs/GPU: rollout only (MPNN fwd + eps-greedy act + env step + replay add)" % B)
        out = {
            "metric": f"env-steps/sec (batched episodes) on {args.graph}-{n} MaxCut",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32-accurate MPNN on f16 MFMA (fp16x2: every operand a power-of-two-scaled pair of fp16 "
                     "pieces, 22 significand bits, three products, f32 accumulate; aggregations and Linears alike; "
                     "f32 MFMA on the CSR fallback) / f64+int (env)",
            "data": f"synthetic: seeded {args.graph}({n}, {gparam}) +-1 graphs, one per episode; random-init MPNN "
                    "(std 0.01)",
            "config": {"workload": wl, "n_spins": n, "envs_per_gpu": B, "max_steps": T,
                       "train_minibatch": args.minibatch, "grad_steps_per_vector_step": agent._k_per_vec if train else 0,
                       "replay_ratio": 2.0, "lr": lr, "target_sync": "every %d gradient steps"
                       % agent.target_sync_grad_steps,
                       "parallelism": f"episodes sharded, dp{world} grad all-reduce"},
            "roofline": dict(mfma_roofline(achieved, forward_kernel_name(n, args.graph)
                                           if dom == "mpnn_forward_kernel" else dom),
                         traffic=pmc_traffic(dom, B, args.minibatch, n, args.graph) if train else None,
                         traffic_unit="HBM bytes per launch (PMC, %s)" % os.path.relpath(PMC_SUMMARY, REPO),
                         avg_launch_ms=avg_ms, launches=cnt, flops_per_launch=fl / max(cnt, 1)),
            "kernels_ms_per_step": {k: v[0] / args.steps for k, v in kern.items()},
            "process_group": pg,
        }
        # the env step kernel alone on this bench's graphs: SURVEY.md 8d's HBM roofline of the env step
        es_rate, es_ms = envstep_rate(dev, B, n, store=store)
        out["env_step_roofline"] = envstep_roofline(es_rate, es_ms, n, B)
        out["untimed_per_episode_costs"] = fixed
        if loop is not None:
            loop["ratio_to_headline"] = loop["value"] / value
            out["learn_loop"] = loop
        mf = pmc_mfma(dom, B, args.minibatch, n, args.graph, mean_gf) if train else None
        if mf:
            issued = achieved * mf["issued_per_algorithmic_flop"]
            out["roofline"].update(mfma_busy=mf["mfma_busy"], issued_f16_tflops=issued,
                                   f16_peak=F16_MFMA_PEAK_TFLOPS, f16_frac=issued / F16_MFMA_PEAK_TFLOPS,
                                   mfma_source=mf["source"])
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline_learn_loop"] = cpu_baseline(n, train=train)
            if args.graph == "ER":
                out["cpu_baseline"] = cpu_refcost_baseline(n, gpus_on_node=torch.cuda.device_count())
                cb = out["cpu_baseline"]
                # like for like: env step vs env step (rollout, random policy) and learn loop vs learn loop
                out["vs_cpu_baseline"] = {
                    "env_step": {"gpu_env_step_kernel": es_rate, "gpu_kernel_ms": es_ms,
                                 "cpu_all_cores": cb["value"], "ratio": es_rate / cb["value"],
                                 "ratio_vs_per_gpu_share": es_rate / cb["per_gpu_share"]},
                    "learn_loop": {"gpu_train_loop": value, "cpu_learn_loop": out["cpu_baseline_learn_loop"]["value"],
                                   "ratio": value / out["cpu_baseline_learn_loop"]["value"]},
                    "note": "env_step: the batched env step kernel alone (ER-%d x %d, random actions, HIP events) "
                            "over the reference-cost env.step on every host core; learn_loop: this line's value "
                            "over the oracle learn loop (act + env.step + train_step(64)/32 steps) on the host" % (n, B)}
        print(json.dumps(out))
    if dist:
        torch.distributed.destroy_process_group()


def inference_bench(args, world, rank, local, dev, dist):
    """configs[4] (gset) / configs[1] (er20): batched greedy rollouts, one vector step = MPNN forward +
    fused greedy argmax (dqn.py:490-512 via experiments/utils.py:154-187) + env step for every episode."""
    from eco_hip import _lib
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    from eco_hip.networks.mpnn import MPNN
    from eco_hip.parallel import max_over_ranks, best_cut_over_ranks
    seed = 1234 + rank
    if args.workload == "gset":
        # G22 is absent from the reference (.MISSING_LARGE_BLOBS:1): unweighted ER(2000, 0.01) stand-in
        n, B, kind, p, weights, ngraphs = 2000, 1024, "ER", 0.01, "uniform", 1
        T = 2 * n  # step_factor 2 (experiments/test_eco.py:84)
    else:
        n, B, kind, p, weights, ngraphs = 20, 4096, "ER", 0.15, "discrete", 4096
        T = 2 * n
    store = GraphStore.random(kind, ngraphs, n, p, seed=1234, weights=weights, device=dev)
    env = VecSpinSystem(store, B, T, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1. / n)
    net = MPNN(device=dev)
    net.init_normal_(0.1, generator=torch.Generator().manual_seed(0))
    gids_np = np.arange(B) % ngraphs
    env.reset(graph_ids=gids_np, seed=seed)
    gids = env.graph_ids
    gids_dev = gids.clone()
    acts = torch.empty(B, dtype=torch.int32, device=dev)
    greedy = _lib.ActConfig(0.0, 1, 0.0, 0, 0)
    timers = []
    # configs[1]: an ER-20 episode is T = 40 steps of ~100 us of GPU work each, paced by the host's two launches per
    # step; each whole episode is replayed from a HIP graph captured once (the same launches, as DQN's evaluation
    # rollouts).  The forward's roofline is then timed with HIP events on one eager episode after the timed region
    # (events cannot sit inside the graph).  configs[4] (T = 4000, ~2.6 ms per step) stays eager, timed live.
    graphed = args.workload == "er20"
    net.timer = None if graphed else timers

    # the episodes' graphs never change: the call's max degree (norm.max(), dqn.py:546-547) is computed by the
    # first forward and reused from the workspace after it (ECO_NORM_PER_CALL_REUSE: same values, one 1-workgroup
    # launch fewer per step)
    scope = [_lib.ECO_NORM_PER_CALL]
    t_ep = [0]  # steps of the current episodes (all B episodes run in lockstep)
    ep_seed = [seed]

    def one_step():
        if t_ep[0] == T:  # every episode is done: a new one on the same graphs (experiments/utils.py:126-147)
            ep_seed[0] += 1
            env.reset(graph_ids=gids_dev, seed=ep_seed[0])
            t_ep[0] = 0
        net.forward_graphs(env.obs_x, store, gids, norm_scope=scope[0], act=greedy, actions_out=acts)
        env.step(acts)
        scope[0] = _lib.ECO_NORM_PER_CALL_REUSE
        t_ep[0] += 1

    episode_graph = [None]

    def run_steps(k):
        """k env-steps of every episode; whole episodes from the captured graph (graphed mode)."""
        while k > 0:
            if graphed and episode_graph[0] is not None and k >= T and t_ep[0] in (0, T):
                if t_ep[0] == T:
                    ep_seed[0] += 1
                    env.reset(graph_ids=gids_dev, seed=ep_seed[0])
                episode_graph[0].replay()
                t_ep[0] = T
                k -= T
            else:
                one_step()
                k -= 1

    for _ in range(max(args.warmup, 1)):
        one_step()
    if graphed:
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):  # captures T forward + step launches; executes nothing
            for _ in range(T):
                net.forward_graphs(env.obs_x, store, gids, norm_scope=_lib.ECO_NORM_PER_CALL_REUSE, act=greedy,
                                   actions_out=acts)
                env.step(acts)
        episode_graph[0] = g
        t_ep[0] = T  # the timed region starts on fresh episodes
    torch.cuda.synchronize()
    timers.clear()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt_rank = time.perf_counter() - t0
    dt = max_over_ranks(dt_rank, device=dev)
    pg = process_group_info(world, dt_rank, args.steps, local, dev)
    if graphed:  # the forward launches of one eager episode, timed with HIP events on the launch stream
        net.timer = timers
        t_ep[0] = T
        for _ in range(T):
            one_step()
        torch.cuda.synchronize()
    net.timer = None
    fwd_ms = sum(e0.elapsed_time(e1) for e0, e1, _, _ in timers) / max(len(timers), 1)
    nnz = int(np.diff(store.row_ptr.cpu().numpy(), axis=1).sum(axis=1).mean())
    fl = mpnn_flops(nnz, n) * B
    st = env.read(best_spins=True)
    best = st["best_solution"].double()
    i = int(best.argmax())
    best_cut, _ = best_cut_over_ranks(float(best[i]), st["best_spins"][i], device=dev)
    if rank == 0:
        name = "GSet G22-like (ER 2000, p=0.01, unit weights)" if args.workload == "gset" else "ER_20spin"
        out = {
            "metric": "env-steps/sec (batched episodes) on " + name + " MaxCut",
            "value": B * args.steps * world / dt,
            "unit": "env-steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": ("f32-accurate MPNN on f16 MFMA (fp16x2 splits)" if n <= 512 else
                      "f32-accurate MPNN: Linears on f16 MFMA (fp16x2 splits), aggregations in f32 from LDS") +
                     " / f64+int (env)",
            "data": "synthetic: seeded graphs; random-init MPNN (std 0.1)",
            "config": {"workload": f"{name} x{B} episodes/GPU: MPNN fwd + greedy act + env step "
                                   f"({'configs[4]' if args.workload == 'gset' else 'configs[1]'})",
                       "n_spins": n, "envs_per_gpu": B, "graphs": ngraphs, "max_steps": T,
                       "parallelism": f"episodes sharded, dp{world}, no collective until the best-cut reduce"},
            "roofline": dict(mfma_roofline(fl / (fwd_ms * 1e-3) / 1e12, forward_kernel_name(n, kind, ngraphs)),
                             traffic=None, avg_launch_ms=fwd_ms, flops_per_launch=fl,
                             timing=("HIP events around the forward launches of one eager episode after the timed "
                                     "region (the timed episodes replay a HIP graph)" if graphed else
                                     "HIP events around every forward launch of the timed region")),
            "execution": ("whole episodes (T steps: forward + fused greedy act + env step) replayed from one HIP "
                          "graph; the episodes are reset on their graphs every T steps inside the timed region"
                          if graphed else "eager launches"),
            "best_cut_after_steps": best_cut,
            "best_cut_note": ("random-init network after the timed steps (a throughput by-product); the full search "
                              "with the pretrained network: tools/gset_search.py, profiles/r05/gset_search_1024.json"
                              if args.workload == "gset" else "random-init network after the timed steps"),
            "process_group": pg,
        }
        if args.workload == "gset":
            # the shared-graph kernels stream node rows through HBM (aggregation from LDS-staged blocks,
            # row-wise Linears): HBM bytes of one forward from the committed PMC pass, over the live time
            tb = pmc_gset_traffic()
            out["roofline"]["traffic"] = tb
            out["roofline"]["traffic_unit"] = "HBM bytes per forward (aggregation + Linear + table launches; PMC, " + \
                os.path.relpath(PMC_GSET, REPO) + ")"
            if tb:
                out["roofline"]["hbm"] = {"bound": "hbm", "achieved": tb / (fwd_ms * 1e-3) / 1e9, "unit": "GB/s",
                                          "peak": HBM_PEAK_GBS, "frac": tb / (fwd_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        print(json.dumps(out))
    if dist:
        torch.distributed.destroy_process_group()


def envstep_bench(args, world, rank, local, dev, dist):
    """SURVEY.md 8d sub-bench: the batched env step kernel alone (spinsystem.py:355-559 for the chosen
    scorer), random actions drawn beforehand, B episodes of ER(n, 0.15).  HBM-bound: algorithmic bytes per
    env-step = state read + write (spins 1, neighbour sum 4, time-since-flip 2 B per vertex, best spins read)
    + fp32 feature rows written (4 W B per vertex) + the flipped vertex's CSR row (+ every row for
    MinDomSet's neighbour counts)."""
    from eco_hip import _lib
    from eco_hip.graphs import GraphStore
    from eco_hip.envs.batched import VecSpinSystem
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, MAIN_OBSERVABLES, RewardSignal, ExtraAction,
                                    OptimisationTarget)
    from eco_hip.parallel import max_over_ranks
    B, n = args.envs, args.n
    T = 2 * n
    cut_like = args.target in ("CUT", "MIN_CUT")
    obs = DEFAULT_OBSERVABLES if cut_like else MAIN_OBSERVABLES
    store = GraphStore.random("ER", B, n, 0.15, seed=1234 + rank, weights="discrete" if cut_like else "uniform",
                              device=dev)
    env = VecSpinSystem(store, B, T, observables=obs, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget[args.target],
                        norm_rewards=True, basin_reward=1. / n)
    env.reset(graph_ids=np.arange(B), seed=1234 + rank)
    g = torch.Generator(device=dev).manual_seed(7 + rank)
    steps = min(args.steps, T - args.warmup)
    acts = torch.randint(0, n, (args.warmup + steps, B), generator=g, device=dev, dtype=torch.int32)
    for i in range(args.warmup):
        env.step(acts[i])
    env.check_errors()
    # the K launches are captured once in a HIP graph and replayed (a Python loop of ctypes launches costs ~20-30
    # us of host time per launch, more than the kernel: timed that way, the host is measured)
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):
        with torch.cuda.graph(graph, stream=cap):
            for i in range(steps):
                env.step(acts[args.warmup + i])
    torch.cuda.current_stream(dev).wait_stream(cap)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt_rank = time.perf_counter() - t0
    dt = max_over_ranks(dt_rank, device=dev)
    pg = process_group_info(world, dt_rank, steps, local, dev)
    env.check_errors()
    k_ms = e0.elapsed_time(e1) / steps
    nnz = float(np.diff(store.row_ptr.cpu().numpy(), axis=1).sum(axis=1).mean())
    W = _lib.obs_x_stride(len(obs))
    per_step = B * (n * (2 * (1 + 4 + 2) + 1 + 4 * W) + 4 * nnz / n + 2 * 192 +
                    (4 * nnz if args.target == "MIN_DOM_SET" else 0))
    achieved = per_step / (k_ms * 1e-3) / 1e9
    if rank == 0:
        out = {
            "metric": f"env-steps/sec (batched episodes) on ER-{n} {args.target}: env step kernel only",
            "value": B * steps * world / dt, "unit": "env-steps/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": dt / steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64+int (env)",
            "data": f"synthetic: seeded ER({n}, 0.15) graphs, one per episode; uniform random actions",
            "config": {"workload": f"ER_{n}spin x{B} episodes/GPU: env step only ({args.target}, "
                                   f"{len(obs)} observables)", "n_spins": n, "envs_per_gpu": B, "max_steps": T,
                       "parallelism": f"episodes sharded, dp{world}, no collective"},
            "roofline": {"bound": "hbm", "kernel": "env_step", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "avg_launch_ms": k_ms, "bytes_per_launch": per_step},
            "process_group": pg,
        }
        print(json.dumps(out))
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
