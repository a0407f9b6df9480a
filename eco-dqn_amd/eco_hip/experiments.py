"""Batched best-cut search harness: experiments/utils.py:22-303 (`test_network`) on the HIP engine.

For every test graph: a Greedy run from the all -1 state, `n_attempts` network-greedy
episodes from random initial spins (all attempts in ONE batch on the device: MPNN
forward + fused argmax + env step per vector step), and a Greedy run from each of the
same random initialisations.  Returns the reference's DataFrame columns.
"""
import os
import time
from collections import namedtuple

import numpy as np
import pandas as pd
import torch

from . import _lib
from .envs.batched import VecSpinSystem
from .envs.utils import SpinBasis
from .graphs import GraphStore


Graph = namedtuple('Graph', 'name n_vertices n_edges matrix bk_val bk_sol')


def read_mc(path):
    """GSet / MaxCut `.mc` instance (experiments/utils.py:400-409): first line `n m`, then `i j w` per edge,
    1-based.  Returns (n, m, i, j, w) with 0-based endpoints."""
    with open(path) as f:
        head = f.readline().split()
        if len(head) != 2:
            raise ValueError("First line in file should define graph dimensions.")
        n, m = int(head[0]), int(head[1])
        rows = np.loadtxt(f, dtype=np.int64, ndmin=2)
    if rows.size == 0:
        rows = np.zeros((0, 3), np.int64)
    if rows.shape[1] != 3:
        raise ValueError("edge lines must be `i j w`")
    return n, m, rows[:, 0] - 1, rows[:, 1] - 1, rows[:, 2]


def load_graph(graph_dir, graph_name, dense=True):
    """experiments/utils.py:391-418: instances/<name>.mc, bkvl/<name>.bkvl, bksol/<name>.bksol.
    `matrix` is the reference's dense f64 adjacency (dense=False: a single-graph GraphStore instead, so
    G22-size graphs never materialise N x N on the host).  The best-known solution gets the reference's
    appended random 'no-action' spin (utils.py:416)."""
    n, m, i, j, w = read_mc(os.path.join(graph_dir, 'instances', graph_name + '.mc'))
    if dense:
        matrix = np.zeros((n, n))
        matrix[i, j] = w
        matrix[j, i] = w
    else:
        matrix = GraphStore.from_edges(n, i, j, w)
    with open(os.path.join(graph_dir, 'bkvl', graph_name + '.bkvl')) as f:
        bk_val = float(f.readline())
    with open(os.path.join(graph_dir, 'bksol', graph_name + '.bksol')) as f:
        s = f.readline().strip()
        bk_sol = np.array([int(ch) for ch in s] + [np.random.choice([0, 1])])
    return Graph(graph_name, n, m, matrix, bk_val, bk_sol)


def load_graph_set(graph_save_loc):
    """experiments/utils.py:420-432: a pickled list of graphs (networkx Graphs, scipy CSR matrices or dense
    arrays, as the reference's `_graphs/*.pkl` test sets) -> list of dense f64 adjacency arrays.
    Unpickling executes code from the file: load only graph sets you trust (e.g. ones written by
    `save_graph_set`).  `GraphStore.from_dense(load_graph_set(path))` puts them on the device."""
    import pickle
    with open(graph_save_loc, "rb") as f:
        graphs = pickle.load(f)

    def to_array(g):
        if type(g).__module__.startswith("networkx"):
            import networkx as nx
            return nx.to_numpy_array(g)
        if hasattr(g, "toarray"):  # scipy.sparse
            return g.toarray()
        return np.asarray(g, dtype=np.float64)

    graphs = [to_array(g) for g in graphs]
    print('{} target graphs loaded from {}'.format(len(graphs), graph_save_loc))
    return graphs


def save_graph_set(graph_save_loc, graphs):
    """Write a graph set in the reference's pickle format (a list of dense adjacency arrays)."""
    import pickle
    with open(graph_save_loc, "wb") as f:
        pickle.dump([np.asarray(g, dtype=np.float64) for g in graphs], f)


def _greedy(env):
    """Run the batched Greedy solver (solver.py:88-131) to completion on `env` (already reset)."""
    for _ in range(env.max_steps):
        a = env.greedy_actions()
        if bool(env.read()["done"].bool().all()):
            break
        env.step(a)
    st = env.read(best_spins=True)
    return st["best_solution"].cpu().numpy(), st["best_spins"].cpu().numpy().astype(np.float64)


def test_network(network, env_args, graphs_test, device=None, step_factor=1, batched=True, n_attempts=50,
                 return_raw=False, return_history=False, max_batch_size=None, seed=None):
    """experiments/utils.py:22-31.  `network`: eco_hip MPNN.  Attempts are batched on the GPU
    (the sequential variant of the reference is broken upstream, utils.py:343-363)."""
    if return_history:
        raise NotImplementedError("return_history is not on the hot path")
    dev = torch.device(device) if device is not None else network.flat.device
    rng = np.random.RandomState(seed) if seed is not None else np.random
    reversible = env_args["reversible_spins"]
    n_attempts = n_attempts if reversible else 1
    results, results_raw = [], []
    basis = env_args.get("spin_basis", SpinBasis.SIGNED)
    allowed = 0.0 if basis == SpinBasis.BINARY else -1.0
    for j, test_graph in enumerate(graphs_test):
        n = test_graph.shape[0]
        n_steps = int(n * step_factor)
        store = GraphStore.from_dense([np.asarray(test_graph, dtype=np.float64)], device=dev)
        # greedy from the all -1 state (utils.py:100-109)
        genv = VecSpinSystem(store, 1, n_steps, **env_args)
        genv.reset(graph_ids=[0], spins=-np.ones((1, n), dtype=np.int64))
        gcut, gsol = _greedy(genv)
        greedy_single_cut, greedy_single_spins = float(gcut[0]), gsol[0]
        best_solutions, best_spins, init_spins, greedy_cuts, greedy_spins = [], [], [], [], []
        t_total = 0.0
        done_attempts = 0
        while done_attempts < n_attempts:
            bsz = n_attempts - done_attempts if max_batch_size is None else min(max_batch_size,
                                                                              n_attempts - done_attempts)
            if reversible:
                spins = 2 * rng.randint(2, size=(bsz, n)) - 1       # spinsystem.py:294 per attempt
            else:
                spins = -np.ones((bsz, n), dtype=np.int64)
            env = VecSpinSystem(store, bsz, n_steps, **env_args)
            env.reset(graph_ids=np.zeros(bsz, dtype=np.int64), spins=spins)
            gids = env.graph_ids
            acts = torch.empty(bsz, dtype=torch.int32, device=dev)
            act = _lib.ActConfig(0.0, int(reversible), allowed, 0, 0)
            torch.cuda.synchronize(dev)
            t0 = time.time()
            scope = _lib.ECO_NORM_PER_CALL  # same batch every step: the call's max degree once, then reused
            for _ in range(n_steps):
                network.forward_graphs(env.obs_x, store, gids, norm_scope=scope, act=act, actions_out=acts)
                env.step(acts)
                scope = _lib.ECO_NORM_PER_CALL_REUSE
            st = env.read(best_spins=True)
            torch.cuda.synchronize(dev)
            t_total += time.time() - t0
            best_solutions += list(st["best_solution"].cpu().numpy())
            best_spins += list(st["best_spins"].cpu().numpy().astype(np.float64))
            init_spins += list(spins.astype(np.float64))
            if reversible:
                genv = VecSpinSystem(store, bsz, n_steps, **env_args)
                genv.reset(graph_ids=np.zeros(bsz, dtype=np.int64), spins=spins)
                gc, gs = _greedy(genv)
                greedy_cuts += list(gc)
                greedy_spins += list(gs)
            done_attempts += bsz
        i_best = int(np.argmax(best_solutions))
        if reversible:
            ig = int(np.argmax(greedy_cuts))
            greedy_random_cut, greedy_random_spins = greedy_cuts[ig], greedy_spins[ig]
            greedy_random_mean_cut = float(np.mean(greedy_cuts))
        else:
            greedy_random_cut, greedy_random_spins = greedy_single_cut, greedy_single_spins
            greedy_random_mean_cut = greedy_single_cut
        results.append([best_solutions[i_best], best_spins[i_best], float(np.mean(best_solutions)),
                        greedy_single_cut, greedy_single_spins, greedy_random_cut, greedy_random_spins,
                        greedy_random_mean_cut, t_total / n_attempts])
        results_raw.append([init_spins, best_solutions, best_spins, greedy_cuts, greedy_spins])
    results = pd.DataFrame(data=results, columns=["cut", "sol", "mean cut", "greedy (+1 init) cut",
                                                  "greedy (+1 init) sol", "greedy (rand init) cut",
                                                  "greedy (rand init) sol", "greedy (rand init) mean cut", "time"])
    if not return_raw:
        return results
    results_raw = pd.DataFrame(data=results_raw, columns=["init spins", "cuts", "sols", "greedy cuts", "greedy sols"])
    return [results, results_raw]
