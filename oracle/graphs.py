"""Seeded synthetic graph generators for tests and fixtures (TEST INFRASTRUCTURE).

The reference draws training graphs with networkx (`src/envs/utils.py:165-236`) and
ships its evaluation graphs as pickles under `_graphs/`.  Pickles are never loaded
here (no unpickling of files that ship with the reference), and networkx's RNG
stream is not reproducible on the GPU, so every fixture and parity case uses the
graphs below instead: plain numpy, fully determined by the seed.

Edge weights follow the reference's `EdgeType` (`src/envs/utils.py:16-19`):
  * "discrete": independent fair +-1 per edge (ER/BA max_cut training, `train_eco.py:258`)
  * "uniform":  weight 1 on every edge (min_cover etc.; G22-style unit weights)
All matrices are float64, symmetric, zero diagonal -- exactly the
`np.ndarray[N,N] f64` contract of `GraphGenerator.get()` (`src/envs/utils.py:121-123`).
"""
import numpy as np


def _weights(rng, n_edges, weights):
    if weights == "discrete":
        return 2.0 * rng.integers(0, 2, size=n_edges) - 1.0
    if weights == "uniform":
        return np.ones(n_edges)
    raise ValueError(weights)


def er_graph(n, p, rng, weights="discrete"):
    """Erdos-Renyi G(n, p) with the reference's weight convention."""
    iu, ju = np.triu_indices(n, 1)
    keep = rng.random(iu.size) < p
    iu, ju = iu[keep], ju[keep]
    w = _weights(rng, iu.size, weights)
    J = np.zeros((n, n))
    J[iu, ju] = w
    J[ju, iu] = w
    return J


def ba_graph(n, m, rng, weights="discrete"):
    """Barabasi-Albert preferential attachment (m edges per inserted vertex),
    the same process as networkx.barabasi_albert_graph used at
    `src/envs/utils.py:228-236` (not the same RNG stream)."""
    J = np.zeros((n, n))
    targets = list(range(m))
    repeated = []
    src = m
    while src < n:
        for t in targets:
            J[src, t] = J[t, src] = 1.0
        repeated.extend(targets)
        repeated.extend([src] * m)
        chosen = set()
        while len(chosen) < m:
            chosen.add(repeated[int(rng.integers(0, len(repeated)))])
        targets = sorted(chosen)
        src += 1
    iu, ju = np.nonzero(np.triu(J, 1))
    w = _weights(rng, iu.size, weights)
    J[iu, ju] = w
    J[ju, iu] = w
    return J


def negative_mlr_graph(n, rng):
    """A graph whose max local reward is negative: every edge weighs -1, so every
    row sum is <= 0 (`score_solver.py:367-375`: mlr = max of NONZERO entries of g(-1))."""
    J = -np.abs(er_graph(n, 0.3, rng))
    if not np.any(J):
        J[0, 1] = J[1, 0] = -1.0
    return J
