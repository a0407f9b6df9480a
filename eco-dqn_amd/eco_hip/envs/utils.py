"""Enums, observable lists and graph generators of the env API.

Names and values are identical to the reference's src/envs/utils.py:10-74 so that
caller code (env_args dicts, experiments/train_eco.py:40-50) works unchanged.
Graph generators keep the reference's class names and `get() -> ndarray[N,N] f64`
contract (src/envs/utils.py:105-436); they draw from numpy's global RNG (the
reference mixes numpy and networkx streams, which cannot be reproduced anyway).
Batched training draws episodes from a device `GraphStore` pool (eco_hip/graphs.py) instead.
"""
import random
from abc import ABC, abstractmethod
from enum import Enum

import numpy as np


class Stopping(Enum):
    NORMAL = 1
    QUARTER = 2
    EARLY = 3


class EdgeType(Enum):
    UNIFORM = 1
    DISCRETE = 2
    RANDOM = 3


class RewardSignal(Enum):
    DENSE = 1
    BLS = 2
    SINGLE = 3
    CUSTOM_BLS = 4


class ExtraAction(Enum):
    PASS = 1
    RANDOMISE = 2
    NONE = 3


class OptimisationTarget(Enum):
    CUT = 1
    ENERGY = 2
    MIN_COVER = 3
    MIN_CUT = 4
    MAX_IND_SET = 5
    MAX_CLIQUE = 6
    MIN_DOM_SET = 7


class SpinBasis(Enum):
    SIGNED = 1
    BINARY = 2


class Observable(Enum):
    SPIN_STATE = 1
    IMMEDIATE_QUALITY_CHANGE = 2
    IMMEDIATE_VALIDITY_DIFFERENCE = 3
    IMMEDIATE_VALIDITY_CHANGE = 4
    TIME_SINCE_FLIP = 5
    EPISODE_TIME = 6
    TERMINATION_IMMANENCY = 7
    NUMBER_OF_QUALITY_IMPROVEMENTS = 8
    NUMBER_OF_VALIDITY_IMPROVEMENTS = 9
    DISTANCE_FROM_BEST_SOLUTION = 10
    DISTANCE_FROM_BEST_STATE = 11
    GLOBAL_VALIDITY_DIFFERENCE = 12
    VALIDITY_BIT = 13


DEFAULT_OBSERVABLES = [Observable.SPIN_STATE,
                       Observable.IMMEDIATE_QUALITY_CHANGE,
                       Observable.TIME_SINCE_FLIP,
                       Observable.DISTANCE_FROM_BEST_SOLUTION,
                       Observable.DISTANCE_FROM_BEST_STATE,
                       Observable.NUMBER_OF_QUALITY_IMPROVEMENTS,
                       Observable.TERMINATION_IMMANENCY]

MAIN_OBSERVABLES = [Observable.SPIN_STATE,
                    Observable.IMMEDIATE_QUALITY_CHANGE,
                    Observable.IMMEDIATE_VALIDITY_DIFFERENCE,
                    Observable.IMMEDIATE_VALIDITY_CHANGE,
                    Observable.TIME_SINCE_FLIP,
                    Observable.EPISODE_TIME,
                    Observable.TERMINATION_IMMANENCY,
                    Observable.NUMBER_OF_QUALITY_IMPROVEMENTS,
                    Observable.NUMBER_OF_VALIDITY_IMPROVEMENTS,
                    Observable.DISTANCE_FROM_BEST_SOLUTION,
                    Observable.DISTANCE_FROM_BEST_STATE,
                    Observable.GLOBAL_VALIDITY_DIFFERENCE,
                    Observable.VALIDITY_BIT]


def _edge_weights(edge_type, size):
    if edge_type == EdgeType.UNIFORM:
        return np.ones(size)
    if edge_type == EdgeType.DISCRETE:
        return 2.0 * np.random.randint(2, size=size) - 1.0
    if edge_type == EdgeType.RANDOM:
        # accepted by the generator; the HIP engine takes integer weights only
        return 2.0 * np.random.rand(size) - 1.0
    raise NotImplementedError()


def _symmetric(n, iu, ju, w):
    m = np.zeros((n, n))
    m[iu, ju] = w
    m[ju, iu] = w
    return m


class GraphGenerator(ABC):
    """src/envs/utils.py:105-126"""

    def __init__(self, n_spins, edge_type, biased=False):
        self.n_spins = n_spins
        self.edge_type = edge_type
        self.biased = biased

    @abstractmethod
    def get(self, with_padding=False):
        raise NotImplementedError


class RandomGraphGenerator(GraphGenerator):
    """Density ~ U(0,1), then each pair connected with that probability (src/envs/utils.py:128-163)."""

    def __init__(self, n_spins=20, edge_type=EdgeType.DISCRETE, biased=False):
        if biased:
            raise NotImplementedError("biased graphs are not on the MaxCut hot path")
        super().__init__(n_spins, edge_type, False)

    def get(self, with_padding=False):
        n = self.n_spins
        density = np.random.uniform()
        iu, ju = np.triu_indices(n, 1)
        keep = np.random.rand(iu.size) < density
        iu, ju = iu[keep], ju[keep]
        return _symmetric(n, iu, ju, _edge_weights(self.edge_type, iu.size))


class RandomErdosRenyiGraphGenerator(GraphGenerator):
    """G(n, p) with p ~ clip(normal(*p_connection), 0, 1) (src/envs/utils.py:165-202)."""

    def __init__(self, n_spins=20, p_connection=[0.1, 0], edge_type=EdgeType.DISCRETE):
        super().__init__(n_spins, edge_type, False)
        if type(p_connection) not in [list, tuple]:
            p_connection = [p_connection, 0]
        assert len(p_connection) == 2, "p_connection must have length 2"
        self.p_connection = p_connection

    def get(self, with_padding=False):
        n = self.n_spins
        p = np.clip(np.random.normal(*self.p_connection), 0, 1)
        iu, ju = np.triu_indices(n, 1)
        keep = np.random.rand(iu.size) < p
        iu, ju = iu[keep], ju[keep]
        return _symmetric(n, iu, ju, _edge_weights(self.edge_type, iu.size))


class RandomBarabasiAlbertGraphGenerator(GraphGenerator):
    """Preferential attachment with m edges per new vertex (src/envs/utils.py:204-236)."""

    def __init__(self, n_spins=20, m_insertion_edges=4, edge_type=EdgeType.DISCRETE):
        super().__init__(n_spins, edge_type, False)
        self.m_insertion_edges = m_insertion_edges

    def get(self, with_padding=False):
        n, m = self.n_spins, self.m_insertion_edges
        targets = list(range(m))
        repeated = []
        iu, ju = [], []
        for src in range(m, n):
            for t in targets:
                iu.append(t)
                ju.append(src)
            repeated.extend(targets)
            repeated.extend([src] * m)
            chosen = set()
            while len(chosen) < m:
                chosen.add(repeated[np.random.randint(len(repeated))])
            targets = sorted(chosen)
        iu, ju = np.array(iu, dtype=np.int64), np.array(ju, dtype=np.int64)
        return _symmetric(n, iu, ju, _edge_weights(self.edge_type, iu.size))


def _edge_type_of(matrices):
    """EdgeType of a collection of adjacency matrices, from the set of weights they use: {0, 1} -> UNIFORM,
    {0, +-1} -> DISCRETE, anything else -> RANDOM (the classification the reference's known-graph generators
    make, src/envs/utils.py:323-330, :351-358)."""
    weights = set()
    for m in matrices:
        weights.update(np.unique(np.asarray(m)).tolist())
    if weights <= {0, 1}:
        return EdgeType.UNIFORM
    if weights <= {0, -1, 1}:
        return EdgeType.DISCRETE
    return EdgeType.RANDOM


class SetGraphGenerator(GraphGenerator):
    """Known graphs of one size (src/envs/utils.py:347-382): `ordered` hands them out in turn, cycling; otherwise
    each get() draws one uniformly with python's `random` module (the stream set_global_seed seeds, consumed as
    the reference's random.sample(graphs, k=1) consumes it).  With biases, get() returns (matrix, bias) pairs."""

    def __init__(self, matrices, biases=None, ordered=False):
        matrices = list(matrices)
        if len({np.asarray(m).shape[0] for m in matrices}) != 1:
            raise NotImplementedError("All graphs in SetGraphGenerator must have the same dimension.")
        super().__init__(np.asarray(matrices[0]).shape[0], _edge_type_of(matrices), biases is not None)
        if self.biased:
            biases = list(biases)
            assert len(biases) == len(matrices), "Must pass through the same number of matrices and biases."
            assert all(len(b) == self.n_spins + 1 for b in biases), \
                "All biases and must have the same dimension as the matrices."
            self.graphs = list(zip(matrices, biases))
        else:
            self.graphs = matrices
        self.ordered = ordered
        self.i = 0

    def get(self, with_padding=False):
        if not self.ordered:
            return self.graphs[random.sample(range(len(self.graphs)), 1)[0]]
        item = self.graphs[self.i]
        self.i = (self.i + 1) % len(self.graphs)
        return item


class SingleGraphGenerator(SetGraphGenerator):
    """One known graph (src/envs/utils.py:319-345): every get() returns it (with its bias, when given)."""

    def __init__(self, matrix, bias=None):
        # the reference's single-graph generator checks no bias length (src/envs/utils.py:319-345), so the set
        # generator's n_spins + 1 assertion is not applied here: the pair is stored as given
        super().__init__([matrix], None, ordered=True)
        self.matrix, self.bias = matrix, bias
        if bias is not None:
            self.biased = True
            self.graphs = [(matrix, bias)]
