"""The known-graph generators of eco_hip.envs.utils (the reference's SingleGraphGenerator / SetGraphGenerator,
src/envs/utils.py:319-382): edge-type classification, ordered cycling, seeded unordered draws consuming python's
`random` as the reference's random.sample(graphs, k=1), and the dimension check."""
import random

import numpy as np
import pytest


def _graphs(rng, n, k, weights):
    out = []
    for _ in range(k):
        J = np.triu((rng.random((n, n)) < 0.3).astype(float), 1)
        if weights == "discrete":
            J *= rng.choice([-1.0, 1.0], size=J.shape)
        elif weights == "random":
            J *= rng.random(J.shape)
        out.append(J + J.T)
    return out


@pytest.mark.parametrize("weights,kind", [("uniform", "UNIFORM"), ("discrete", "DISCRETE"), ("random", "RANDOM")])
def test_edge_type_and_ordered_cycle(weights, kind):
    from eco_hip.envs.utils import SetGraphGenerator, SingleGraphGenerator, EdgeType
    gs = _graphs(np.random.default_rng(1), 12, 5, weights)
    gen = SetGraphGenerator(gs, ordered=True)
    assert gen.edge_type == EdgeType[kind] and gen.n_spins == 12
    for i in range(12):
        assert gen.get() is gs[i % 5]
    one = SingleGraphGenerator(gs[2])
    assert one.edge_type == EdgeType[kind] and all(one.get() is gs[2] for _ in range(3))


def test_unordered_draws_follow_python_random():
    from eco_hip.envs.utils import SetGraphGenerator
    gs = _graphs(np.random.default_rng(2), 10, 7, "discrete")
    gen = SetGraphGenerator(gs)
    random.seed(5)
    got = [gen.get() for _ in range(20)]
    random.seed(5)
    ref = [random.sample(gs, k=1)[0] for _ in range(20)]  # the reference's draw (utils.py:380)
    assert all(a is b for a, b in zip(got, ref))


def test_mixed_dimensions_rejected():
    from eco_hip.envs.utils import SetGraphGenerator
    with pytest.raises(NotImplementedError):
        SetGraphGenerator([np.zeros((4, 4)), np.zeros((5, 5))])


def test_single_graph_generator_takes_any_bias_length():
    """The reference's SingleGraphGenerator stores (matrix, bias) as given (src/envs/utils.py:319-345): an N-long bias
    is accepted (the set generator's N + 1 check does not apply) and returned with the matrix on every get()."""
    from eco_hip.envs.utils import SingleGraphGenerator
    J = _graphs(np.random.default_rng(3), 9, 1, "discrete")[0]
    bias = np.arange(9, dtype=float)
    gen = SingleGraphGenerator(J, bias)
    assert gen.biased
    for _ in range(3):
        m, b = gen.get()
        assert m is J and b is bias
