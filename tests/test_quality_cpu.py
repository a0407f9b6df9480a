"""The exact MaxCut oracle (oracle/maxcut_exact.py) behind the training-quality test: checked against a
plain itertools enumeration on small graphs, and the committed ER-20 optima (tests/golden/er20_opt.npz)
re-derived for a few graphs, with the stored optimal spins achieving the stored cut."""
import itertools
import os

import numpy as np

from conftest import GOLDEN
from oracle import graphs
from oracle.maxcut_exact import cut_value, max_cut


def _naive(J):
    n = J.shape[0]
    best = -np.inf
    for bits in itertools.product((-1.0, 1.0), repeat=n):
        s = np.array(bits)
        best = max(best, 0.25 * np.sum(J * (1 - np.outer(s, s))))   # src/envs/utils.py:90-94
    return best


def test_exhaustive_matches_naive_enumeration():
    rng = np.random.default_rng(3)
    for n, p, w in ((6, 0.5, "discrete"), (9, 0.4, "discrete"), (10, 0.3, "uniform"), (8, 0.0, "discrete")):
        J = graphs.er_graph(n, p, rng, weights=w)
        best, s = max_cut(J, block_bits=4)
        assert best == _naive(J)
        assert cut_value(J, s) == best


def test_er20_optima_fixture():
    f = np.load(os.path.join(GOLDEN, "er20_opt.npz"))
    mats, opt, spins = f["graphs"].astype(np.float64), f["opt_cut"], f["opt_spins"]
    assert mats.shape == (50, 20, 20) and np.all(mats == mats.transpose(0, 2, 1))
    for g in range(50):
        assert cut_value(mats[g], spins[g]) == opt[g]
    for g in (0, 17, 49):
        assert max_cut(mats[g])[0] == opt[g]
