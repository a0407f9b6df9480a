"""Training-quality test set: 50 seeded ER(20, p=0.15) graphs with fair +-1 weights (the reference's
ER_20 max_cut training distribution, experiments/train_eco.py:255-264, 322-327) and their exact maximum
cuts by exhaustive enumeration (oracle/maxcut_exact.py) -> tests/golden/er20_opt.npz.

The reference's own ER_20 test pickles (_graphs/testing/ER_20spin_p15_50graphs.pkl) are not unpickled;
its reported best-known mean for the ER_20 validation set (10.68) is the same distribution.
Run in the build container:  python tests/golden/make_er20_opt.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import graphs  # noqa: E402
from oracle.maxcut_exact import max_cut  # noqa: E402


def main(n_graphs=50, n=20, seed=2020):
    rng = np.random.default_rng(seed)
    mats = np.stack([graphs.er_graph(n, 0.15, rng) for _ in range(n_graphs)])
    opt, spins = zip(*(max_cut(J) for J in mats))
    np.savez_compressed(os.path.join(HERE, "er20_opt.npz"), graphs=mats.astype(np.int8),
                        opt_cut=np.array(opt), opt_spins=np.array(spins, dtype=np.int8), seed=np.int64(seed))
    print("mean optimal cut", np.mean(opt))


if __name__ == "__main__":
    main()
