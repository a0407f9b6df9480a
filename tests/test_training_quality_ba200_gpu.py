"""Training quality of configs[3]'s recipe on its graph family (VERDICT r04 missing #3): bench.build_train_agent
with BA(200, m = 4) graphs -- the recipe bench.py --graph BA runs at N = 500 (M = 2048, lr 1e-4 sqrt(M/64) =
5.66e-4, target sync every 16 gradient steps, a fresh graph per episode, a ring of one episode's worth) at the size
the reference ships a pretrained network for -- trained by DQN.learn() for the reference's 10 M env-steps
(experiments/train_eco.py:322-333, 368-377: BA m = 4, the N = 200 parameters), the `_best` snapshot selected by
learn()'s evaluation on 50 held-out BA-200 validation graphs every 50 k env-steps (dqn.py:349-361), then rolled out
greedily on 50 other seeded BA-200 test graphs beside the reference's network_best_BA_200spin.pth (exported
weights-only by tests/golden/make_pretrained.py; BINARY basis as its test script).  Three seeds; bars: single-attempt
ratio >= 0.99 on the mean over seeds, best of 50 >= 0.99 for every seed (measured 1.010 / 0.999-1.005 at sync 16,
profiles/r05/quality/sweep_r05m_sync16_ba200.jsonl; 1.012 / 1.002 at 125)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
import quality_common as qc

pytestmark = pytest.mark.gpu

N = 200


def test_benched_recipe_matches_pretrained_ba200():
    graphs = qc.family_graphs("BA", N, 20201)
    pre = qc.pretrained(os.path.join(GOLDEN, "pretrained_ba200.npz"), "ba200/")
    ref1 = qc.best_cuts(pre, graphs, 1, seed=0, basis="BINARY", n=N)
    ref50 = qc.best_cuts(pre, graphs, 50, seed=1, basis="BINARY", n=N)
    ratios1, ratios50 = [], []
    for seed in (1234, 1, 2):
        best, info = qc.train_and_select("BA", 4, N, seed)
        one = qc.best_cuts(best, graphs, 1, seed=0, basis="SIGNED", n=N)
        fifty = qc.best_cuts(best, graphs, 50, seed=1, basis="SIGNED", n=N)
        ratios1.append(one.mean() / ref1.mean())
        ratios50.append(fifty.mean() / ref50.mean())
        print(f"BA-200 seed {seed}: {info['steps']} env-steps, {info['grad_steps']} gradient steps, "
              f"{info['evaluations']} evaluations, learn() {info['train_s']:.1f} s, graphs regenerated "
              f"{info['graphs_regenerated']} / reused {info['graphs_reused']}; _best at {info['best_at']} "
              f"(validation {info['best_val']:.2f}); test mean best cut {one.mean():.2f} (1 attempt) / "
              f"{fifty.mean():.2f} (best of 50) vs pretrained {ref1.mean():.2f} / {ref50.mean():.2f}: ratios "
              f"{ratios1[-1]:.4f} / {ratios50[-1]:.4f}", flush=True)
    print("BA-200 single-attempt ratio mean over seeds", float(np.mean(ratios1)))
    assert np.mean(ratios1) >= 0.99
    assert min(ratios50) >= 0.99
