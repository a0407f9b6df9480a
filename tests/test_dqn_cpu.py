"""Host-side DQN logic without a GPU: the epsilon / learning-rate schedules against values recorded
from the reference (tests/golden/schedules.npz, dqn.py:467-488), and save -> load of the flat
parameter buffer through the reference's state_dict format (dqn.py:604-610)."""
import os
import types

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import mpnn_oracle as mo


def _hp(f, i):
    keys = ("initial_exploration_rate", "final_exploration_rate", "final_exploration_step",
            "initial_learning_rate", "peak_learning_rate", "peak_learning_rate_step", "final_learning_rate",
            "final_learning_rate_step")
    return {k: float(f[f"h{i}/{k}"]) for k in keys}


@pytest.mark.parametrize("i", [0, 1])
def test_schedules_match_reference(i):
    from eco_hip.agents.dqn.dqn import DQN
    f = np.load(os.path.join(GOLDEN, "schedules.npz"))
    hp = _hp(f, i)
    ns = types.SimpleNamespace(**hp)
    ns.lr = hp["initial_learning_rate"]
    ns.epsilon = hp["initial_exploration_rate"]
    for t, eps, lr in zip(f["timesteps"], f[f"h{i}/eps"], f[f"h{i}/lr"]):
        DQN.update_epsilon(ns, int(t))
        DQN.update_lr(ns, int(t))
        assert ns.epsilon == eps, (int(t), ns.epsilon, eps)   # same float64 expression: exact
        assert ns.lr == lr, (int(t), ns.lr, lr)


def test_save_load_round_trip(tmp_path):
    from eco_hip.agents.dqn.dqn import DQN
    from eco_hip.networks.mpnn import MPNN
    net = MPNN(device="cpu")
    w = mo.init_weights(torch.Generator().manual_seed(3), std=0.05)
    net.load_state_dict(w)
    ns = types.SimpleNamespace(network=net)
    path = str(tmp_path / "net.pth")
    DQN.save(ns, path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    assert list(sd) == mo.KEYS                       # the reference MPNN's state_dict keys, in order
    for k in mo.KEYS:
        assert torch.equal(sd[k], w[k])
    net2 = MPNN(device="cpu")
    DQN.load(types.SimpleNamespace(network=net2), path)
    assert torch.equal(net2.flat, net.flat)
    # the reference's extension fix-up is a no-op (dqn.py:605-606): the path is used as given
    DQN.save(ns, str(tmp_path / "noext"))
    assert (tmp_path / "noext").exists() and not (tmp_path / "noext.pth").exists()
