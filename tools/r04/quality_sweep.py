"""GPU box: ER-200 training-quality sweep of large-batch recipes (B=8192, 10M env-steps each) against the pretrained
ECO ER-200 network, same evaluation as tests/test_training_quality_er200_gpu.py.  One JSON line per variant.
usage: python tools/r04/quality_sweep.py name:key=val,key=val ..."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "eco-dqn_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from test_training_quality_er200_gpu import _best_cuts, _test_graphs, N  # noqa: E402


def run(name, kv):
    from oracle import mpnn_oracle as mo
    from eco_hip.networks.mpnn import MPNN
    dev = torch.device("cuda", 0)
    M = int(kv.get("M", 2048))
    B = int(kv.get("B", 8192))
    agent, _, _, lr = bench.build_train_agent(dev, B, N, "ER", 0.15, M, seed=int(kv.get("seed", 1234)),
                                              replay_episodes=float(kv.get("replay_episodes", 1)),
                                              n_graphs=int(kv.get("graphs", B)))
    if "lr" in kv:
        agent.lr = agent.initial_learning_rate = agent.peak_learning_rate = agent.final_learning_rate = float(kv["lr"])
    if "sync" in kv:
        agent.target_sync_grad_steps = int(kv["sync"])
    graphs = _test_graphs()
    agent.start()
    t0 = time.perf_counter()
    steps = int(float(kv.get("steps", 10e6)))
    curve = []
    while agent._timestep < steps:
        agent.iteration()
        if agent._timestep // 2_000_000 > (agent._timestep - B) // 2_000_000:
            curve.append((agent._timestep, float(_best_cuts(agent.network, graphs, 1, 0, "SIGNED").mean())))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    one = _best_cuts(agent.network, graphs, 1, seed=0, basis="SIGNED").mean()
    fifty = _best_cuts(agent.network, graphs, 50, seed=1, basis="SIGNED").mean()
    print(json.dumps({"name": name, "kv": kv, "lr": agent.lr, "sync": agent.target_sync_grad_steps,
                      "replay": agent.replay_buffer_size, "grad_steps": agent.grad_steps, "train_s": dt,
                      "one": float(one), "fifty": float(fifty), "curve": curve}), flush=True)


def reference():
    from oracle import mpnn_oracle as mo
    from eco_hip.networks.mpnn import MPNN
    f = np.load(os.path.join(REPO, "tests", "golden", "mpnn_fwd.npz"))
    pre = MPNN(device="cuda")
    pre.load_state_dict({k: torch.from_numpy(f["er200/" + k]) for k in mo.KEYS})
    g = _test_graphs()
    print(json.dumps({"name": "pretrained", "one": float(_best_cuts(pre, g, 1, 0, "BINARY").mean()),
                      "fifty": float(_best_cuts(pre, g, 50, 1, "BINARY").mean())}), flush=True)


if __name__ == "__main__":
    reference()
    for arg in sys.argv[1:]:
        name, _, rest = arg.partition(":")
        kv = dict(p.split("=") for p in rest.split(",") if p)
        run(name, kv)
