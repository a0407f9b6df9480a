"""GPU box: like-for-like quality sweep (tests/quality_common.py: the benched agent with fresh graphs per episode,
learn() with its own _best selection on 50 validation graphs every 50 k env-steps) over learning-rate schedules,
target-sync periods, staggered episodes (stagger=1) and ring sizes (ring=<vector steps>).
One JSON line per (variant, seed): test-graph single-attempt and best-of-50 mean best cuts of the _best and of the
final network.  usage: python tools/r06/quality_sweep.py ER|BA name:key=val,... [name:...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "eco-dqn_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import quality_common as qc  # noqa: E402


def configure(agent, kv):
    lr = float(kv.get("lr", agent.peak_learning_rate))  # default: bench's 1e-4 x sqrt(M / 64)
    if "decay_to" in kv:  # linear decay from lr (constant until decay_from) to decay_to at 10 M env-steps
        agent.update_learning_rate = True
        agent.initial_learning_rate = agent.peak_learning_rate = agent.lr = lr
        agent.peak_learning_rate_step = int(float(kv.get("decay_from", 5e6)))
        agent.final_learning_rate = float(kv["decay_to"])
        agent.final_learning_rate_step = int(float(kv.get("decay_end", 10e6)))
    else:
        agent.lr = agent.initial_learning_rate = agent.peak_learning_rate = agent.final_learning_rate = lr
    if "sync" in kv:
        agent.target_sync_grad_steps = int(kv["sync"])
    if "stagger" in kv:
        agent.stagger_episodes = bool(int(kv["stagger"]))


def main():
    kind = sys.argv[1]
    n = 200
    graphs = qc.family_graphs(kind, n, 20200 if kind == "ER" else 20201)
    pre = qc.pretrained(os.path.join(REPO, "tests", "golden", "mpnn_fwd.npz" if kind == "ER" else "pretrained_ba200.npz"),
                        "er200/" if kind == "ER" else "ba200/")
    r1 = qc.best_cuts(pre, graphs, 1, 0, "BINARY", n).mean()
    r50 = qc.best_cuts(pre, graphs, 50, 1, "BINARY", n).mean()
    print(json.dumps({"name": "pretrained", "one": float(r1), "fifty": float(r50)}), flush=True)
    for spec in sys.argv[2:]:
        name, _, rest = spec.partition(":")
        kv = dict(p.split("=") for p in rest.split(",") if p)
        for seed in [int(s) for s in kv.pop("seeds", "1234/1/2").split("/")]:
            M = int(kv.get("M", 2048))
            # ring: the replay ring in vector steps of B transitions (default: the benched ring)
            rep = {} if "ring" not in kv else {"replay_episodes": float(kv["ring"]) / (2 * n)}
            best, info = qc.train_and_select(kind, 0.15 if kind == "ER" else 4, n, seed, M=M,
                                             configure=lambda ag: configure(ag, kv), **rep)
            out = {"name": name, "kv": kv, "seed": seed, "best_at": info["best_at"], "train_s": info["train_s"]}
            for tag, net in (("best", best), ("final", info["final_net"])):
                out[tag + "_one"] = float(qc.best_cuts(net, graphs, 1, 0, "SIGNED", n).mean() / r1)
                out[tag + "_fifty"] = float(qc.best_cuts(net, graphs, 50, 1, "SIGNED", n).mean() / r50)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
