"""Generate tests/golden/per.npz by running the REFERENCE PrioritisedReplayBuffer
(src/agents/dqn/utils.py:86-277) through a scripted call sequence.

Run in the build container only (needs /root/reference; never on the GPU box):
    python tests/golden/make_per_golden.py

The reference module is imported from /root/reference (its imports are math, pickle, random,
threading, numpy, torch -- no shim needed).  Transitions are tiny tensors whose contents name the
buffer position they were added at, so a sampled batch can be checked for the right rows.

The fixture holds, per call of the script: the op code and its arguments, the heap afterwards
(buffer position and td error per heap position 1..len), beta, and for samples the partitions, the
ranks the reference drew (replayed from the saved numpy RNG state), the buffer positions, the float32
importance weights and the ids found in the sampled transitions.  Data only, no reference source.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")

from src.agents.dqn.utils import PrioritisedReplayBuffer  # noqa: E402

OP_ADD, OP_UPDATE, OP_SAMPLE, OP_REBALANCE = 0, 1, 2, 3


def heap_of(buf):
    n = len(buf)
    bp = np.array([buf.priority_heap[h][0] for h in range(1, n + 1)], dtype=np.int64)
    td = np.array([buf.priority_heap[h][1] for h in range(1, n + 1)], dtype=np.float64)
    return bp, td


def run_case(capacity, alpha, beta0, anneal, script_seed, n_ops):
    rng = np.random.default_rng(script_seed)
    np.random.seed(script_seed + 1000)
    buf = PrioritisedReplayBuffer(capacity=capacity, alpha=alpha, beta0=beta0)
    buf.configure_beta_anneal_time(anneal)
    rec = {k: [] for k in ("op", "arg_n", "arg_bp", "arg_td", "heap_bp", "heap_td", "beta", "parts", "ranks",
                           "s_bp", "s_w", "s_ids")}
    counter = 0
    added = []

    def record(op, n=0, bps=(), tds=(), parts=(), ranks=(), s_bp=(), s_w=(), s_ids=()):
        hb, ht = heap_of(buf)
        rec["op"].append(op)
        rec["arg_n"].append(n)
        rec["arg_bp"].append(np.array(bps, dtype=np.int64))
        rec["arg_td"].append(np.array(tds, dtype=np.float64))
        rec["heap_bp"].append(hb)
        rec["heap_td"].append(ht)
        rec["beta"].append(buf.beta)
        rec["parts"].append(np.array(parts, dtype=np.int64).reshape(-1, 2))
        rec["ranks"].append(np.array(ranks, dtype=np.int64))
        rec["s_bp"].append(np.array(s_bp, dtype=np.int64))
        rec["s_w"].append(np.array(s_w, dtype=np.float32))
        rec["s_ids"].append(np.array(s_ids, dtype=np.int64))

    for _ in range(n_ops):
        u = rng.random()
        if len(buf) < 4 or u < 0.45:
            n = int(rng.integers(1, max(2, capacity // 3)))
            for _ in range(n):
                counter += 1
                t = torch.full((3,), float(counter))
                added.append(counter)
                buf.add(t, torch.tensor([counter]), torch.tensor([0.5]), t + 0.5, torch.tensor([0.]))
            record(OP_ADD, n)
        elif u < 0.75:
            n = int(rng.integers(1, 12))
            live = sorted(buf.buffer2heap.keys())
            bps = [int(b) for b in rng.choice(live, size=min(n, len(live)), replace=False)]
            # ties on purpose (td errors rounded to 0.25) exercise the strict comparisons
            tds = [float(np.round(rng.exponential(1.0) * 4) / 4) if rng.random() < 0.5 else float(rng.exponential(1.0))
                   for _ in bps]
            buf.update_priorities(bps, tds)
            record(OP_UPDATE, len(bps), bps, tds)
        elif u < 0.95 or not buf.full:
            bs = int(rng.integers(2, 9))
            try:
                parts, _ = buf.update_partitions(bs)   # pure: skip sizes with an empty partition (randint(lo, lo))
            except KeyError:
                continue
            if any(lo >= hi for lo, hi in parts):
                continue
            st = np.random.get_state()
            batch, w, bps = buf.sample(bs)
            after = np.random.get_state()
            np.random.set_state(st)
            ranks = [np.random.randint(lo, hi) for lo, hi in buf.partitions]
            np.random.set_state(after)
            assert [buf.priority_heap[r][0] for r in ranks] == list(bps)
            ids = batch[1].reshape(-1).tolist()
            record(OP_SAMPLE, bs, parts=buf.partitions, ranks=ranks, s_bp=bps, s_w=w.reshape(-1).numpy(), s_ids=ids)
        else:
            buf.rebalance()
            record(OP_REBALANCE)
    return rec


def pack(prefix, rec, out):
    for k, v in rec.items():
        if k in ("op", "arg_n", "beta"):
            out[f"{prefix}_{k}"] = np.array(v)
        else:
            lens = np.array([len(a) for a in v], dtype=np.int64)
            out[f"{prefix}_{k}_len"] = lens
            out[f"{prefix}_{k}"] = np.concatenate([a.reshape(-1) for a in v]) if len(v) else np.zeros(0)


def main():
    cases = [(37, 0.7, 0.5, 20, 1, 120), (64, 0.6, 0.4, 50, 2, 160), (10, 0.7, 0.5, 5, 3, 80)]
    out = {"cases": np.array([[c[0], c[3], c[4], c[5]] for c in cases], dtype=np.int64),
           "alpha_beta": np.array([[c[1], c[2]] for c in cases])}
    for i, c in enumerate(cases):
        rec = run_case(*c)
        pack(f"c{i}", rec, out)
        print("case", i, "ops", len(rec["op"]), "samples", sum(1 for o in rec["op"] if o == OP_SAMPLE),
              "rebalances", sum(1 for o in rec["op"] if o == OP_REBALANCE))
    np.savez_compressed(os.path.join(HERE, "per.npz"), **out)


if __name__ == "__main__":
    main()
