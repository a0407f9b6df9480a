"""Debug: replay tests/test_problems_gpu.py::test_problem_env_batched_vs_oracle for one case and report the first
mismatching step in detail (reward, the oracle's history verdict and local-minimum test, our rows)."""
import sys
import zlib
import os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eco-dqn_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
from oracle import graphs as og
from oracle import problems_oracle as po
import test_problems_gpu as tp
from eco_hip.envs.batched import VecSpinSystem
from eco_hip.graphs import GraphStore

target, mode, n, kind = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
rng = np.random.default_rng(zlib.crc32(f"{target}/{mode}/{n}".encode()))
w = "discrete" if target in ("MIN_CUT", "CUT") else "uniform"
Js = [og.er_graph(n, 0.2, rng, w) if kind == "ER" else og.ba_graph(n, 4, rng, w) for _ in range(3)]
B = 6
gids = np.array([b % 3 for b in range(B)])
T = 2 * n if mode == "eco" else n
vec = VecSpinSystem(GraphStore.from_dense(Js), B, T, want_f64=True, **tp._env_args(target, mode, n))
spins = (2 * rng.integers(0, 2, (B, n)) - 1) if mode == "eco" else -np.ones((B, n), dtype=np.int64)
vec.reset(graph_ids=gids, spins=spins)
envs = []
for b in range(B):
    e = po.ProblemSpinSystemOracle(Js[gids[b]], T, init_reset=False, **tp._oracle_kwargs(target, mode, n))
    e.reset(spins=spins[b])
    envs.append(e)
done = np.zeros(B, bool)
n_random = T // 2 if mode == "eco" else n // 2
for t in range(T):
    if t < n_random:
        acts = rng.integers(0, n, B)
        a_dev = torch.tensor(acts, dtype=torch.int32, device="cuda")
        greedy_stop = np.zeros(B, bool)
    else:
        a_dev = vec.greedy_actions()
        acts = a_dev.cpu().numpy()
        gacts = [po.greedy_action(e) if not d else None for e, d in zip(envs, done)]
        greedy_stop = np.array([g is None for g in gacts]) & ~done
        done |= greedy_stop
    pre_rows = vec.obs_f64.cpu().numpy().copy()
    st8 = vec.state.cpu().numpy().view(np.uint8)
    off_scal = (256 + 12 * (T + 1) + 255) // 256 * 256
    rec = st8[off_scal:off_scal + 128].view(np.uint32)
    al = lambda x: (x + 255) // 256 * 256
    cap = 16
    while cap < 2 * (T + 1):
        cap *= 2
    o_sp = al(off_scal + 128 * B); o_f = al(o_sp + B * n); o_t = al(o_f + 4 * B * n); o_b = al(o_t + 2 * B * n)
    o_vi = al(o_b + B * n); o_vh = al(o_vi + B * cap * 4); o_vs = al(o_vh + B * cap * 8)
    W = (n + 63) // 64
    vidx = st8[o_vi:o_vi + cap * 4].view(np.uint32)
    vh = st8[o_vh:o_vh + cap * 8].view(np.uint64)
    vst = st8[o_vs:o_vs + (T + 1) * W * 8].view(np.uint64)
    if t >= 50:
        hsh = int(rec[16]) | (int(rec[17]) << 32)
        occ = np.flatnonzero(vidx)
        print("  occupied slots", len(occ), "ids", sorted(vidx[occ].tolist())[-5:], "slot of hash", hsh & (cap - 1),
              "vidx there", vidx[hsh & (cap - 1)], "vh there %x" % vh[hsh & (cap - 1)])
        print("  vst rows 48..52", [hex(x) for x in vst[48 * W:53 * W]])
    if t >= 44:
        print(f"t={t} b0 hash={int(rec[16]) | (int(rec[17]) << 32):016x} t={rec[18]} visits={rec[23]} early={rec[22]} act_next={acts[0]}")
    _, rew, dn = vec.step(a_dev)
    vec.check_errors()
    rew = rew.cpu().numpy()
    rows = vec.obs_f64.cpu().numpy()
    bad = False
    for b, e in enumerate(envs):
        if done[b]:
            continue
        hist_before = set(tuple(x) for x in getattr(e.history, "_states", [])) if e.history is not None else None
        _, r, d, _ = e.step(int(acts[b]))
        ref = e.state_rows()
        if rew[b] != r or not np.array_equal(rows[b], ref):
            diff = np.argwhere(rows[b] != ref)
            print(f"t={t} b={b} act={acts[b]} rew ours={rew[b]} ref={r} done ours={dn[b].item()} ref={d}")
            print("  rows differ at (obs, vertex):", diff[:10].tolist(), "count", len(diff))
            print("  ours g>0 count:", int((rows[b][1] > 0).sum()), "ref:", int((ref[1] > 0).sum()))
            print("  ours obs row 3..6:", rows[b][3:7, 0].tolist(), "ref:", ref[3:7, 0].tolist())
            print("  pre-step ours row1 at act:", pre_rows[b][1, acts[b]])
            print("  history attrs:", [a for a in dir(e.history) if not a.startswith("__")] if e.history else None)
            bad = True
        done[b] |= d
    if bad:
        break
print("end t", t)
