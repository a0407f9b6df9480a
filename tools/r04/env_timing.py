"""Per-phase timing of the batched env step kernel (diagnostic, GPU only): loads libecohip_timing.so
(`make -C eco-dqn_amd timing`: wall_clock64 stamps at the phases of env_step_kernel) and reports, over the
episodes of one ER-200 x 8192 step, the mean duration of each phase and the spread of wave start / end times.
usage: python tools/r04/env_timing.py [--envs 8192] [--n 200]"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ECO_HIP_LIB"] = os.environ.get("ECO_HIP_LIB") or os.path.join(ROOT, "eco-dqn_amd", "eco_hip",
                                                                          "libecohip_timing.so")
sys.path.insert(0, os.path.join(ROOT, "eco-dqn_amd"))
import torch  # noqa: E402

from eco_hip import _lib  # noqa: E402
from eco_hip.graphs import GraphStore  # noqa: E402
from eco_hip.envs.batched import VecSpinSystem  # noqa: E402
from eco_hip.envs.utils import DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget  # noqa: E402

NAMES = ["scalars + state rows", "CSR row + field update", "flip, ballots, history", "reward, best, writes",
         "observation rows"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--n", type=int, default=200)
    args = ap.parse_args()
    B, n = args.envs, args.n
    dev = torch.device("cuda:0")
    store = GraphStore.random("ER", B, n, 0.15, seed=1234, device=dev)
    env = VecSpinSystem(store, B, 2 * n, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                        extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                        norm_rewards=True, basin_reward=1. / n)
    env.reset(graph_ids=np.arange(B), seed=1)
    g = torch.Generator(device=dev).manual_seed(7)
    f = _lib.lib.eco_debug_env_ts
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    for it in range(12):
        acts = torch.randint(0, n, (B,), generator=g, device=dev, dtype=torch.int32)
        env.step(acts)
        torch.cuda.synchronize()
    m = min(B, 16384)
    buf = (ctypes.c_ulonglong * (m * 8))()
    assert f(buf, m * 8) == 0
    ts = np.frombuffer(buf, dtype=np.uint64).reshape(m, 8)[:, :6].astype(np.int64)
    us = 10.0 / 1000.0  # 100 MHz ticks
    d = np.diff(ts, axis=1) * us
    t0 = ts[:, 0].min()
    print(f"env step ER-{n} x {B}: launch span {(ts[:, 5].max() - t0) * us:.1f} us; wave start spread "
          f"{(ts[:, 0].max() - t0) * us:.1f} us; mean wave life {(ts[:, 5] - ts[:, 0]).mean() * us:.1f} us "
          f"(p90 {np.percentile(ts[:, 5] - ts[:, 0], 90) * us:.1f})")
    for k, nm in enumerate(NAMES):
        print(f"  {nm:28s} {d[:, k].mean():7.2f} us (p90 {np.percentile(d[:, k], 90):7.2f})")
    hist = np.histogram((ts[:, 0] - t0) * us, bins=8)
    print("  wave starts (us):", [round(x, 1) for x in hist[1]], list(hist[0]))


if __name__ == "__main__":
    main()
