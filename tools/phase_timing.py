"""Per-phase timing of the MPNN forward/backward kernels (diagnostic, GPU only).

Loads eco_hip/libecohip_timing.so (`make -C eco-dqn_amd timing`: the same kernels with
wall_clock64() stamps at every block-wide barrier) and reports the mean duration of each
phase over all blocks of one launch, for the bench's M=2048 ER-200 minibatch shape.

usage: python tools/phase_timing.py [--batch 2048] [--n 200] [--p 0.15]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["ECO_HIP_LIB"] = os.environ.get("ECO_HIP_LIB") or os.path.join(ROOT, "eco-dqn_amd", "eco_hip", "libecohip_timing.so")
sys.path.insert(0, os.path.join(ROOT, "eco-dqn_amd"))

import torch  # noqa: E402

from eco_hip import _lib  # noqa: E402
from eco_hip.graphs import GraphStore  # noqa: E402
from eco_hip.networks.mpnn import MPNN  # noqa: E402

FWD = ["staging", "A: Z=Wx.x", "B: edge agg + Wf", "C: h0", "layer 0", "layer 1", "layer 2", "readout"]
BWD = ["staging", "readout bwd", "layer 2", "layer 1", "layer 0", "du0 + due + Wf^T", "dz gather + dwa"]


def stamps(nblk):
    if not hasattr(_lib.lib, "eco_debug_phase_ts"):
        return None
    buf = (ctypes.c_ulonglong * (nblk * 32))()
    _lib.lib.eco_debug_phase_ts.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    if _lib.lib.eco_debug_phase_ts(buf, nblk * 32):
        raise RuntimeError("eco_debug_phase_ts failed")
    return np.frombuffer(buf, dtype=np.uint64).reshape(nblk, 32).astype(np.int64)


def report(title, ts, idx, names):
    if ts is None:
        print(f"{title}: (no stamps in this build)")
        return
    d = np.diff(ts[:, idx], axis=1) * 10.0 / 1000.0  # 100 MHz ticks -> us
    span = (ts[:, idx[-1]].max() - ts[:, idx[0]].min()) * 10.0 / 1000.0
    print(f"{title}: launch span {span:.1f} us, mean block {d.sum(1).mean():.1f} us")
    for k, nm in enumerate(names):
        print(f"  {nm:22s} {d[:, k].mean():8.2f} us  (p90 {np.percentile(d[:, k], 90):8.2f})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--p", type=float, default=0.15, help="ER p, or BA m with --graph BA")
    ap.add_argument("--graph", default="ER", choices=["ER", "BA"])
    ap.add_argument("--paths", type=int, default=0, help="eco_set_kernel_paths mask (16: the 16-wave dense2 kernels)")
    args = ap.parse_args()
    _lib.lib.eco_set_kernel_paths(args.paths)
    dev = torch.device("cuda:0")
    B, N = args.batch, args.n
    store = GraphStore.generated(args.graph, B, N, args.p if args.graph == "ER" else int(args.p), seed=1, device=dev)
    gids = torch.arange(B, dtype=torch.int32, device=dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.zeros(B, N, 8)
    x[:, :, 0] = torch.randint(0, 2, (B, N), generator=g).float() * 2 - 1
    x[:, :, 1:7] = torch.rand(B, N, 6, generator=g)
    x = x.to(dev)
    net = MPNN(n_obs_in=7, device=dev)
    net.init_normal_(0.01, generator=torch.Generator(device="cpu").manual_seed(0))
    saved = torch.empty(MPNN.saved_bytes(N, B), dtype=torch.uint8, device=dev)
    gpb = 1 if N >= 208 else 208 // N
    nblk = (B + gpb - 1) // gpb
    for _ in range(3):
        net.forward_graphs(x, store, gids, norm_scope=_lib.ECO_NORM_PER_CALL)
    torch.cuda.synchronize()
    ts = stamps(nblk)
    # dense kernels for 224 < N <= 512 (eco_mpnn_dl.h): stamps 1..4 = staging | edge aggregation | Wf | h0
    dl = 224 < N <= 512 and args.graph in ("ER", "BA") and not os.environ.get("ECO_MPNN_NO_DL")
    fwd_names = (["staging", "edge agg (A+, A-)", "Wf", "h0"] + FWD[4:]) if dl else FWD
    report(f"forward (no save) B={B} N={N}", ts, list(range(0, 9)), fwd_names)
    if ts is not None and ts[:, 10].any():
        if dl:  # mpnn_forward_dl_kernel
            report("  layer 0 detail (wave 0)", ts, [4, 10, 11, 12, 13, 5],
                   ["lo planes + wait", "agg lo", "hi planes + agg hi", "message + update", "B_d wait"])
        elif os.environ.get("ECO_DENSE_V1"):
            report("  layer 0 detail (wave 0)", ts, [4, 10, 11, 12, 13, 14, 5],
                   ["weight staging", "MFMA half 1 issue", "gather", "MFMA half 2", "(drain)", "to barrier"])
        else:  # mpnn_forward_dense2_kernel / dense3 (wave 0's first tile)
            report("  layer 0 detail (wave 0)", ts, [4, 10, 11, 12, 13, 14, 5],
                   ["aggregation", "B1 wait", "message", "update", "h' planes", "B2 wait"])
    if ts is not None and ts[:, 9].any():  # dense3: the prologue in detail (wave 0)
        report("  prologue detail (wave 0)", ts, [0, 1, 9, 15, 2],
               ["staging loads", "phase A compute + planes", "Wf DMA wait", "barrier"])
    q = net.forward_graphs(x, store, gids, norm_scope=_lib.ECO_NORM_PER_CALL, saved=saved)
    torch.cuda.synchronize()
    report(f"forward (save)    B={B} N={N}", stamps(nblk), list(range(0, 9)), fwd_names)
    dq = torch.zeros_like(q)
    dq[torch.arange(B), torch.randint(0, N, (B,))] = 1e-3
    grad = torch.zeros_like(net.flat)
    net.backward_graphs(x, store, gids, saved, dq, grad)
    torch.cuda.synchronize()
    ts = stamps(nblk)
    report(f"backward          B={B} N={N}", ts, list(range(16, 24)), BWD)
    if ts is not None and ts[:, 29].any():  # mpnn_backward_dense3_kernel's readout
        report("  readout detail (wave 0)", ts, [17, 29, 30, 31, 18],
               ["DQ staging", "dq . h3 sums", "per-graph (wave 0)", "dh3 + DMA wait + pad"])
    if ts is not None and ts[:, 24].any():
        if dl:
            report("  layer 1 detail (wave 0)", ts, [19, 24, 20], ["Linears + lo planes", "barrier + agg lo/hi"])
        elif os.environ.get("ECO_DENSE_V1"):
            report("  layer 1 detail (wave 0)", ts, [19, 24, 25, 26, 27, 28, 29, 30, 20],
                   ["h,m loads + duu", "B0 wait", "Wu^T x2 + dum", "B1 wait", "dagg + G planes", "B2 wait",
                    "de + A.G", "B3 wait"])
        else:  # mpnn_backward_dense2_kernel
            report("  layer 1 detail (wave 0)", ts, [19, 24, 25, 26, 27, 28, 20],
                   ["duu, Wu^T x2, dum", "B0 wait (Wm^T DMA)", "stores, Wm^T x2, G planes", "B1 wait", "A.G",
                    "B2 wait"])


if __name__ == "__main__":
    main()
