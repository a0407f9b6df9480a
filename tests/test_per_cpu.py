"""PrioritisedReplayBuffer (src/agents/dqn/utils.py:86-277): the oracle restatement and the native heap of
libecohip.so (eco_per_*, host-only calls, no GPU needed) replayed through the scripted call sequences the
reference itself was run through (tests/golden/make_per_golden.py -> per.npz).  Bars: heap layout (buffer
position and td error per heap position), partitions, ranks -> buffer positions and beta exact; float32
importance weights bitwise for torch's special-cased exponents (beta = 0.5: 1/sqrt) and within 2 ulp
otherwise (torch's vectorised powf is 1-ulp accurate, the restatements round correctly, and the
normalisation by the batch maximum can add one more)."""
import ctypes
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "eco-dqn_amd"))
sys.path.insert(0, REPO)

from oracle.per_oracle import PEROracle  # noqa: E402

GOLD = np.load(os.path.join(REPO, "tests", "golden", "per.npz"))
OP_ADD, OP_UPDATE, OP_SAMPLE, OP_REBALANCE = 0, 1, 2, 3


def ops(ci):
    """Yield the recorded calls of case ci: (op, n, arg_bp, arg_td, heap_bp, heap_td, beta, parts, ranks, s_bp,
    s_w, s_ids)."""
    g = {k[len(f"c{ci}_"):]: GOLD[k] for k in GOLD.files if k.startswith(f"c{ci}_")}
    offs = {}
    for k in ("arg_bp", "arg_td", "heap_bp", "heap_td", "parts", "ranks", "s_bp", "s_w", "s_ids"):
        mult = 2 if k == "parts" else 1
        offs[k] = np.concatenate([[0], np.cumsum(g[k + "_len"] * mult)])
    for i, op in enumerate(g["op"]):
        sl = {k: g[k][offs[k][i]:offs[k][i + 1]] for k in offs}
        yield (int(op), int(g["arg_n"][i]), sl["arg_bp"], sl["arg_td"], sl["heap_bp"], sl["heap_td"],
               float(g["beta"][i]), sl["parts"].reshape(-1, 2), sl["ranks"], sl["s_bp"], sl["s_w"], sl["s_ids"])


def case_params(ci):
    cap, anneal, _, _ = GOLD["cases"][ci]
    alpha, beta0 = GOLD["alpha_beta"][ci]
    return int(cap), float(alpha), float(beta0), int(anneal)


def close_f32(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return np.all(np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64)) <= 2)


def weights_ok(w, ref, beta):
    """bitwise where torch special-cases the exponent (-0.5 -> 1/sqrt, -1 -> reciprocal), else 2 ulp"""
    if np.float32(-beta) in (np.float32(-0.5), np.float32(-1.0)):
        return np.array_equal(np.asarray(w, np.float32).view(np.int32), np.asarray(ref, np.float32).view(np.int32))
    return close_f32(w, ref)


@pytest.mark.parametrize("ci", [0, 1, 2])
def test_oracle_matches_reference(ci):
    cap, alpha, beta0, anneal = case_params(ci)
    o = PEROracle(cap, alpha, beta0)
    o.configure_beta_anneal_time(anneal)
    n_samples = 0
    counter, newest = 0, {}
    for op, n, abp, atd, hbp, htd, beta, parts, ranks, sbp, sw, sids in ops(ci):
        if op == OP_ADD:
            for _ in range(n):
                counter += 1
                newest[o.add()] = counter
        elif op == OP_UPDATE:
            o.update_priorities(abp.tolist(), atd.tolist())
        elif op == OP_SAMPLE:
            r, bps, w = o.sample(n, ranks=ranks.tolist())
            assert [tuple(p) for p in o.partitions] == [tuple(p) for p in parts]
            assert bps == sbp.tolist()
            assert [newest[b] for b in bps] == sids.tolist()   # ring slot = buffer position - 1, newest add
            assert weights_ok(w, sw, beta), (beta, w, sw)
            n_samples += 1
        else:
            o.rebalance()
        b, t = o.heap()
        np.testing.assert_array_equal(b, hbp)
        np.testing.assert_array_equal(t, htd)
        assert o.beta == beta
    assert n_samples > 5


class NativePER:
    def __init__(self, cap, alpha, beta0):
        from eco_hip import _lib
        self.L = _lib
        self.h = _lib.lib.eco_per_create(cap, alpha, beta0)
        assert self.h

    def call(self, name, *a):
        self.L.check(getattr(self.L.lib, name)(self.h, *a))

    def heap(self):
        n = self.L.lib.eco_per_len(self.h)
        b = np.zeros(n, np.int32)
        t = np.zeros(n, np.float64)
        self.call("eco_per_heap", b.ctypes.data_as(ctypes.c_void_p), t.ctypes.data_as(ctypes.c_void_p))
        return b, t


@pytest.mark.parametrize("ci", [0, 1, 2])
def test_native_heap_matches_reference(ci):
    cap, alpha, beta0, anneal = case_params(ci)
    p = NativePER(cap, alpha, beta0)
    lib = p.L.lib
    p.call("eco_per_configure_beta_anneal_time", ctypes.c_double(anneal))
    for op, n, abp, atd, hbp, htd, beta, parts, ranks, sbp, sw, sids in ops(ci):
        if op == OP_ADD:
            out = np.zeros(n, np.int32)
            before = lib.eco_per_len(p.h)
            p.call("eco_per_add", n, out.ctypes.data_as(ctypes.c_void_p))
            assert before <= lib.eco_per_len(p.h)
        elif op == OP_UPDATE:
            b = np.ascontiguousarray(abp, np.int32)
            t = np.ascontiguousarray(atd, np.float64)
            p.call("eco_per_update_priorities", len(b), b.ctypes.data_as(ctypes.c_void_p), t.ctypes.data_as(ctypes.c_void_p))
        elif op == OP_SAMPLE:
            bounds = np.zeros(n + 1, np.int32)
            p.call("eco_per_sample_begin", n, bounds.ctypes.data_as(ctypes.c_void_p))
            np.testing.assert_array_equal(np.stack([bounds[:-1], bounds[1:]], 1), parts)
            rk = np.ascontiguousarray(ranks, np.int64)
            bps = np.zeros(n, np.int32)
            w = np.zeros(n, np.float32)
            rout = np.zeros(n, np.int64)
            p.call("eco_per_sample_finish", n, rk.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(0),
                   bps.ctypes.data_as(ctypes.c_void_p), w.ctypes.data_as(ctypes.c_void_p),
                   rout.ctypes.data_as(ctypes.c_void_p))
            np.testing.assert_array_equal(bps, sbp)
            np.testing.assert_array_equal(rout, ranks)
            assert weights_ok(w, sw, beta), (beta, w, sw)
            # the sampled transitions named their buffer position when added (ids = add counter); the ring
            # slot of a buffer position holds the newest add there
            assert len(sids) == n
        else:
            p.call("eco_per_rebalance")
        b, t = p.heap()
        np.testing.assert_array_equal(b, hbp)
        np.testing.assert_array_equal(t, htd)
        assert lib.eco_per_beta(p.h) == beta
    lib.eco_per_destroy(p.h)


def test_native_errors_follow_reference_exceptions():
    p = NativePER(8, 0.7, 0.5)
    with pytest.raises(KeyError):          # sample from an empty heap (priority_heap[rank] KeyError)
        p.call("eco_per_sample_begin", 2, None)
    out = np.zeros(5, np.int32)
    p.call("eco_per_add", 5, out.ctypes.data_as(ctypes.c_void_p))
    assert out.tolist() == [1, 2, 3, 4, 5]
    with pytest.raises(IndexError):        # rebalance before the heap is full (utils.py:196)
        p.call("eco_per_rebalance")
    bad = np.array([7], np.int32)
    td = np.array([0.5])
    with pytest.raises(KeyError):          # buffer2heap[buf_id] of a position never added (utils.py:236)
        p.call("eco_per_update_priorities", 1, bad.ctypes.data_as(ctypes.c_void_p), td.ctypes.data_as(ctypes.c_void_p))
    # native rank draws land inside their partitions and the weights are normalised to max 1
    bounds = np.zeros(3, np.int32)
    p.call("eco_per_sample_begin", 2, bounds.ctypes.data_as(ctypes.c_void_p))
    bps = np.zeros(2, np.int32)
    w = np.zeros(2, np.float32)
    rk = np.zeros(2, np.int64)
    p.call("eco_per_sample_finish", 2, None, ctypes.c_uint64(3), bps.ctypes.data_as(ctypes.c_void_p),
           w.ctypes.data_as(ctypes.c_void_p), rk.ctypes.data_as(ctypes.c_void_p))
    assert all(bounds[k] <= rk[k] < bounds[k + 1] for k in range(2))
    assert w.max() == 1.0
    p.L.lib.eco_per_destroy(p.h)
