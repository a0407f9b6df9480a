"""Exact MaxCut by exhaustive enumeration (TEST INFRASTRUCTURE ONLY: the optimum that training-quality
tests divide by; never shipped).

cut(s) = 1/4 sum_ij J_ij (1 - s_i s_j) (src/envs/utils.py:90-94, `calculate_cut`).  Spin 0 is fixed to +1
(a cut and its complement are equal), so 2^(N-1) assignments are scored in blocks of 2^16 with one
[block, N] x [N, N] product each.  N = 20 takes ~0.1 s per graph."""
import numpy as np


def max_cut(J, block_bits=16):
    """-> (optimal cut value, one optimal spin vector in {-1, +1}^N) for a symmetric zero-diagonal J."""
    J = np.asarray(J, dtype=np.float64)
    n = J.shape[0]
    if n > 26:
        raise ValueError("exhaustive enumeration is for N <= 26")
    total = J.sum()
    m = n - 1
    bits = np.arange(m, dtype=np.int64)
    step = 1 << min(block_bits, m)
    best, best_s = -np.inf, None
    for lo in range(0, 1 << m, step):
        idx = np.arange(lo, lo + step, dtype=np.int64)
        s = np.ones((step, n))
        s[:, 1:] = 1.0 - 2.0 * ((idx[:, None] >> bits) & 1)
        cut = 0.25 * (total - np.einsum("bi,bi->b", s @ J, s))
        k = int(np.argmax(cut))
        if cut[k] > best:
            best, best_s = float(cut[k]), s[k].copy()
    return best, best_s


def cut_value(J, s):
    J = np.asarray(J, dtype=np.float64)
    s = np.asarray(s, dtype=np.float64)
    return float(0.25 * (J.sum() - s @ J @ s))
