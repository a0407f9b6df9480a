"""Device graph store: G graphs of N vertices as CSR (eco_graph_set, include/eco_hip.h).

Replaces the dense `GraphGenerator.get() -> ndarray[N,N] f64` adjacency that the
reference stacks under every observation (spinsystem.py:561-574): on the device a
graph is CSR with integer weights, shared by every episode that references its id.
Host-side construction is numpy (input preparation, not the hot path); the
normalisers (mlr, qn, lb, degrees) are computed on the device by
eco_graphs_prepare.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def _pack_edges(cols, weights):
    w = np.asarray(weights)
    if not np.all(np.equal(np.mod(w, 1), 0)) or w.min(initial=0) < -128 or w.max(initial=0) > 127:
        raise ValueError("eco_hip graphs take integer edge weights in [-128, 127] "
                         "(EdgeType.UNIFORM / DISCRETE); EdgeType.RANDOM is not supported on the device")
    return (np.asarray(cols, dtype=np.uint32) | ((w.astype(np.int64) & 0xFF).astype(np.uint32) << 24)).astype(np.uint32)


def dense_to_csr(matrices):
    """list of [N,N] symmetric zero-diagonal matrices -> (row_ptr [G][N+1], edge_base [G], edges)."""
    mats = [np.asarray(m) for m in matrices]
    n = mats[0].shape[0]
    row_ptr = np.zeros((len(mats), n + 1), dtype=np.int32)
    bases = np.zeros(len(mats), dtype=np.int64)
    chunks = []
    off = 0
    for g, m in enumerate(mats):
        if m.shape != (n, n):
            raise ValueError("all graphs in a store must have the same N")
        if np.any(np.diag(m) != 0):
            raise ValueError("adjacency must have a zero diagonal (src/envs/utils.py:198-199)")
        if not np.array_equal(m, m.T):
            raise ValueError("adjacency must be symmetric (unbiased MaxCut)")
        r, c = np.nonzero(m)
        row_ptr[g, 1:] = np.cumsum(np.bincount(r, minlength=n))
        bases[g] = off
        chunks.append(_pack_edges(c, m[r, c]))
        off += r.size
    edges = np.concatenate(chunks) if chunks else np.zeros(0, np.uint32)
    return row_ptr, bases, edges


def edges_to_csr(n, i, j, w):
    """One graph from an undirected edge list (each edge once, 0-based) -> (row_ptr [1][N+1], edge_base [1],
    edges): the CSR of the symmetric matrix load_graph builds (matrix[[i,j],[j,i]] = w), without the dense
    N x N array (GSet graphs, N = 800 .. 20,000).  A repeated pair keeps its last weight, as the reference."""
    i, j, w = (np.asarray(v, dtype=np.int64) for v in (i, j, w))
    if i.size and (min(i.min(), j.min()) < 0 or max(i.max(), j.max()) >= n):
        raise ValueError("edge endpoint out of range")
    if np.any(i == j):
        raise ValueError("self-loops are not allowed (zero diagonal)")
    key = np.minimum(i, j) * n + np.maximum(i, j)
    _, last = np.unique(key[::-1], return_index=True)   # last occurrence of every pair
    keep = np.sort(key.size - 1 - last)
    i, j, w = i[keep], j[keep], w[keep]
    nz = w != 0
    i, j, w = i[nz], j[nz], w[nz]
    r = np.concatenate([i, j])
    c = np.concatenate([j, i])
    ww = np.concatenate([w, w])
    order = np.lexsort((c, r))
    r, c, ww = r[order], c[order], ww[order]
    row_ptr = np.zeros((1, n + 1), dtype=np.int32)
    row_ptr[0, 1:] = np.cumsum(np.bincount(r, minlength=n))
    return row_ptr, np.zeros(1, dtype=np.int64), _pack_edges(c, ww)


def random_csr(kind, n_graphs, n, param, seed, weights="discrete", chunk=512):
    """Seeded synthetic graph pool built directly as CSR (no dense N x N per graph).
    kind 'ER': G(n, p=param); 'BA': preferential attachment with m=param.
    weights 'discrete' = fair +-1 per edge (EdgeType.DISCRETE), 'uniform' = 1."""
    rng = np.random.default_rng(seed)
    row_ptr = np.zeros((n_graphs, n + 1), dtype=np.int32)
    bases = np.zeros(n_graphs, dtype=np.int64)
    parts = []
    off = 0
    iu_all, ju_all = np.triu_indices(n, 1)
    for g0 in range(0, n_graphs, chunk):
        g1 = min(n_graphs, g0 + chunk)
        for g in range(g0, g1):
            if kind == "ER":
                keep = rng.random(iu_all.size) < param
                iu, ju = iu_all[keep], ju_all[keep]
            elif kind == "BA":
                iu, ju = _ba_edges(n, int(param), rng)
            else:
                raise ValueError(kind)
            w = (2 * rng.integers(0, 2, iu.size) - 1) if weights == "discrete" else np.ones(iu.size, np.int64)
            r = np.concatenate([iu, ju])
            c = np.concatenate([ju, iu])
            ww = np.concatenate([w, w])
            order = np.lexsort((c, r))
            r, c, ww = r[order], c[order], ww[order]
            row_ptr[g, 1:] = np.cumsum(np.bincount(r, minlength=n))
            bases[g] = off
            parts.append(_pack_edges(c, ww))
            off += r.size
    return row_ptr, bases, np.concatenate(parts)


def _ba_edges(n, m, rng):
    targets = list(range(m))
    repeated = []
    iu, ju = [], []
    for src in range(m, n):
        iu.extend(targets)
        ju.extend([src] * m)
        repeated.extend(targets)
        repeated.extend([src] * m)
        chosen = set()
        while len(chosen) < m:
            chosen.add(repeated[int(rng.integers(0, len(repeated)))])
        targets = sorted(chosen)
    return np.array(iu, dtype=np.int64), np.array(ju, dtype=np.int64)


def edge_cap(kind, n, param, slack_sd=10.0):
    """Edge-slot size per graph for on-device generation: exact for BA (2 m (N - m)),
    mean + slack_sd standard deviations for ER."""
    if kind == "BA":
        return 2 * int(param) * (n - int(param))
    pairs = n * (n - 1) / 2.0
    mean, sd = 2.0 * pairs * param, 2.0 * np.sqrt(pairs * param * (1 - param))
    return int(mean + slack_sd * sd + 64)


class GraphStore:
    """G graphs of N vertices resident on the device (eco_graph_set)."""

    def __init__(self, row_ptr, edge_base, edges, device="cuda", stream=None, unit_weights=None):
        dev = torch.device(device)
        self.device = dev
        if isinstance(row_ptr, torch.Tensor):
            self.row_ptr, self.edge_base, self.edges = row_ptr, edge_base, edges
            self.n_graphs, n1 = row_ptr.shape
        else:
            row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
            self.n_graphs, n1 = row_ptr.shape
            self.row_ptr = torch.from_numpy(row_ptr).to(dev)
            self.edge_base = torch.from_numpy(np.ascontiguousarray(edge_base, dtype=np.int64)).to(dev)
            e = np.ascontiguousarray(edges, dtype=np.uint32).view(np.int32)
            self.edges = torch.from_numpy(e if e.size else np.zeros(1, np.int32)).to(dev)
        self.n_spins = n1 - 1
        if self.n_spins > _lib.ECO_MAX_SPINS:
            raise ValueError(f"N={self.n_spins} exceeds ECO_MAX_SPINS={_lib.ECO_MAX_SPINS}")
        self.deg = torch.zeros(self.n_graphs, self.n_spins, dtype=torch.int32, device=dev)
        self.max_deg = torch.zeros(self.n_graphs, dtype=torch.int32, device=dev)
        self.meta = torch.zeros(self.n_graphs, 4, dtype=torch.float64, device=dev)
        self.valid = torch.zeros(self.n_graphs, dtype=torch.int32, device=dev)
        if unit_weights is None:  # every stored weight +-1: the dense-aggregation MPNN path applies
            w = (self.edges.view(torch.int32) >> 24).to(torch.int8)
            unit_weights = bool((w.abs() == 1).all().item()) if self.edges.numel() > 1 else True
        self.unit_weights = bool(unit_weights)
        # dense-MPNN bitmask operand, built by eco_graphs_prepare (one graph per workgroup sizes only)
        nb = _lib.lib.eco_graphs_adjbits_bytes(self.n_spins, self.n_graphs) if self.unit_weights else 0
        self.adjbits = torch.zeros(nb // 4, dtype=torch.int32, device=dev) if nb else None
        self.gs = _lib.GraphSet(self.n_graphs, self.n_spins, self.row_ptr.data_ptr(), self.edge_base.data_ptr(),
                                self.edges.data_ptr(), self.deg.data_ptr(), self.max_deg.data_ptr(),
                                self.meta.data_ptr(), self.valid.data_ptr(), int(self.unit_weights),
                                self.adjbits.data_ptr() if nb else None)
        _lib.check(_lib.lib.eco_graphs_prepare(ctypes.byref(self.gs), _lib.stream_ptr(stream)))

    @classmethod
    def slots(cls, n_graphs, n, cap, device="cuda"):
        """Empty store with fixed edge slots (edge_base[g] = g * cap) for eco_graphs_generate."""
        dev = torch.device(device)
        rp = torch.zeros(n_graphs, n + 1, dtype=torch.int32, device=dev)
        eb = torch.arange(n_graphs, dtype=torch.int64, device=dev) * int(cap)
        ed = torch.zeros(max(1, n_graphs * int(cap)), dtype=torch.int32, device=dev)
        st = cls(rp, eb, ed, device=dev, unit_weights=True)  # eco_graphs_generate writes +-1 / 1 weights
        st.cap = int(cap)
        return st

    @classmethod
    def generated(cls, kind, n_graphs, n, param, seed=0, weights="discrete", device="cuda"):
        """Pool of n_graphs ER(n, p=param) / BA(n, m=param) graphs generated on the device."""
        st = cls.slots(n_graphs, n, edge_cap(kind, n, param), device=device)
        st.generate(0, n_graphs, kind, param, seed, weights)
        return st

    def generate(self, first, count, kind, param, seed, weights="discrete", stream=None, check=True):
        """Regenerate graphs [first, first+count) in place on the device (eco_graphs_generate);
        check=True synchronises and raises on an edge-slot overflow."""
        if not hasattr(self, "cap"):
            raise ValueError("generate() needs a store created with GraphStore.slots()")
        ws = torch.empty(_lib.lib.eco_graphs_generate_workspace_bytes(self.n_spins, count), dtype=torch.uint8,
                         device=self.device)
        k = {"ER": _lib.ECO_GRAPH_ER, "BA": _lib.ECO_GRAPH_BA}[kind]
        _lib.check(_lib.lib.eco_graphs_generate(ctypes.byref(self.gs), first, count, k, float(param),
                                                int(weights == "discrete"), ctypes.c_uint64(seed), self.cap,
                                                _lib.ptr(ws), _lib.stream_ptr(stream)))
        if check:  # an edge-slot overflow leaves an empty graph and sets the device error word
            self.check_errors(stream)

    def check_errors(self, stream=None):
        """Synchronise `stream` and raise the first device-side error (eco_check_errors)."""
        _lib.check(_lib.lib.eco_check_errors(_lib.stream_ptr(stream)))

    @classmethod
    def from_dense(cls, matrices, device="cuda"):
        return cls(*dense_to_csr(matrices), device=device)

    @classmethod
    def from_edges(cls, n, i, j, w, device="cuda"):
        """Single-graph store from an undirected edge list (GSet .mc instances, load_gset)."""
        return cls(*edges_to_csr(n, i, j, w), device=device)

    @classmethod
    def random(cls, kind, n_graphs, n, param, seed=0, weights="discrete", device="cuda"):
        return cls(*random_csr(kind, n_graphs, n, param, seed, weights), device=device)

    def dense(self, g):
        """Host dense adjacency of graph g (for the reference-format observation)."""
        rp = self.row_ptr[g].cpu().numpy()
        b = int(self.edge_base[g].item())
        e = self.edges[b:b + int(rp[-1])].cpu().numpy().view(np.uint32)
        m = np.zeros((self.n_spins, self.n_spins))
        rows = np.repeat(np.arange(self.n_spins), np.diff(rp))
        m[rows, e & 0xFFFFFF] = ((e >> 24).astype(np.uint8)).view(np.int8)
        return m
