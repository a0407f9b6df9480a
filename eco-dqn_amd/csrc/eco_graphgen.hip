// On-device graph generation for training resets (reference:
// RandomErdosRenyiGraphGenerator / RandomBarabasiAlbertGraphGenerator, src/envs/utils.py:165-236,
// which draw a fresh networkx graph on the host for every episode).
//
// Graphs are written into fixed edge slots of a graph set (edge_base[g] .. + cap), so a
// pool can be regenerated in place, then eco_graphs_prepare computes the normalisers.
// ER: edge {i,j} present iff hash(seed, g, i, j) < p; the hash is symmetric by construction,
//     so each row is generated independently (wave per row: count pass, scan, ballot fill;
//     columns come out sorted).
// BA: preferential attachment exactly as networkx.barabasi_albert_graph (initial star of m
//     targets, repeated-nodes list, m distinct draws per new vertex); the process is
//     sequential per graph, so one wave owns one graph with its lists in LDS.
// Weights: +-1 fair per edge (EdgeType.DISCRETE, symmetric hash) or 1 (UNIFORM).
// Parity is distributional only (different RNG streams from numpy/networkx).
#include "eco_common.h"

namespace eco {

__device__ __forceinline__ uint32_t pair_key(int i, int j, int N) {
  const int a = min(i, j), b = max(i, j);
  return (uint32_t)a * (uint32_t)N + (uint32_t)b;
}
__device__ __forceinline__ bool er_edge(uint64_t seed, int g, int i, int j, int N, float p) {
  return i != j && u01(rng3(seed, (uint64_t)g, pair_key(i, j, N))) < p;
}
__device__ __forceinline__ int edge_sign(uint64_t seed, int g, int i, int j, int N, int discrete) {
  if (!discrete) return 1;
  return (rng3(seed ^ 0x5157A3C1ull, (uint64_t)g, pair_key(i, j, N)) >> 63) ? 1 : -1;
}

// pass 1: per-row degree (wave per row)
__global__ void er_count_kernel(int first, int count, int N, float p, uint64_t seed, int32_t* row_cnt) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long long)count * N) return;
  const int g = first + (int)(row / N);
  const int i = (int)(row % N);
  int c = 0;
  for (int j0 = 0; j0 < N; j0 += 64) {
    const int j = j0 + lane;
    c += __popcll(__ballot(j < N && er_edge(seed, g, i, j, N, p)));
  }
  if (lane == 0) row_cnt[row] = c;
}

// pass 2: per-graph exclusive scan into row_ptr (wave per graph); overflow -> error word
__global__ void er_scan_kernel(int first, int count, int N, const int32_t* row_cnt, int32_t* row_ptr, long long cap,
                               int32_t* err) {
  const int lane = threadIdx.x & 63;
  const int gi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gi >= count) return;
  const int g = first + gi;
  int32_t* rp = row_ptr + (size_t)g * (N + 1);
  const int32_t* rc = row_cnt + (size_t)gi * N;
  int total = 0;
  for (int i = lane; i < N; i += 64) total += rc[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
  if (total > cap) {  // overflow: leave an empty graph (valid = 0 after prepare) and report it
    for (int i = lane; i <= N; i += 64) rp[i] = 0;
    if (lane == 0) atomicCAS(err, 0, ECO_ERR_GRAPH);
    return;
  }
  int base = 0;
  if (lane == 0) rp[0] = 0;
  for (int i0 = 0; i0 < N; i0 += 64) {
    const int i = i0 + lane;
    int v = i < N ? rc[i] : 0;
    // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o, 64);
      if (lane >= o) v += u;
    }
    if (i < N) rp[i + 1] = base + v;
    base += __shfl(v, 63, 64);
  }
}

// pass 3: fill sorted columns (wave per row)
__global__ void er_fill_kernel(int first, int count, int N, float p, uint64_t seed, int discrete,
                               const int32_t* row_ptr, const int64_t* edge_base, uint32_t* edges, long long cap) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long long)count * N) return;
  const int g = first + (int)(row / N);
  const int i = (int)(row % N);
  const int32_t* rp = row_ptr + (size_t)g * (N + 1);
  if (rp[N] > cap) return;
  uint32_t* ed = edges + edge_base[g];
  int pos = rp[i];
  for (int j0 = 0; j0 < N; j0 += 64) {
    const int j = j0 + lane;
    const bool on = j < N && er_edge(seed, g, i, j, N, p);
    const uint64_t bal = __ballot(on);
    if (on) {
      const int k = __popcll(bal & ((1ull << lane) - 1ull));
      const int w = edge_sign(seed, g, i, j, N, discrete);
      ed[pos + k] = (uint32_t)j | ((uint32_t)(uint8_t)(int8_t)w << 24);
    }
    pos += __popcll(bal);
  }
}

// Barabasi-Albert (networkx.barabasi_albert_graph semantics), one wave per graph.
// LDS per wave: repeated list [2 m (N - m)] int32, edge list [(N - m) m] x2 int16, degree [N], fill cursor [N]
__global__ void ba_kernel(int first, int count, int N, int m, uint64_t seed, int discrete, int32_t* row_ptr,
                          const int64_t* edge_base, uint32_t* edges, long long cap, int32_t* err) {
  extern __shared__ int32_t sm[];
  const int lane = threadIdx.x;
  const int gi = blockIdx.x;
  if (gi >= count) return;
  const int g = first + gi;
  const int E = (N - m) * m;
  int32_t* rep = sm;                    // [2E]
  int32_t* es = rep + 2 * E;            // [E] source
  int32_t* et = es + E;                 // [E] target
  int32_t* deg = et + E;                // [N]
  int32_t* cur = deg + N;               // [N]
  for (int i = lane; i < N; i += 64) deg[i] = 0;
  if (lane == 0) {
    int nrep = 0, ne = 0;
    int targets[64];
    for (int k = 0; k < m; ++k) targets[k] = k;
    uint64_t ctr = 0;
    for (int src = m; src < N; ++src) {
      for (int k = 0; k < m; ++k) {
        es[ne] = src;
        et[ne] = targets[k];
        ++ne;
        rep[nrep++] = targets[k];
      }
      for (int k = 0; k < m; ++k) rep[nrep++] = src;
      // m distinct uniform draws from the repeated list
      int got = 0;
      while (got < m) {
        const int x = rep[(int)(rng3(seed, (uint64_t)g, ctr++) % (uint64_t)nrep)];
        bool dup = false;
        for (int k = 0; k < got; ++k) dup = dup || (targets[k] == x);
        if (!dup) targets[got++] = x;
      }
    }
  }
  __syncthreads();
  for (int e = lane; e < E; e += 64) {
    atomicAdd(&deg[es[e]], 1);
    atomicAdd(&deg[et[e]], 1);
  }
  __syncthreads();
  int32_t* rp = row_ptr + (size_t)g * (N + 1);
  __shared__ int overflow;
  if (lane == 0) {
    int s = 0;
    for (int i = 0; i < N; ++i) {
      cur[i] = s;
      s += deg[i];
    }
    overflow = s > cap;
    if (overflow) atomicCAS(err, 0, ECO_ERR_GRAPH);
  }
  __syncthreads();
  for (int i = lane; i <= N; i += 64)  // overflow: an empty graph (valid = 0 after prepare)
    rp[i] = overflow ? 0 : (i == 0 ? 0 : cur[i - 1] + deg[i - 1]);
  if (overflow) return;
  __syncthreads();
  uint32_t* ed = edges + edge_base[g];
  if (lane == 0) {  // deterministic fill order
    for (int e = 0; e < E; ++e) {
      const int a = es[e], b = et[e];
      const int w = edge_sign(seed, g, a, b, N, discrete);
      ed[cur[a]++] = (uint32_t)b | ((uint32_t)(uint8_t)(int8_t)w << 24);
      ed[cur[b]++] = (uint32_t)a | ((uint32_t)(uint8_t)(int8_t)w << 24);
    }
  }
  __syncthreads();
  // sort each row by column (insertion sort; rows are short except hubs)
  for (int i = lane; i < N; i += 64) {
    for (int q = rp[i] + 1; q < rp[i + 1]; ++q) {
      const uint32_t x = ed[q];
      int r = q - 1;
      while (r >= rp[i] && (ed[r] & 0xFFFFFFu) > (x & 0xFFFFFFu)) {
        ed[r + 1] = ed[r];
        --r;
      }
      ed[r + 1] = x;
    }
  }
}

}  // namespace eco

using namespace eco;

extern "C" int eco_graphs_generate(eco_graph_set* gs, int32_t first, int32_t count, int32_t kind, double param,
                                   int32_t discrete_weights, uint64_t seed, int64_t edge_cap, void* workspace,
                                   eco_stream_t stream) {
  if (!gs || !gs->row_ptr || !gs->edges || !gs->edge_base) return fail(ECO_ERR_ARG, "incomplete graph set");
  if (first < 0 || count < 1 || first + count > gs->n_graphs) return fail(ECO_ERR_ARG, "graph range out of set");
  const int N = gs->n_spins;
  hipStream_t st = (hipStream_t)stream;
  int32_t* err = err_word();  // read by eco_check_errors
  if (!err) return fail(ECO_ERR_HIP, "cannot allocate error word");
  if (!workspace) return fail(ECO_ERR_ARG, "null workspace (eco_graphs_generate_workspace_bytes)");
  int32_t* rp = const_cast<int32_t*>(gs->row_ptr);
  uint32_t* ed = const_cast<uint32_t*>(gs->edges);
  if (kind == ECO_GRAPH_ER) {
    if (!(param >= 0.0 && param <= 1.0)) return fail(ECO_ERR_ARG, "ER p must be in [0, 1]");
    int32_t* cnt = (int32_t*)((char*)workspace + 256);
    const long long rows = (long long)count * N;
    const int rblocks = (int)((rows + 3) / 4);
    er_count_kernel<<<rblocks, 256, 0, st>>>(first, count, N, (float)param, seed, cnt);
    er_scan_kernel<<<(count + 3) / 4, 256, 0, st>>>(first, count, N, cnt, rp, edge_cap, err);
    er_fill_kernel<<<rblocks, 256, 0, st>>>(first, count, N, (float)param, seed, discrete_weights, rp, gs->edge_base,
                                            ed, edge_cap);
  } else if (kind == ECO_GRAPH_BA) {
    const int m = (int)param;
    if (m < 1 || m >= N || m > 64) return fail(ECO_ERR_ARG, "BA m must be in [1, min(N-1, 64)]");
    const size_t E = (size_t)(N - m) * m;
    const size_t lds = (4 * E + 2 * (size_t)N) * sizeof(int32_t);
    if (lds > 160 * 1024) return fail(ECO_ERR_ARG, "BA graph too large for one workgroup's LDS");
    (void)hipFuncSetAttribute((const void*)ba_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    ba_kernel<<<count, 64, lds, st>>>(first, count, N, m, seed, discrete_weights, rp, gs->edge_base, ed, edge_cap,
                                      err);
  } else {
    return fail(ECO_ERR_ARG, "unknown graph kind");
  }
  int rc = check_launch("graphs_generate");
  if (rc) return rc;
  return graphs_prepare_range(gs, first, count, st);
}

extern "C" size_t eco_graphs_generate_workspace_bytes(int32_t n_spins, int32_t count) {
  return 256 + (size_t)n_spins * count * sizeof(int32_t);
}
