// Device-side helpers shared by the MPNN kernels (eco_mpnn.hip: CSR-gather forward/backward,
// eco_mpnn_dense.hip: dense-aggregation forward/backward).
#pragma once
#include "eco_mpnn.h"

namespace eco {

struct MpnnArgs {
  const float* P;
  eco_graph_set gs;
  const int32_t* gids;
  int B, N, gpb, nobs;
  int xw;                // floats per node row of x: 8, or 16 when nobs > 8
  const float* x;        // [B*N][xw]
  int norm_scope;
  const int* call_maxdeg;
  float* q;              // [B*N] or null
  float* sv;             // saved activations (training forward) or null
  int has_act;
  eco_act_config act;
  int32_t* actions;
  int32_t* err;          // device error word (eco_check_errors)
  // backward
  const float* dq;       // [B*N]
  float* gr;             // gradient workspace
};

__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }

// acc[nt] += sum_c A_c * W[nt*16 + (l&15)][16c + 4(l>>4) + 0..3] over NC chunks of 16 k, with the
// weight fragments of chunk c+1 loaded while chunk c's MFMAs run (one-chunk-ahead software
// pipeline: without it every weight load is followed by s_waitcnt vmcnt(0)).
// SW = false: acc[nt] = D[node][out] in the 16x16 C layout (row 4(l>>4)+r, col l&15).
// SW = true: the weight is the A operand and the node tile the B operand, D[out][node]: lane l holds
// node l&15, features 16nt + 4(l>>4) + r -- exactly the operand layout of `a`, so a Linear's output
// feeds the next Linear (or a row store) without a transpose.  Same products, same fma order.
template <int NT, int NC, bool SW = false>
__device__ __forceinline__ void mm_k(f32x4 (&acc)[NT], const float4 (&a)[NC], const float* __restrict__ W, int ldw,
                                     int lane) {
  const float* wp = W + (lane & 15) * ldw + 4 * (lane >> 4);
  float4 b[2][NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) b[0][nt] = *reinterpret_cast<const float4*>(wp + nt * 16 * ldw);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c + 1 < NC) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        b[(c + 1) & 1][nt] = *reinterpret_cast<const float4*>(wp + nt * 16 * ldw + 16 * (c + 1));
    }
    // kk outer, nt inner: consecutive MFMAs write different accumulators (no dependent-issue
    // stall); each accumulator still sums its k in the same order.
#define ECO_MM_STEP(K)                                                                           \
  _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                            \
    if constexpr (SW) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[c & 1][nt].K, a[c].K, acc[nt], 0, 0, 0); \
    else acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c].K, b[c & 1][nt].K, acc[nt], 0, 0, 0);            \
  }
    ECO_MM_STEP(x)
    ECO_MM_STEP(y)
    ECO_MM_STEP(z)
    ECO_MM_STEP(w)
#undef ECO_MM_STEP
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float4 f4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ float4 relu4(const f32x4& v) {
  return make_float4(fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f));
}

// forward LDS region after the weights: x rows (WLDS) or the readout scratch (weights from L2)
__host__ __device__ constexpr int fwd_mreg_floats(int rows_pad, int gpb, int nw, bool wlds) {
  return wlds ? rows_pad * 8 : (gpb < nw ? gpb * nw * 64 : 0) + ((gpb + 3) & ~3) + rows_pad;
}

// stage a rows x cols fp32 matrix (cols % 4 == 0) from global (row stride lds_) into LDS (row stride ldd)
template <int NTHREADS>
__device__ __forceinline__ void stage_rows(float* dst, int ldd, const float* __restrict__ src, int lds_, int rows,
                                           int cols) {
  const int per_row = cols >> 2;
  for (int i = threadIdx.x; i < rows * per_row; i += NTHREADS) {
    const int r = i / per_row, c = (i - r * per_row) * 4;
    *reinterpret_cast<float4*>(dst + r * ldd + c) = *reinterpret_cast<const float4*>(src + r * lds_ + c);
  }
}

// Per-row CSR info, staged in LDS once per block (instead of a dependent chain of global loads per
// tile and phase): edge start within the graph, row length and the 0->1 clamped norm
// (mpnn.py:36-37), packed as int2 {e0, len | norm << 16}; each graph's edge base and norm.max()
// (per-graph scope of mpnn.py:102) sit in small per-graph arrays next to it.
struct RowInfo {
  int e0, e1, norm;
};

__device__ __forceinline__ int2 pack_row_info(const MpnnArgs& a, int blk, int r, int rows_valid) {
  if (r >= rows_valid) return make_int2(0, 1 << 16);
  const int gl = r / a.N, v = r - gl * a.N;
  const int gid = a.gids[blk * a.gpb + gl];
  const int32_t* rp = a.gs.row_ptr + (size_t)gid * (a.N + 1);
  const int b = rp[v], e = rp[v + 1];
  const int nrm = max(a.gs.deg[(size_t)gid * a.N + v], 1);
  return make_int2(b, (e - b) | (nrm << 16));
}

__device__ __forceinline__ RowInfo row_info_packed(int2 p) { return RowInfo{p.x, p.x + (p.y & 0xFFFF), p.y >> 16}; }

__device__ __forceinline__ RowInfo row_info(const int2* RI, int r) {
  const int2 p = RI[r];
  return RowInfo{p.x, p.x + (p.y & 0xFFFF), p.y >> 16};
}

// Balanced tile schedule of the CSR-gather kernels, built by one wave once the row info RI is staged:
// SCH[v] = the 16-row tile that virtual slot v = w + ti * nw (wave w's ti-th tile) processes, or ntiles
// for an empty slot.  A tile's gathers run as long as its largest degree, and preferential-attachment
// graphs put their hubs in the first tiles; so the tiles are ranked by that cost (descending, index on
// ties) and the ranks dealt to the waves in a snake (ti even: rank ti*nw + w, odd: ti*nw + nw-1-w), which
// pairs each wave's heavy tile with light ones.  ntiles <= 64 and ntiles <= nw * maxt.
__device__ __forceinline__ void build_tile_schedule(int* SCH, const int2* RI, int ntiles, int nw, int maxt) {
  const int lane = threadIdx.x & 63;
  int cost = -1;
  if (lane < ntiles) {
    cost = 0;
    for (int i = 0; i < 16; ++i) cost = max(cost, RI[lane * 16 + i].y & 0xFFFF);
  }
  int rank = 0;
  for (int u = 0; u < ntiles; ++u) {
    const int cu = __shfl(cost, u, 64);
    rank += (cu > cost) || (cu == cost && u < lane);
  }
  for (int v = lane; v < nw * maxt; v += 64) SCH[v] = ntiles;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < ntiles) {
    const int ti = rank / nw, j = rank - ti * nw;
    SCH[((ti & 1) ? nw - 1 - j : j) + ti * nw] = lane;
  }
}

// Visit the packed edges [e0, e1): groups of 4 edge words, the next group's loads issued before
// the current group is consumed (one exposed load latency per 4 edges instead of per edge).
template <typename F>
__device__ __forceinline__ void for_edges(const uint32_t* __restrict__ edges, int e0, int e1, F&& f) {
  int q = e0;
  uint32_t cur[4], nxt[4];
  if (q + 4 <= e1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) cur[k] = edges[q + k];
  }
  while (q + 4 <= e1) {
    const bool more = q + 8 <= e1;
    if (more) {
#pragma unroll
      for (int k = 0; k < 4; ++k) nxt[k] = edges[q + 4 + k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) f(cur[k]);
    q += 4;
    if (more) {
#pragma unroll
      for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
    }
  }
  for (; q < e1; ++q) f(edges[q]);
}

// sum_j w_ij * S[j][16c + 4(l>>4) + 0..3] over the CSR row (S: LDS rows of the block, stride LDH)
__device__ __forceinline__ void gather_ri(const RowInfo& ri, const uint32_t* __restrict__ edges, const float* S,
                                          int rbase, int s4, float4 (&acc)[4]) {
  for_edges(edges, ri.e0, ri.e1, [&](uint32_t ex) {
    const float wv = (float)edge_w(ex);
    const float* hr = S + (rbase + edge_col(ex)) * LDH + 4 * s4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 hv = f4(hr + 16 * c);
      acc[c].x = fmaf(wv, hv.x, acc[c].x);
      acc[c].y = fmaf(wv, hv.y, acc[c].y);
      acc[c].z = fmaf(wv, hv.z, acc[c].z);
      acc[c].w = fmaf(wv, hv.w, acc[c].w);
    }
  });
}



// ReadoutLayer (mpnn.py:143-159) + epsilon-greedy act (dqn.py:453-465, :490-512) over a block of whole
// graphs whose final embeddings sit in LDS (Hs, row stride ldh).  Column sums: all waves on each
// graph when `split` (few graphs per block), else one wave per graph.  Scr: LDS scratch of
// readout_scratch_floats() floats.
__host__ __device__ constexpr int readout_scratch_floats(int rows_pad, int gpb, int nw, bool split) {
  return (split ? gpb * nw * 64 : 0) + ((gpb + 3) & ~3) + rows_pad;
}

template <int NW>
__device__ __forceinline__ void graph_act(const MpnnArgs& a, const float* Qb, int blk, int g_valid, size_t R0);

// VNW (>= NW, a multiple of it): the number of strided column-sum partials when `split` -- the summation order of a
// kernel with VNW waves, kept by a kernel with fewer (mpnn_forward_dense3_kernel: 8 waves, dense2's 16 partials).
template <bool SAVE, int NW, int VNW = NW>
__device__ __forceinline__ void readout_act(const MpnnArgs& a, const float* Hs, int ldh, float* Scr, bool split,
                                            int blk, int g_valid, int rows_valid, size_t R0, size_t RT) {
  static_assert(VNW % NW == 0, "virtual waves: a multiple of the waves");
  constexpr int NT = 64 * NW;
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int N = a.N;
  const float* P = a.P;
  // column sums: all waves on each graph when there are fewer graphs than waves, else one wave per graph
  float* Red = Scr;                                   // [gpb][VNW][64] column-sum partials (split)
  float* CG = Red + (split ? a.gpb * VNW * 64 : 0);  // [gpb] relu(p) . wr[:64]
  float* Qb = CG + ((a.gpb + 3) & ~3);               // [rows_pad] q values
  if (split) {
    for (int gl = 0; gl < g_valid; ++gl) {
      const float* hg = Hs + gl * N * ldh;
      for (int vw = w; vw < VNW; vw += NW) {
        float cs = 0.f;
        for (int v = vw; v < N; v += VNW) cs += hg[v * ldh + lane];
        Red[(gl * VNW + vw) * 64 + lane] = cs;
      }
    }
    __syncthreads();
  }
  for (int gl = w; gl < g_valid; gl += NW) {
    const int e = blk * a.gpb + gl;
    float cs = 0.f;
    if (split) {
#pragma unroll
      for (int k = 0; k < VNW; ++k) cs += Red[(gl * VNW + k) * 64 + lane];  // fixed order
    } else {
      const float* hg = Hs + gl * N * ldh;
      for (int v = 0; v < N; ++v) cs += hg[v * ldh + lane];
    }
    const float mean = cs / (float)N;
    const float* wp = P + PK_WP + lane * 64;
    float4 wr4[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) wr4[k] = f4(wp + 4 * k);
    float p = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      p = fmaf(wr4[k].x, __shfl(mean, 4 * k + 0, 64), p);
      p = fmaf(wr4[k].y, __shfl(mean, 4 * k + 1, 64), p);
      p = fmaf(wr4[k].z, __shfl(mean, 4 * k + 2, 64), p);
      p = fmaf(wr4[k].w, __shfl(mean, 4 * k + 3, 64), p);
    }
    if (SAVE) {
      a.sv[(size_t)SV_NODE_TENSORS * RT * 64 + (size_t)e * 64 + lane] = mean;
      a.sv[(size_t)SV_NODE_TENSORS * RT * 64 + (size_t)a.B * 64 + (size_t)e * 64 + lane] = p;
    }
    const float cg = wave_sum_f(relu(p) * P[PK_WR + lane]);
    if (lane == 0) CG[gl] = cg;
  }
  __syncthreads();
  const float br = P[PK_BR];
  for (int r = threadIdx.x; r < rows_valid; r += NT) {
    const float* hr = Hs + r * ldh;
    float ql = 0.f;
#pragma unroll 4
    for (int f = 0; f < 64; f += 4) {
      const float4 hv = f4(hr + f);
      ql = fmaf(hv.x, P[PK_WR + 64 + f], ql);
      ql = fmaf(hv.y, P[PK_WR + 65 + f], ql);
      ql = fmaf(hv.z, P[PK_WR + 66 + f], ql);
      ql = fmaf(hv.w, P[PK_WR + 67 + f], ql);
    }
    const float qv = CG[r / N] + ql + br;
    Qb[r] = qv;
    if (a.q) a.q[R0 + r] = qv;
  }
  if (!a.has_act) return;
  __syncthreads();
  graph_act<NW>(a, Qb, blk, g_valid, R0);
}

// epsilon-greedy act (dqn.py:453-465, :490-512) of the block's graphs from their q values in LDS (Qb [rows]):
// wave w handles graphs w, w + NW, ...
template <int NW>
__device__ __forceinline__ void graph_act(const MpnnArgs& a, const float* Qb, int blk, int g_valid, size_t R0) {
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int N = a.N;
  for (int gl = w; gl < g_valid; gl += NW) {
    const int e = blk * a.gpb + gl;
    float bestq = -INFINITY;
    int besti = 0x7fffffff;
    int n_allowed = 0;
    for (int v0 = 0; v0 < N; v0 += 64) {
      const int v = v0 + lane;
      bool allowed = false;
      float qv = -INFINITY;
      if (v < N) {
        qv = Qb[gl * N + v];
        allowed = a.act.reversible || (a.x[(R0 + gl * N + v) * a.xw] == a.act.allowed_value);
      }
      n_allowed += __popcll(__ballot(allowed));
      if (allowed && (qv > bestq || (qv == bestq && v < besti))) { bestq = qv; besti = v; }
    }
    // first index of the max (torch argmax)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float oq = __shfl_xor(bestq, o, 64);
      const int oi = __shfl_xor(besti, o, 64);
      if (oq > bestq || (oq == bestq && oi < besti)) { bestq = oq; besti = oi; }
    }
    // no allowed vertex (irreversible episode with every spin flipped): the reference's
    // masked_fill(-10000).argmax over an all-masked row returns index 0 (dqn.py:416-428, :505-511)
    int action = besti == 0x7fffffff ? 0 : besti;
    const uint64_t r0 = rng3(a.act.seed, a.act.counter, (uint64_t)e);
    if (u01(r0) < a.act.epsilon && n_allowed > 0) {  // random.uniform(0,1) >= eps -> greedy
      const uint64_t r1 = rng3(a.act.seed ^ 0xA5A5A5A5ull, a.act.counter, (uint64_t)e);
      int k = (int)(r1 % (uint64_t)n_allowed);
      if (a.act.reversible) {
        action = k;
      } else {
        action = -1;  // k-th allowed vertex
        for (int v0 = 0; v0 < N && action < 0; v0 += 64) {
          const int v = v0 + lane;
          const bool al = v < N && a.x[(R0 + gl * N + v) * a.xw] == a.act.allowed_value;
          const uint64_t bal = __ballot(al);
          const int c = __popcll(bal);
          if (k < c) {
            uint64_t b = bal;
            for (int i = 0; i < k; ++i) b &= b - 1;
            action = v0 + __ffsll((long long)b) - 1;
          } else {
            k -= c;
          }
        }
      }
    }
    if (lane == 0) a.actions[e] = action;
  }
}

}  // namespace eco
