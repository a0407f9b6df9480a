// MPNN forward for many episodes on ONE shared large graph (N > 512: GSet G22 best-cut search,
// configs[4]; src/networks/mpnn.py:40-159 batched as in experiments/utils.py:154-187).
//
// The per-episode large kernel (mpnn_forward_large_kernel) gathers a 256-B embedding row per edge per
// episode from that episode's private rows: 4 x nnz x 256 B per episode, ~41 GB per 1024-episode call,
// served by HBM.  Here every buffer is NODE-major, [node][episode][64] fp32, so one wave tile = one node
// x 16 episodes (the 16 rows of the MFMA node operand) and one neighbour's contribution to the tile is
// one contiguous 4-KB row block.  The aggregation A.[H_1 ... H_B] reads each neighbour block once per
// 16 episodes, and the episode slices are dealt so that all workgroups of one group (one per XCD: block
// b works for group b % 8) sweep the nodes of the same 16-episode slice together: the slice's H
// (N x 4 KB = 8 MB at G22) is what the gathers of that XCD re-read, from L2 / the Infinity Cache, while
// HBM sees each H row written once and read about once per layer.
//
// Phases (one launch each, the layer weights staged in LDS by LDS-DMA once per persistent workgroup):
//   prep:    U = relu(Wx.x + w_a), V = relu(Wx.x - w_a) and h0 = relu(W0.x) per node and episode
//   edge:    e = relu(Wf.[(A+.U + A-.V) / deg, deg / norm.max()])   (mpnn.py:89-104, +-1 weights)
//   layers:  agg = A.h / deg, m = relu(Wm.[agg, e]), h' = relu(Wu.[h, m])  (mpnn.py:114-120, x3)
//            the last layer writes no h3: it emits q_local = Wr[64:].h3 per node and episode and the
//            per-episode column sums of h3 (fixed-order partials per workgroup)
//   readout: mean -> p = Wp.mean -> q = relu(p).Wr[:64] + q_local + b, fused epsilon-greedy act
//            (mpnn.py:143-159, dqn.py:453-465, :490-512)
// Linears: the six-product bf16x3 MFMAs of the dense kernels (f32-accurate).  Integer weights must be
// +-1 (the edge phase reads U or V per edge); other graphs take mpnn_forward_large_kernel.
#pragma once
#include "eco_mpnn_dense.h"

namespace eco {

constexpr int SH_EPS = 16;     // episodes per wave tile
constexpr int SH_NW = 8;       // waves per workgroup
constexpr int SH_GROUPS = 8;   // episode-slice groups: one per XCD (block b -> group b % 8)
constexpr int SH_TILE = SH_EPS * 64;  // floats of one node's 16-episode row block

struct SharedBufs {
  float* U;     // [N][Epad][64]
  float* V;
  float* HA;
  float* HB;
  float* EB;
  float* part;  // [S][nlb][16][64] column-sum partials of h3
  float* ql;    // [Epad][N] Wr[64:] . h3
  int Epad, S, nlb;
};

inline int shared_grid() {  // persistent workgroups: one per CU, a multiple of the group count
  static const int g = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                               hipSuccess || n < SH_GROUPS)
      n = 256;
    return (n / SH_GROUPS) * SH_GROUPS;
  }();
  return g;
}

inline size_t shared_ws_bytes(int N, int B) {
  const size_t S = ((size_t)B + SH_EPS - 1) / SH_EPS, Epad = S * SH_EPS;
  const size_t nlb = shared_grid() / SH_GROUPS;
  return (5 * (size_t)N * Epad * 64 + S * nlb * SH_TILE + Epad * (size_t)N) * sizeof(float);
}

inline SharedBufs shared_carve(float* base, int N, int B) {
  SharedBufs sb;
  sb.S = (B + SH_EPS - 1) / SH_EPS;
  sb.Epad = sb.S * SH_EPS;
  sb.nlb = shared_grid() / SH_GROUPS;
  const size_t T = (size_t)N * sb.Epad * 64;
  sb.U = base;
  sb.V = sb.U + T;
  sb.HA = sb.V + T;
  sb.HB = sb.HA + T;
  sb.EB = sb.HB + T;
  sb.part = sb.EB + T;
  sb.ql = sb.part + (size_t)sb.S * sb.nlb * SH_TILE;
  return sb;
}

// mm_bf3 over LDS fragments with one output tile's fragments in flight at a time (the shared-graph layer
// runs four Linears back to back: unbounded, the compiler hoists all 96 fragment reads and spills)
__device__ __forceinline__ void mm_bf3_seq(f32x4 (&acc)[4], const float4 (&x)[4], const uint16_t* WH, int lane) {
  const uint16_t* wl = WH + lane * 8;
#pragma unroll
  for (int kc2 = 0; kc2 < 2; ++kc2) {
    bf16x8 x1, x2, x3;
    split_frag(x[2 * kc2], x[2 * kc2 + 1], x1, x2, x3);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(wl + ((0 * 4 + nt) * 2 + kc2) * BF_FRAG);
      const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(wl + ((1 * 4 + nt) * 2 + kc2) * BF_FRAG);
      const bf16x8 w3 = *reinterpret_cast<const bf16x8*>(wl + ((2 * 4 + nt) * 2 + kc2) * BF_FRAG);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3, x1, acc[nt], 0, 0, 0);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, x2, acc[nt], 0, 0, 0);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x3, acc[nt], 0, 0, 0);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, x1, acc[nt], 0, 0, 0);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x2, acc[nt], 0, 0, 0);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x1, acc[nt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// U, V, h0 rows: thread (episode row er, feature quad q) of node blockIdx.x, episodes 16 blockIdx.y ..
// (16 threads write one 256-B row).  Same arithmetic as the phase-A / phase-C expressions of the dense
// kernel; rows of padding episodes are zero.
__global__ __launch_bounds__(256) void shared_prep_kernel(MpnnArgs a, SharedBufs sb) {
  const int n = blockIdx.x;
  const int er = threadIdx.x >> 4, q = threadIdx.x & 15;
  const int e = blockIdx.y * SH_EPS + er;
  if (e >= sb.Epad) return;
  const bool valid = e < a.B;
  float4 xa = zero4(), xb = zero4();
  if (valid) {
    xa = f4(a.x + ((size_t)e * a.N + n) * 8);
    xb = f4(a.x + ((size_t)e * a.N + n) * 8 + 4);
  }
  const float* P = a.P;
  float u[4], v[4], h[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = 4 * q + i;
    const float* wx = P + PK_WX + f * 8;
    const float z = wx[0] * xa.x + wx[1] * xa.y + wx[2] * xa.z + wx[3] * xa.w + wx[4] * xb.x + wx[5] * xb.y +
                    wx[6] * xb.z + wx[7] * xb.w;
    const float* w0 = P + PK_W0 + f * 8;
    const float h0 = w0[0] * xa.x + w0[1] * xa.y + w0[2] * xa.z + w0[3] * xa.w + w0[4] * xb.x + w0[5] * xb.y +
                     w0[6] * xb.z + w0[7] * xb.w;
    u[i] = valid ? relu(fmaf(1.f, P[PK_WA + f], z)) : 0.f;
    v[i] = valid ? relu(fmaf(-1.f, P[PK_WA + f], z)) : 0.f;
    h[i] = valid ? relu(h0) : 0.f;
  }
  const size_t o = ((size_t)n * sb.Epad + e) * 64 + 4 * q;
  st4(sb.U + o, make_float4(u[0], u[1], u[2], u[3]));
  st4(sb.V + o, make_float4(v[0], v[1], v[2], v[3]));
  st4(sb.HA + o, make_float4(h[0], h[1], h[2], h[3]));
}

// PHASE 0: edge embedding -> EB; 1: update layer Hc -> Hn; 2: last update layer -> q_local + column sums.
template <int PHASE>
__global__ __launch_bounds__(64 * SH_NW, 1) void shared_layer_kernel(MpnnArgs a, SharedBufs sb, int layer,
                                                                     const float* Hc, float* Hn) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  uint16_t* WL = reinterpret_cast<uint16_t*>(lds);  // Wf (24 fragments) or Wm, Wu (96 fragments)
  float* RED = lds + (96 * BF_FRAG) / 2;            // [SH_NW][16][64] column sums (PHASE 2)
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int c16 = lane & 15, s4 = lane >> 4;
  const uint16_t* PB = reinterpret_cast<const uint16_t*>(a.P + PK_BF);
  if (PHASE == 0) glds_frags<SH_NW>(WL, PB + BF_WF, 24, w, lane);
  else glds_frags<SH_NW>(WL, PB + BF_LAYER + layer * BF_LAYER_STRIDE, 96, w, lane);
  const int N = a.N;
  const int gid = a.gids[0];
  const int32_t* rp = a.gs.row_ptr + (size_t)gid * (N + 1);
  const uint32_t* __restrict__ eg = a.gs.edges + a.gs.edge_base[gid];
  const int32_t* degp = a.gs.deg + (size_t)gid * N;
  const int grp = blockIdx.x % SH_GROUPS, lb = blockIdx.x / SH_GROUPS;
  const int nlb = gridDim.x / SH_GROUPS;
  const float* P = a.P;
  const float md = PHASE == 0 ? (float)(a.norm_scope == ECO_NORM_PER_CALL ? *a.call_maxdeg : a.gs.max_deg[gid]) : 1.f;
  const size_t ld = (size_t)sb.Epad * 64;  // floats per node row block of all episodes
  glds_wait();
  __syncthreads();
  for (int s = grp; s < sb.S; s += SH_GROUPS) {
    const int ep = s * SH_EPS + c16;
    const bool evalid = ep < a.B;
    const size_t co = (size_t)ep * 64 + 4 * s4;  // this lane's offset inside a node row block
    float4 col[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) col[c] = zero4();
    for (int n = lb * SH_NW + w; n < N; n += nlb * SH_NW) {
      const int e0 = rp[n], e1 = rp[n + 1];
      const float nf = (float)max(degp[n], 1);
      float4 acc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = zero4();
      // gather: 4 neighbours' row blocks in flight, accumulated in CSR order
      int q = e0;
      for (; q + 4 <= e1; q += 4) {
        uint32_t ex[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) ex[k] = eg[q + k];
        float4 r[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int wv = edge_w(ex[k]);
          const float* src = (PHASE == 0 ? (wv > 0 ? sb.U : sb.V) : Hc) + (size_t)edge_col(ex[k]) * ld + co;
#pragma unroll
          for (int c = 0; c < 4; ++c) r[k][c] = f4(src + 16 * c);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float wv = (float)edge_w(ex[k]);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (PHASE == 0) {
              acc[c].x += r[k][c].x; acc[c].y += r[k][c].y; acc[c].z += r[k][c].z; acc[c].w += r[k][c].w;
            } else {
              acc[c].x = fmaf(wv, r[k][c].x, acc[c].x); acc[c].y = fmaf(wv, r[k][c].y, acc[c].y);
              acc[c].z = fmaf(wv, r[k][c].z, acc[c].z); acc[c].w = fmaf(wv, r[k][c].w, acc[c].w);
            }
          }
        }
      }
      for (; q < e1; ++q) {
        const uint32_t ex = eg[q];
        const int wv = edge_w(ex);
        const float* src = (PHASE == 0 ? (wv > 0 ? sb.U : sb.V) : Hc) + (size_t)edge_col(ex) * ld + co;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 rv = f4(src + 16 * c);
          if (PHASE == 0) {
            acc[c].x += rv.x; acc[c].y += rv.y; acc[c].z += rv.z; acc[c].w += rv.w;
          } else {
            const float fw = (float)wv;
            acc[c].x = fmaf(fw, rv.x, acc[c].x); acc[c].y = fmaf(fw, rv.y, acc[c].y);
            acc[c].z = fmaf(fw, rv.z, acc[c].z); acc[c].w = fmaf(fw, rv.w, acc[c].w);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c].x = acc[c].x / nf; acc[c].y = acc[c].y / nf; acc[c].z = acc[c].z / nf; acc[c].w = acc[c].w / nf;
      }
      const size_t ro = (size_t)n * ld + co;  // this lane's row (node n, episode ep)
      if (PHASE == 0) {
        if (s4 == 3) acc[3].w = nf / md;  // feature 63 = norm / norm.max() (mpnn.py:102)
        f32x4 d[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        mm_bf3_seq(d, acc, WL, lane);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) st4(sb.EB + ro + 16 * nt, evalid ? relu4(d[nt]) : zero4());
      } else {
        float4 ev[4], hc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          ev[c] = f4(sb.EB + ro + 16 * c);
          hc[c] = f4(Hc + ro + 16 * c);
        }
        f32x4 d[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        mm_bf3_seq(d, acc, WL, lane);               // message = relu(Wm . [agg, e])
        mm_bf3_seq(d, ev, WL + BF_HALF, lane);
        float4 mr[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) mr[c] = relu4(d[c]);
        f32x4 hn[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) hn[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        mm_bf3_seq(hn, hc, WL + 2 * BF_HALF, lane);  // h' = relu(Wu . [h, m])
        mm_bf3_seq(hn, mr, WL + 3 * BF_HALF, lane);
        if (PHASE == 1) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) st4(Hn + ro + 16 * nt, evalid ? relu4(hn[nt]) : zero4());
        } else {
          float qp = 0.f;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const float4 h3 = evalid ? relu4(hn[nt]) : zero4();
            const int f = 16 * nt + 4 * s4;
            qp = fmaf(h3.x, P[PK_WR + 64 + f], qp);
            qp = fmaf(h3.y, P[PK_WR + 65 + f], qp);
            qp = fmaf(h3.z, P[PK_WR + 66 + f], qp);
            qp = fmaf(h3.w, P[PK_WR + 67 + f], qp);
            col[nt].x += h3.x; col[nt].y += h3.y; col[nt].z += h3.z; col[nt].w += h3.w;
          }
          qp += __shfl_xor(qp, 16, 64);
          qp += __shfl_xor(qp, 32, 64);
          if (s4 == 0 && evalid) sb.ql[(size_t)ep * N + n] = qp;
        }
      }
    }
    if (PHASE == 2) {  // per-workgroup column sums of this slice, waves combined in a fixed order
#pragma unroll
      for (int c = 0; c < 4; ++c) st4(RED + (w * SH_EPS + c16) * 64 + 16 * c + 4 * s4, col[c]);
      __syncthreads();
      for (int i = threadIdx.x; i < SH_TILE; i += 64 * SH_NW) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < SH_NW; ++k) t += RED[k * SH_TILE + i];
        sb.part[((size_t)s * nlb + lb) * SH_TILE + i] = t;
      }
      __syncthreads();
    }
  }
}

// ReadoutLayer (mpnn.py:143-159) + epsilon-greedy act, one wave per episode: column sums from the
// partials (fixed order), p = Wp . mean, q = relu(p) . Wr[:64] + q_local + b, then the act of readout_act.
__global__ __launch_bounds__(64) void shared_readout_kernel(MpnnArgs a, SharedBufs sb) {
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = a.N;
  const float* P = a.P;
  const int s = e / SH_EPS, er = e % SH_EPS;
  float cs = 0.f;
  for (int k = 0; k < sb.nlb; ++k) cs += sb.part[((size_t)s * sb.nlb + k) * SH_TILE + er * 64 + lane];
  const float mean = cs / (float)N;
  const float* wp = P + PK_WP + lane * 64;
  float p = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float4 wr4 = f4(wp + 4 * k);
    p = fmaf(wr4.x, __shfl(mean, 4 * k + 0, 64), p);
    p = fmaf(wr4.y, __shfl(mean, 4 * k + 1, 64), p);
    p = fmaf(wr4.z, __shfl(mean, 4 * k + 2, 64), p);
    p = fmaf(wr4.w, __shfl(mean, 4 * k + 3, 64), p);
  }
  const float cg = wave_sum_f(relu(p) * P[PK_WR + lane]);
  const float br = P[PK_BR];
  const float* qloc = sb.ql + (size_t)e * N;
  const float* xe = a.x + (size_t)e * N * a.xw;
  float bestq = -INFINITY;
  int besti = 0x7fffffff;
  int n_allowed = 0;
  for (int v0 = 0; v0 < N; v0 += 64) {
    const int v = v0 + lane;
    bool allowed = false;
    float qv = -INFINITY;
    if (v < N) {
      qv = cg + qloc[v] + br;
      if (a.q) a.q[(size_t)e * N + v] = qv;
      allowed = a.has_act && (a.act.reversible || xe[(size_t)v * a.xw] == a.act.allowed_value);
    }
    n_allowed += __popcll(__ballot(allowed));
    if (allowed && (qv > bestq || (qv == bestq && v < besti))) { bestq = qv; besti = v; }
  }
  if (!a.has_act) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float oq = __shfl_xor(bestq, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (oq > bestq || (oq == bestq && oi < besti)) { bestq = oq; besti = oi; }
  }
  int action = besti == 0x7fffffff ? 0 : besti;  // no allowed vertex: argmax of an all-masked row is 0
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
        const bool al = v < N && xe[(size_t)v * a.xw] == a.act.allowed_value;
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

static int mpnn_forward_shared_launch(const MpnnArgs& a, void* workspace, hipStream_t st) {
  SharedBufs sb = shared_carve((float*)((char*)workspace + 256), a.N, a.B);
  shared_prep_kernel<<<dim3(a.N, sb.S), 256, 0, st>>>(a, sb);
  const int grid = shared_grid();
  const size_t lds_edge = 24 * BF_FRAG * 2, lds_layer = 96 * BF_FRAG * 2,
               lds_last = lds_layer + (size_t)SH_NW * SH_TILE * sizeof(float);
  (void)hipFuncSetAttribute((const void*)shared_layer_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_edge);
  (void)hipFuncSetAttribute((const void*)shared_layer_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_layer);
  (void)hipFuncSetAttribute((const void*)shared_layer_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_last);
  shared_layer_kernel<0><<<grid, 64 * SH_NW, lds_edge, st>>>(a, sb, 0, nullptr, nullptr);
  shared_layer_kernel<1><<<grid, 64 * SH_NW, lds_layer, st>>>(a, sb, 0, sb.HA, sb.HB);
  shared_layer_kernel<1><<<grid, 64 * SH_NW, lds_layer, st>>>(a, sb, 1, sb.HB, sb.HA);
  shared_layer_kernel<2><<<grid, 64 * SH_NW, lds_last, st>>>(a, sb, 2, sb.HA, nullptr);
  shared_readout_kernel<<<a.B, 64, 0, st>>>(a, sb);
  return check_launch("mpnn_forward_shared");
}

}  // namespace eco
