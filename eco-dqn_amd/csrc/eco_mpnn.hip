// MPNN Q-network forward (src/networks/mpnn.py) fused per graph block on gfx950,
// with the epsilon-greedy act (dqn.py:453-465, :490-512) fused into the readout.
//
// One 256-thread workgroup (4 waves) owns a block of whole graphs (graphs_per_block
// = max(1, 256/N)); the block's node embeddings H [rows][64] fp32 live in LDS for
// the whole forward.  Every stage runs on the same layout:
//   * message aggregation (A.H / deg and the edge embedding) is a sparse gather over
//     the CSR rows from LDS, accumulated DIRECTLY in the MFMA A-operand layout (lane l:
//     node l&15, features 16c + 4(l>>4) + 0..3), so no transpose is needed;
//   * every per-node Linear (128->64, 64->64) is v_mfma_f32_16x16x4_f32 (exact f32,
//     no TF32 on gfx950) with the k index permuted so that both operands are single
//     16-byte loads: MFMA kk of a 16-wide k chunk takes k = 16c + 4(l>>4) + kk;
//   * the edge layer never builds the [N,N,63] edge tensor (mpnn.py:90-100): with
//     Z = Wx.x per node in LDS, relu(We.[A_ij, x_j]) = relu(A_ij*w_a + Z_j) per edge.
#include "eco_common.h"

namespace eco {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- packed parameter image (floats) ----
constexpr int PK_W0 = 0;                   // [64][8]  node_init_embedding (cols >= n_obs zero)
constexpr int PK_WX = 512;                 // [64][8]  edge_embedding_NN.weight[:, 1:] (row 63 zero)
constexpr int PK_WA = 1024;                // [64]     edge_embedding_NN.weight[:, 0]  ([63] = 0)
constexpr int PK_WF = 1088;                // [64][64] edge_feature_NN
constexpr int PK_LAYER = 5184;             // + l*16384: message [64][128], +8192: update [64][128]
constexpr int PK_WP = PK_LAYER + 3 * 16384;  // [64][64] layer_pooled
constexpr int PK_WR = PK_WP + 4096;        // [128] layers_readout.0.weight
constexpr int PK_BR = PK_WR + 128;         // [1]   layers_readout.0.bias
constexpr int PK_TOTAL = PK_BR + 64;

constexpr int LDH = 68;   // LDS row stride (floats) of node-embedding tiles: 16 rows -> distinct bank quads
constexpr int NWAVE = 4;
constexpr int TPB = 64 * NWAVE;

__host__ __device__ inline int flat_count(int nobs) { return 64 * nobs + 63 * (1 + nobs) + 4096 + 6 * 8192 + 4096 + 128 + 1; }

__global__ void pack_kernel(const float* __restrict__ f, int nobs, float* __restrict__ p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= PK_TOTAL) return;
  const int oW0 = 0, oWe = 64 * nobs, oWf = oWe + 63 * (1 + nobs), oL = oWf + 4096, oWp = oL + 6 * 8192;
  const int oWr = oWp + 4096, oBr = oWr + 128;
  float v = 0.f;
  if (i < PK_WX) {
    const int r = i >> 3, c = i & 7;
    v = c < nobs ? f[oW0 + r * nobs + c] : 0.f;
  } else if (i < PK_WA) {
    const int r = (i - PK_WX) >> 3, c = (i - PK_WX) & 7;
    v = (r < 63 && c < nobs) ? f[oWe + r * (1 + nobs) + 1 + c] : 0.f;
  } else if (i < PK_WF) {
    const int r = i - PK_WA;
    v = r < 63 ? f[oWe + r * (1 + nobs)] : 0.f;
  } else if (i < PK_LAYER) {
    v = f[oWf + (i - PK_WF)];
  } else if (i < PK_WP) {
    v = f[oL + (i - PK_LAYER)];  // message0, update0, message1, ... same order as state_dict
  } else if (i < PK_WR) {
    v = f[oWp + (i - PK_WP)];
  } else if (i < PK_BR) {
    v = f[oWr + (i - PK_WR)];
  } else if (i == PK_BR) {
    v = f[oBr];
  }
  p[i] = v;
}

struct MpnnArgs {
  const float* P;
  eco_graph_set gs;
  const int32_t* gids;
  int B, N, gpb, nobs;
  const float* x;        // [B*N][8]
  int norm_scope;
  const int* call_maxdeg;
  float* q;              // [B*N] or null
  float* E;              // workspace [B*N][64]
  int has_act;
  eco_act_config act;
  int32_t* actions;
};

__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }

// acc[nt] += A(16 rows x 16 k, one float4 per lane) * W[nt*16 + (l&15)][kbase + 4(l>>4) + 0..3]
__device__ __forceinline__ void mm_chunk(f32x4 (&acc)[4], float4 a, const float* __restrict__ W, int ldw, int kbase,
                                         int lane) {
  const float* wp = W + (lane & 15) * ldw + kbase + 4 * (lane >> 4);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const float4 b = *reinterpret_cast<const float4*>(wp + nt * 16 * ldw);
    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc[nt], 0, 0, 0);
    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc[nt], 0, 0, 0);
    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc[nt], 0, 0, 0);
    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc[nt], 0, 0, 0);
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct NodeRef {
  bool valid;
  int gl, v, e, gid, e0, e1, norm;
  const uint32_t* ed;
};

__device__ __forceinline__ NodeRef node_ref(const MpnnArgs& a, int blk, int r, int rows_valid) {
  NodeRef n;
  n.valid = r < rows_valid;
  const int rr = n.valid ? r : 0;
  n.gl = rr / a.N;
  n.v = rr - n.gl * a.N;
  n.e = blk * a.gpb + n.gl;
  n.gid = a.gids[n.e];
  const int32_t* rp = a.gs.row_ptr + (size_t)n.gid * (a.N + 1);
  n.e0 = n.valid ? rp[n.v] : 0;
  n.e1 = n.valid ? rp[n.v + 1] : 0;
  n.norm = max(a.gs.deg[(size_t)n.gid * a.N + n.v], 1);  // mpnn.py:36-37
  n.ed = a.gs.edges + a.gs.edge_base[n.gid];
  return n;
}

template <int MAXT>
__global__ __launch_bounds__(TPB) void mpnn_forward_kernel(MpnnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int blk = blockIdx.x;
  const int N = a.N;
  const int g_valid = min(a.gpb, a.B - blk * a.gpb);
  const int rows_valid = g_valid * N;
  const int rows_pad = (a.gpb * N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  float* Hs = lds;                                  // [rows_pad][LDH]
  float* Ms = lds + rows_pad * LDH + w * 16 * LDH;  // per-wave [16][LDH]
  const size_t R0 = (size_t)blk * a.gpb * N;        // first global row of the block
  const float* P = a.P;
  const int s4 = lane >> 4;

  // ---- phase A: Z = Wx . x  (edge-embedding node term) into Hs ----
  {
    float wx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) wx[k] = P[PK_WX + lane * 8 + k];
    for (int r = w; r < rows_pad; r += NWAVE) {
      float z = 0.f;
      if (r < rows_valid) {
        const float4* xp = reinterpret_cast<const float4*>(a.x + (R0 + r) * 8);
        const float4 x0 = xp[0], x1 = xp[1];
        z = wx[0] * x0.x + wx[1] * x0.y + wx[2] * x0.z + wx[3] * x0.w + wx[4] * x1.x + wx[5] * x1.y + wx[6] * x1.z +
            wx[7] * x1.w;
      }
      Hs[r * LDH + lane] = z;
    }
  }
  __syncthreads();

  // ---- phase B: edge embedding (mpnn.py:89-104) -> E (global workspace) ----
  {
    int maxdeg_call = 0;
    if (a.norm_scope == ECO_NORM_PER_CALL) maxdeg_call = *a.call_maxdeg;
    float wa[16];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) wa[c * 4 + i] = P[PK_WA + 16 * c + 4 * s4 + i];
    for (int t = w; t < ntiles; t += NWAVE) {
      const int r = t * 16 + (lane & 15);
      const NodeRef n = node_ref(a, blk, r, rows_valid);
      float4 acc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      const int rbase = n.gl * N;
      for (int q = n.e0; q < n.e1; ++q) {
        const uint32_t ex = n.ed[q];
        const float wv = (float)edge_w(ex);
        const float* zr = Hs + (rbase + edge_col(ex)) * LDH + 4 * s4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 z = *reinterpret_cast<const float4*>(zr + 16 * c);
          acc[c].x += relu(fmaf(wv, wa[4 * c + 0], z.x));
          acc[c].y += relu(fmaf(wv, wa[4 * c + 1], z.y));
          acc[c].z += relu(fmaf(wv, wa[4 * c + 2], z.z));
          acc[c].w += relu(fmaf(wv, wa[4 * c + 3], z.w));
        }
      }
      const float nf = (float)n.norm;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c].x = acc[c].x / nf; acc[c].y = acc[c].y / nf; acc[c].z = acc[c].z / nf; acc[c].w = acc[c].w / nf;
      }
      // feature 63 = norm / norm.max()  (mpnn.py:102)
      const int md = a.norm_scope == ECO_NORM_PER_CALL ? maxdeg_call : a.gs.max_deg[n.gid];
      if (s4 == 3) acc[3].w = nf / (float)md;
      if (!n.valid) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      f32x4 d[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) mm_chunk(d, acc[c], P + PK_WF, 64, 16 * c, lane);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = t * 16 + 4 * s4 + rr;
        if (row < rows_valid) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) a.E[(R0 + row) * 64 + nt * 16 + (lane & 15)] = relu(d[nt][rr]);
        }
      }
    }
  }
  __syncthreads();

  // ---- phase C: h0 = relu(W0 . x) (mpnn.py:20-23, :55) into Hs ----
  {
    float w0[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w0[k] = P[PK_W0 + lane * 8 + k];
    for (int r = w; r < rows_pad; r += NWAVE) {
      float z = 0.f;
      if (r < rows_valid) {
        const float4* xp = reinterpret_cast<const float4*>(a.x + (R0 + r) * 8);
        const float4 x0 = xp[0], x1 = xp[1];
        z = w0[0] * x0.x + w0[1] * x0.y + w0[2] * x0.z + w0[3] * x0.w + w0[4] * x1.x + w0[5] * x1.y + w0[6] * x1.z +
            w0[7] * x1.w;
      }
      Hs[r * LDH + lane] = relu(z);
    }
  }
  __syncthreads();

  // ---- phase D: 3 x UpdateNodeEmbeddingLayer (mpnn.py:114-120) ----
  for (int layer = 0; layer < 3; ++layer) {
    const float* Wm = P + PK_LAYER + layer * 16384;
    const float* Wu = Wm + 8192;
    f32x4 hn[MAXT][4];
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = w + ti * NWAVE;
      if (t < ntiles) {
        const int r = t * 16 + (lane & 15);
        const NodeRef n = node_ref(a, blk, r, rows_valid);
        // aggregation (A . h) / norm, in A-operand layout
        float4 agg[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) agg[c] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int rbase = n.gl * N;
        for (int q = n.e0; q < n.e1; ++q) {
          const uint32_t ex = n.ed[q];
          const float wv = (float)edge_w(ex);
          const float* hr = Hs + (rbase + edge_col(ex)) * LDH + 4 * s4;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float4 hv = *reinterpret_cast<const float4*>(hr + 16 * c);
            agg[c].x = fmaf(wv, hv.x, agg[c].x);
            agg[c].y = fmaf(wv, hv.y, agg[c].y);
            agg[c].z = fmaf(wv, hv.z, agg[c].z);
            agg[c].w = fmaf(wv, hv.w, agg[c].w);
          }
        }
        const float nf = (float)n.norm;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          agg[c].x = agg[c].x / nf; agg[c].y = agg[c].y / nf; agg[c].z = agg[c].z / nf; agg[c].w = agg[c].w / nf;
        }
        // message = relu(Wm . [agg, e])
        f32x4 d[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) mm_chunk(d, agg[c], Wm, 128, 16 * c, lane);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float4 ev = make_float4(0.f, 0.f, 0.f, 0.f);
          if (n.valid) ev = *reinterpret_cast<const float4*>(a.E + (R0 + r) * 64 + 16 * c + 4 * s4);
          mm_chunk(d, ev, Wm, 128, 64 + 16 * c, lane);
        }
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) Ms[(4 * s4 + rr) * LDH + nt * 16 + (lane & 15)] = relu(d[nt][rr]);
        wave_lds_sync();
        // h' = relu(Wu . [h, m])
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) hn[ti][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c)
          mm_chunk(hn[ti], *reinterpret_cast<const float4*>(Hs + r * LDH + 16 * c + 4 * s4), Wu, 128, 16 * c, lane);
#pragma unroll
        for (int c = 0; c < 4; ++c)
          mm_chunk(hn[ti], *reinterpret_cast<const float4*>(Ms + (lane & 15) * LDH + 16 * c + 4 * s4), Wu, 128,
                   64 + 16 * c, lane);
        wave_lds_sync();
      }
    }
    __syncthreads();
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = w + ti * NWAVE;
      if (t < ntiles) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) Hs[(t * 16 + 4 * s4 + rr) * LDH + nt * 16 + (lane & 15)] = relu(hn[ti][nt][rr]);
      }
    }
    __syncthreads();
  }

  // ---- phase E: ReadoutLayer (mpnn.py:143-159) + epsilon-greedy act ----
  const float br = P[PK_BR];
  for (int gl = w; gl < g_valid; gl += NWAVE) {
    const int e = blk * a.gpb + gl;
    const float* hg = Hs + gl * N * LDH;
    float cs = 0.f;
    for (int v = 0; v < N; ++v) cs += hg[v * LDH + lane];
    const float mean = cs / (float)N;
    float p = 0.f;
    const float* wp = P + PK_WP + lane * 64;
#pragma unroll 8
    for (int k = 0; k < 64; ++k) p = fmaf(wp[k], __shfl(mean, k, 64), p);
    const float cg = wave_sum_f(relu(p) * P[PK_WR + lane]);
    float bestq = -INFINITY;
    int besti = 0x7fffffff;
    int n_allowed = 0;
    for (int v0 = 0; v0 < N; v0 += 64) {
      const int v = v0 + lane;
      float qv = -INFINITY;
      bool allowed = false;
      if (v < N) {
        const float* hr = hg + v * LDH;
        float ql = 0.f;
#pragma unroll 4
        for (int f = 0; f < 64; f += 4) {
          const float4 hv = *reinterpret_cast<const float4*>(hr + f);
          ql = fmaf(hv.x, P[PK_WR + 64 + f], ql);
          ql = fmaf(hv.y, P[PK_WR + 65 + f], ql);
          ql = fmaf(hv.z, P[PK_WR + 66 + f], ql);
          ql = fmaf(hv.w, P[PK_WR + 67 + f], ql);
        }
        qv = cg + ql + br;
        if (a.q) a.q[(size_t)e * N + v] = qv;
        allowed = a.act.reversible || (a.x[((size_t)e * N + v) * 8] == a.act.allowed_value);
      }
      n_allowed += __popcll(__ballot(allowed));
      if (allowed && (qv > bestq || (qv == bestq && v < besti))) { bestq = qv; besti = v; }
    }
    if (a.has_act) {
      // first index of the max (torch argmax)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float oq = __shfl_xor(bestq, o, 64);
        const int oi = __shfl_xor(besti, o, 64);
        if (oq > bestq || (oq == bestq && oi < besti)) { bestq = oq; besti = oi; }
      }
      int action = besti;
      const uint64_t r0 = rng3(a.act.seed, a.act.counter, (uint64_t)e);
      if (u01(r0) < a.act.epsilon && n_allowed > 0) {  // random.uniform(0,1) >= eps -> greedy
        const uint64_t r1 = rng3(a.act.seed ^ 0xA5A5A5A5ull, a.act.counter, (uint64_t)e);
        int k = (int)(r1 % (uint64_t)n_allowed);
        if (a.act.reversible) {
          action = k;
        } else {
          // k-th allowed vertex
          action = -1;
          for (int v0 = 0; v0 < N && action < 0; v0 += 64) {
            const int v = v0 + lane;
            const bool al = v < N && a.x[((size_t)e * N + v) * 8] == a.act.allowed_value;
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
}

__global__ void call_maxdeg_kernel(const eco_graph_set gs, const int32_t* gids, int B, int* out) {
  int m = 1;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B; i += gridDim.x * blockDim.x) m = max(m, gs.max_deg[gids[i]]);
  m = wave_max_i(m);
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

static int graphs_per_block(int N) { return N >= 256 ? 1 : 256 / N; }

}  // namespace eco

using namespace eco;

extern "C" size_t eco_mpnn_param_count(int32_t n_obs_in) {
  if (n_obs_in < 1 || n_obs_in > ECO_MAX_OBS) return 0;
  return (size_t)flat_count(n_obs_in);
}

extern "C" size_t eco_mpnn_packed_count(void) { return (size_t)PK_TOTAL; }

extern "C" int eco_mpnn_pack(const float* params, int32_t n_obs_in, float* packed, eco_stream_t stream) {
  if (!params || !packed) return fail(ECO_ERR_ARG, "null params/packed");
  if (n_obs_in < 1 || n_obs_in > ECO_MAX_OBS) return fail(ECO_ERR_ARG, "n_obs_in out of range [1, 8]");
  pack_kernel<<<(PK_TOTAL + 255) / 256, 256, 0, (hipStream_t)stream>>>(params, n_obs_in, packed);
  return check_launch("mpnn_pack");
}

extern "C" size_t eco_mpnn_workspace_bytes(int32_t n_spins, int32_t batch) {
  if (n_spins < 1 || batch < 1) return 0;
  return 256 + (size_t)n_spins * batch * 64 * sizeof(float);
}

extern "C" int eco_mpnn_forward(const float* packed, int32_t n_obs_in, const eco_graph_set* gs,
                                const int32_t* graph_ids, int32_t batch, const float* obs_x, int32_t norm_scope,
                                float* q, const eco_act_config* act, int32_t* actions, void* workspace,
                                eco_stream_t stream) {
  if (!packed || !gs || !graph_ids || !obs_x || !workspace) return fail(ECO_ERR_ARG, "null argument");
  if (n_obs_in < 1 || n_obs_in > ECO_MAX_OBS) return fail(ECO_ERR_ARG, "n_obs_in out of range [1, 8]");
  if (batch < 1) return fail(ECO_ERR_ARG, "batch must be >= 1");
  const int N = gs->n_spins;
  if (N < 1 || N > 512) return fail(ECO_ERR_ARG, "mpnn_forward supports 1 <= N <= 512");
  if (norm_scope != ECO_NORM_PER_GRAPH && norm_scope != ECO_NORM_PER_CALL)
    return fail(ECO_ERR_ARG, "bad norm_scope");
  if (act && !actions) return fail(ECO_ERR_ARG, "act config without actions buffer");
  if (!q && !act) return fail(ECO_ERR_ARG, "nothing to compute (q and act both null)");
  hipStream_t st = (hipStream_t)stream;
  MpnnArgs a{};
  a.P = packed; a.gs = *gs; a.gids = graph_ids; a.B = batch; a.N = N; a.gpb = graphs_per_block(N);
  a.nobs = n_obs_in; a.x = obs_x; a.norm_scope = norm_scope; a.q = q;
  int* cmax = (int*)workspace;
  a.call_maxdeg = cmax;
  a.E = (float*)((char*)workspace + 256);
  a.has_act = act != nullptr;
  if (act) a.act = *act;
  a.actions = actions;
  if (norm_scope == ECO_NORM_PER_CALL) {
    if (hipMemsetAsync(cmax, 0, sizeof(int), st) != hipSuccess) return fail(ECO_ERR_HIP, "memset failed");
    call_maxdeg_kernel<<<min(256, (batch + 255) / 256), 256, 0, st>>>(*gs, graph_ids, batch, cmax);
  }
  const int blocks = (batch + a.gpb - 1) / a.gpb;
  const int rows_pad = (a.gpb * N + 15) & ~15;
  const size_t lds = ((size_t)rows_pad * LDH + (size_t)NWAVE * 16 * LDH) * sizeof(float);
  const int ntiles = rows_pad / 16;
  if (ntiles <= 4 * NWAVE) {
    (void)hipFuncSetAttribute((const void*)mpnn_forward_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    mpnn_forward_kernel<4><<<blocks, TPB, lds, st>>>(a);
  } else {
    (void)hipFuncSetAttribute((const void*)mpnn_forward_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    mpnn_forward_kernel<8><<<blocks, TPB, lds, st>>>(a);
  }
  return check_launch("mpnn_forward");
}
