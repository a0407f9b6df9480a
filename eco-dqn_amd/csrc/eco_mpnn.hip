// MPNN Q-network (src/networks/mpnn.py) forward + backward, fused per graph block on
// gfx950, with the epsilon-greedy act (dqn.py:453-465, :490-512) fused into the readout.
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
// The backward (autograd of the same graph, dqn.py:440-449) mirrors it: activation
// gradients per block (A^T.x aggregations are gathers because A is symmetric), weight
// gradients as separate split-K reductions over all nodes (eco_train.hip).
#include "eco_common.h"
#include "eco_mpnn.h"
#include "eco_mpnn_dev.h"

#include <atomic>
#include <cstdlib>

namespace eco {

// Optional per-phase wall-clock stamps (make timing -> libecohip_timing.so; tools/phase_timing.py).
// Slots [blk][0..15] forward, [blk][16..31] backward, first ECO_TS_BLOCKS blocks only.
#ifdef ECO_PHASE_TIMING
constexpr int ECO_TS_BLOCKS = 8192;
__device__ unsigned long long eco_phase_ts[ECO_TS_BLOCKS * 32];
#define ECO_TS(k)                                                                                           \
  do {                                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < ECO_TS_BLOCKS) eco_phase_ts[blockIdx.x * 32 + (k)] = wall_clock64(); \
  } while (0)
// stamps of logical block b (persistent kernels: one workgroup walks several blocks)
#define ECO_TSB(k, b)                                                                       \
  do {                                                                                      \
    if (threadIdx.x == 0 && (b) < ECO_TS_BLOCKS) eco_phase_ts[(b) * 32 + (k)] = wall_clock64(); \
  } while (0)
#else
#define ECO_TS(k) \
  do {            \
  } while (0)
#define ECO_TSB(k, b) \
  do {                \
  } while (0)
#endif


}  // namespace eco
#include "eco_mpnn_dense.h"  // dense-aggregation kernels (after the phase-timing buffer)
#include "eco_mpnn_dense2.h"  // their fp16x2 successors
#include "eco_mpnn_dense3.h"  // the fp16x2 forward, two tiles per wave
#include "eco_mpnn_dl.h"      // one graph of 224 < N <= 512 per workgroup
#include "eco_mpnn_shared.h"  // many episodes on one shared large graph (G22)
namespace eco {

// Per-matrix power-of-two scale of the fp16x2 Linear pieces (PK_FHS, eco_mpnn.h): one block per matrix
// (Wf, then Wm / Wu of each layer); kw puts max |w| 2^kw into [2^14, 2^15).
__device__ __forceinline__ float wave_fmax(float v) {  // fmaxf over the wave (NaNs dropped, as fmaxf does)
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x128, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x124, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x122, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x121, 0xF, 0xF, false)));
  auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(s16[0]), __uint_as_float(s16[1]));
  auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(s32[0]), __uint_as_float(s32[1]));
}

// Per-matrix power-of-two scale of the fp16x2 Linear pieces (PK_FHS, eco_mpnn.h): one block per matrix
// (Wf, then Wm / Wu of each layer); kw puts max |w| 2^kw into [2^14, 2^15).  1024 threads, wave maxima.
constexpr int PS_THREADS = 1024;
__global__ __launch_bounds__(PS_THREADS) void pack_scale_kernel(const float* __restrict__ f, int nobs,
                                                                 float* __restrict__ p) {
  const FlatOffsets o = flat_offsets(nobs);
  const int m = blockIdx.x;
  const float* W = m == 0 ? f + o.Wf : f + o.L + (m - 1) * 8192;
  const int n = m == 0 ? 4096 : 8192;
  float mx = 0.f;
  for (int i = threadIdx.x; i < n; i += PS_THREADS) mx = fmaxf(mx, fabsf(W[i]));
  mx = wave_fmax(mx);
  __shared__ float red[PS_THREADS / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = 0.f;
    for (int k = 0; k < PS_THREADS / 64; ++k) v = fmaxf(v, red[k]);
    const int kw = (v > 0.f && v < INFINITY) ? 15 - __builtin_amdgcn_frexp_expf(v) : 0;
    p[PK_FHS + m] = __int_as_float(kw);
  }
}

__global__ void pack_kernel(const float* __restrict__ f, int nobs, float* __restrict__ p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= PK_TOTAL) return;
  const FlatOffsets o = flat_offsets(nobs);
  float v = 0.f;
  if (i >= PK_FHS && i < PK_FH) return;  // scale exponents: pack_scale_kernel
  if (i >= PK_FH) {  // fp16x2 pieces, two fp16 per float slot
    uint16_t h[2];
    for (int t = 0; t < 2; ++t) {
      const int e = 2 * (i - PK_FH) + t;
      const bool tr = e >= FH_FWD_END;
      const int et = tr ? e - FH_FWD_END : e;
      const float* W;
      int in_dim, lin, mat;
      if (et < FH_LAYER) {
        W = f + o.Wf;
        in_dim = 64;
        lin = et;
        mat = 0;
      } else {
        const int e2 = et - FH_LAYER;
        const int l = e2 / FH_LAYER_STRIDE, r = e2 % FH_LAYER_STRIDE;
        const int which = r / (2 * FH_HALF);
        W = f + o.L + l * 16384 + which * 8192;
        in_dim = 128;
        lin = r % (2 * FH_HALF);
        mat = 1 + 2 * l + which;
      }
      const int frag = lin / FH_FRAG, within = lin % FH_FRAG;
      const int ln = within >> 3, jj = within & 7;
      const int kc2 = frag & 1, nt = (frag >> 1) & 3, pl = (frag >> 3) & 1, half = frag >> 4;
      const int kp = 64 * half + 32 * kc2 + 8 * (ln >> 4) + jj;
      const float wv = tr ? W[bf16_kprime_feature(kp & 63) * in_dim + 64 * half + 16 * nt + (ln & 15)]
                          : W[(16 * nt + (ln & 15)) * in_dim + bf16_kprime_feature(kp)];
      const float s = ldexpf(wv, __float_as_int(p[PK_FHS + mat]));
      const _Float16 h1 = (_Float16)s;
      const _Float16 h2 = (_Float16)(s - (float)h1);
      h[t] = __builtin_bit_cast(uint16_t, pl == 0 ? h1 : h2);
    }
    v = __uint_as_float((uint32_t)h[0] | ((uint32_t)h[1] << 16));
  } else if (i >= PK_W0H) {  // feature columns 8..15
    const bool wx = i >= PK_WXH;
    const int j = i - (wx ? PK_WXH : PK_W0H);
    const int r = j >> 3, c = 8 + (j & 7);
    if (!wx) v = c < nobs ? f[o.W0 + r * nobs + c] : 0.f;
    else v = (r < 63 && c < nobs) ? f[o.We + r * (1 + nobs) + 1 + c] : 0.f;
  } else if (i < PK_WX) {
    const int r = i >> 3, c = i & 7;
    v = c < nobs ? f[o.W0 + r * nobs + c] : 0.f;
  } else if (i < PK_WA) {
    const int r = (i - PK_WX) >> 3, c = (i - PK_WX) & 7;
    v = (r < 63 && c < nobs) ? f[o.We + r * (1 + nobs) + 1 + c] : 0.f;
  } else if (i < PK_WF) {
    const int r = i - PK_WA;
    v = r < 63 ? f[o.We + r * (1 + nobs)] : 0.f;
  } else if (i < PK_LAYER) {
    v = f[o.Wf + (i - PK_WF)];
  } else if (i < PK_WP) {
    v = f[o.L + (i - PK_LAYER)];  // message0, update0, message1, ... same order as state_dict
  } else if (i < PK_WR) {
    v = f[o.Wp + (i - PK_WP)];
  } else if (i < PK_BR) {
    v = f[o.Wr + (i - PK_WR)];
  } else if (i == PK_BR) {
    v = f[o.Br];
  } else if (i >= PK_WFT && i < PK_LAYERT) {
    const int j = i - PK_WFT;  // WfT[in][out] = Wf[out][in]
    v = f[o.Wf + (j & 63) * 64 + (j >> 6)];
  } else if (i >= PK_LAYERT && i < PK_LAYERT + 3 * 16384) {
    const int l = (i - PK_LAYERT) / 16384;
    const int j = (i - PK_LAYERT) % 16384;
    const int which = j / 8192;  // 0: message, 1: update
    const int jj = j % 8192;     // T[in (128)][out (64)]
    v = f[o.L + l * 16384 + which * 8192 + (jj & 63) * 128 + (jj >> 6)];
  } else if (i >= PK_BF) {
    // two bf16 plane elements per float slot
    uint16_t h[2];
    for (int t = 0; t < 2; ++t) {
      const int e = 2 * (i - PK_BF) + t;
      const float* W;
      int in_dim, lin;
      const bool tr = e >= BF_FWD_END;  // transposed fragments of the backward
      const int et = tr ? e - BF_FWD_END : e;
      if (et < BF_LAYER) {
        W = f + o.Wf;
        in_dim = 64;
        lin = et;
      } else {
        const int e2 = et - BF_LAYER;
        const int l = e2 / BF_LAYER_STRIDE, r = e2 % BF_LAYER_STRIDE;
        W = f + o.L + l * 16384 + (r / (2 * BF_HALF)) * 8192;
        in_dim = 128;
        lin = r % (2 * BF_HALF);
      }
      const int frag = lin / BF_FRAG, within = lin % BF_FRAG;
      const int ln = within >> 3, jj = within & 7;
      const int kc2 = frag & 1, nt = (frag >> 1) & 3, pl = (frag >> 3) % 3, half = frag / 24;
      const int kp = 64 * half + 32 * kc2 + 8 * (ln >> 4) + jj;
      // forward: W[16nt + (l&15)][feature(kp)];  transposed: W^T[64 half + 16nt + (l&15)][feature(kp & 63)]
      const float wv = tr ? W[bf16_kprime_feature(kp & 63) * in_dim + 64 * half + 16 * nt + (ln & 15)]
                          : W[(16 * nt + (ln & 15)) * in_dim + bf16_kprime_feature(kp)];
      uint16_t p1, p2, p3;
      split3_bits(wv, p1, p2, p3);
      h[t] = pl == 0 ? p1 : (pl == 1 ? p2 : p3);
    }
    v = __uint_as_float((uint32_t)h[0] | ((uint32_t)h[1] << 16));
  }
  p[i] = v;
}

// MAXT: max 16-node tiles per wave; NW: waves per workgroup; WLDS: stage each layer's weights in
// LDS (one copy per workgroup, read as conflict-free ds_read_b128 B operands) instead of
// streaming them from L2 in every wave.
// LDS: Hs [rows_pad][LDH] | Wl [2][64][LDW] (WLDS) | Xs [rows_pad][8] (WLDS) or readout scratch |
//      RI [rows_pad] int2 | GB [gpb] i64 | MD [gpb]
template <int MAXT, bool SAVE, int NW, bool WLDS>
__global__ __launch_bounds__(64 * NW, (NW == 8 && WLDS ? 2 : 1)) void mpnn_forward_kernel(MpnnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  ECO_TS(0);
  constexpr int NT = 64 * NW;
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int blk = blockIdx.x;
  const int N = a.N;
  const int g_valid = min(a.gpb, a.B - blk * a.gpb);
  const int rows_valid = g_valid * N;
  const int rows_pad = (a.gpb * N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  float* Hs = lds;
  float* Wl = lds + rows_pad * LDH;
  float* Mreg = Wl + (WLDS ? 2 * 64 * LDW : 0);
  float* Xs = Mreg;                 // [rows_pad][8] node features (WLDS; else x is read from global)
  int2* RI = reinterpret_cast<int2*>(Mreg + fwd_mreg_floats(rows_pad, a.gpb, NW, WLDS));
  int64_t* GB = reinterpret_cast<int64_t*>(RI + rows_pad);  // [gpb] per-graph edge base
  int* MD = reinterpret_cast<int*>(GB + a.gpb);               // [gpb] per-graph max degree
  int* SCH = MD + ((a.gpb + 1) & ~1);                           // [64] tile schedule
  float* Es = WLDS ? Wl : Mreg;     // phase-E scratch
  const size_t R0 = (size_t)blk * a.gpb * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const uint16_t* BFP = reinterpret_cast<const uint16_t*>(P + PK_BF);
  const int s4 = lane >> 4;
  const int c16 = lane & 15;
  const uint32_t* __restrict__ edges = a.gs.edges;

  // ---- staging: x rows (WLDS, 8-float rows), row info, Wf ----
  const bool xwide = a.xw == 16;  // features 8..15 (read from global memory, never staged)
  if (WLDS && !xwide) {
    for (int i = threadIdx.x; i < rows_pad * 2; i += NT) {
      const int r = i >> 1;
      float4 v = zero4();
      if (r < rows_valid) v = f4(a.x + (R0 + r) * 8 + 4 * (i & 1));
      st4(Xs + 8 * r + 4 * (i & 1), v);
    }
  }
  // node features 0..7 of row r (zero for padding rows)
  auto xrow = [&](int r, float4& x0, float4& x1) {
    if (WLDS && !xwide) {
      x0 = f4(Xs + 8 * r);
      x1 = f4(Xs + 8 * r + 4);
    } else {
      x0 = r < rows_valid ? f4(a.x + (R0 + r) * a.xw) : zero4();
      x1 = r < rows_valid ? f4(a.x + (R0 + r) * a.xw + 4) : zero4();
    }
  };
  // w . x over features 8..15 (wide rows only)
  auto xdot_hi = [&](int r, const float* wh) {
    if (!xwide || r >= rows_valid) return 0.f;
    const float4 x2 = f4(a.x + (R0 + r) * 16 + 8), x3 = f4(a.x + (R0 + r) * 16 + 12);
    return wh[0] * x2.x + wh[1] * x2.y + wh[2] * x2.z + wh[3] * x2.w + wh[4] * x3.x + wh[5] * x3.y + wh[6] * x3.z +
           wh[7] * x3.w;
  };
  for (int r = threadIdx.x; r < rows_pad; r += NT) RI[r] = pack_row_info(a, blk, r, rows_valid);
  for (int gl = threadIdx.x; gl < g_valid; gl += NT) {
    const int gid = a.gids[blk * a.gpb + gl];
    GB[gl] = a.gs.edge_base[gid];
    MD[gl] = a.gs.max_deg[gid];
  }
  if constexpr (WLDS) stage_rows<NT>(Wl, LDH, P + PK_WF, 64, 64, 64);
  __syncthreads();
  if (w == 0) build_tile_schedule(SCH, RI, ntiles, NW, MAXT);  // published by the barrier after phase A
  ECO_TS(1);

  // ---- phase A: Z = Wx . x  (edge-embedding node term) into Hs ----
  {
    float wx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) wx[k] = P[PK_WX + lane * 8 + k];
    for (int r = w; r < rows_pad; r += NW) {
      float4 x0, x1;
      xrow(r, x0, x1);
      Hs[r * LDH + lane] = wx[0] * x0.x + wx[1] * x0.y + wx[2] * x0.z + wx[3] * x0.w + wx[4] * x1.x +
                           wx[5] * x1.y + wx[6] * x1.z + wx[7] * x1.w + xdot_hi(r, P + PK_WXH + lane * 8);
    }
  }
  __syncthreads();
  ECO_TS(2);

  // ---- phase B: edge embedding (mpnn.py:89-104) -> e (registers, operand layout) ----
  float4 ereg[MAXT][4];
  {
    const int maxdeg_call = a.norm_scope == ECO_NORM_PER_CALL ? *a.call_maxdeg : 0;
    float wa[16];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) wa[c * 4 + i] = P[PK_WA + 16 * c + 4 * s4 + i];
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = SCH[w + ti * NW];
      if (t >= ntiles) break;
      const int r = t * 16 + c16;
      const RowInfo ri = row_info(RI, r);
      const bool valid = r < rows_valid;
      const int rbase = (r / N) * N;
      float4 acc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = zero4();
      for_edges(edges + (valid ? GB[r / N] : 0), ri.e0, ri.e1, [&](uint32_t ex) {
        const float wv = (float)edge_w(ex);
        const float* zr = Hs + (rbase + edge_col(ex)) * LDH + 4 * s4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 z = f4(zr + 16 * c);
          acc[c].x += relu(fmaf(wv, wa[4 * c + 0], z.x));
          acc[c].y += relu(fmaf(wv, wa[4 * c + 1], z.y));
          acc[c].z += relu(fmaf(wv, wa[4 * c + 2], z.z));
          acc[c].w += relu(fmaf(wv, wa[4 * c + 3], z.w));
        }
      });
      const float nf = (float)ri.norm;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c].x = acc[c].x / nf; acc[c].y = acc[c].y / nf; acc[c].z = acc[c].z / nf; acc[c].w = acc[c].w / nf;
      }
      // feature 63 = norm / norm.max()  (mpnn.py:102)
      const int md = a.norm_scope == ECO_NORM_PER_CALL ? maxdeg_call : (valid ? MD[r / N] : 1);
      if (s4 == 3) acc[3].w = nf / (float)md;
      if (!valid) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = zero4();
      } else if (SAVE) {
        float* ea = a.sv + (size_t)SV_EAGG * RT * 64 + (R0 + r) * 64 + 4 * s4;
#pragma unroll
        for (int c = 0; c < 4; ++c) st4(ea + 16 * c, acc[c]);
      }
      f32x4 d[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (WLDS) mm_k<4, 4, true>(d, acc, Wl, LDH, lane);
      else mm_bf3_lean(d, acc, BFP + BF_WF, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        ereg[ti][nt] = relu4(d[nt]);  // the tile's e rows stay in this wave's registers for the layers
        if (SAVE && valid) st4(a.sv + (size_t)SV_E * RT * 64 + (R0 + r) * 64 + 16 * nt + 4 * s4, ereg[ti][nt]);
      }
    }
  }
  __syncthreads();
  ECO_TS(3);

  // ---- phase C: h0 = relu(W0 . x) (mpnn.py:20-23, :55) into Hs ----
  {
    float w0[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w0[k] = P[PK_W0 + lane * 8 + k];
    for (int r = w; r < rows_pad; r += NW) {
      float4 x0, x1;
      xrow(r, x0, x1);
      const float z = relu(w0[0] * x0.x + w0[1] * x0.y + w0[2] * x0.z + w0[3] * x0.w + w0[4] * x1.x +
                           w0[5] * x1.y + w0[6] * x1.z + w0[7] * x1.w + xdot_hi(r, P + PK_W0H + lane * 8));
      if (SAVE && r < rows_valid) a.sv[(size_t)SV_H0 * RT * 64 + (R0 + r) * 64 + lane] = z;
      Hs[r * LDH + lane] = z;
    }
  }
  __syncthreads();
  ECO_TS(4);

  // ---- phase D: 3 x UpdateNodeEmbeddingLayer (mpnn.py:114-120) ----
  for (int layer = 0; layer < 3; ++layer) {
    const float* Wm = P + PK_LAYER + layer * 16384;
    const float* Wu = Wm + 8192;
    if constexpr (WLDS) {  // the previous readers of Wl finished at the last barrier
      stage_rows<NT>(Wl, LDW, Wm, 128, 64, 128);
      stage_rows<NT>(Wl + 64 * LDW, LDW, Wu, 128, 64, 128);
      __syncthreads();
    }
    if (layer == 0) ECO_TS(10);
    // Half of each tile's MFMAs do not depend on the aggregation: Wm[:, 64:].e and Wu[:, :64].h.
    // Waves with (w >> 2) even issue that half BEFORE their gather, the others after it, so each
    // SIMD's MFMA pipe has work while its other waves gather from LDS (waves w, w+4 share a SIMD).
    const bool mfma_first = ((w >> 2) & 1) == 0;
    const float* WmL = WLDS ? Wl : Wm;
    const float* WuL = WLDS ? Wl + 64 * LDW : Wu;
    // weights from L2 (no LDS staging): the exact bf16x3-split fragments of the dense path (six products
    // above 2^-24, f32-accurate) -- 2.7x the f32 MFMA rate, and no f32 weight double buffer in registers
    const uint16_t* BFL = BFP + BF_LAYER + layer * BF_LAYER_STRIDE;  // message halves, then update halves
    constexpr int ldw = WLDS ? LDW : 128;
    f32x4 hn[MAXT][4];
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = SCH[w + ti * NW];
      if (t < ntiles) {
        const int r = t * 16 + c16;
        const RowInfo ri = row_info(RI, r);
        const bool valid = r < rows_valid;
        float4 agg[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) agg[c] = zero4();
        const uint32_t* eg = edges + (valid ? GB[r / N] : 0);
        if (!mfma_first) gather_ri(ri, eg, Hs, (r / N) * N, s4, agg);
        // gather-independent half: d = Wm[:, 64:] . e ; hn = Wu[:, :64] . h
        f32x4 d[4];
        float4 hcur[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
          hn[ti][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
          hcur[nt] = f4(Hs + r * LDH + 16 * nt + 4 * s4);
        }
        if constexpr (WLDS) {
          mm_k<4, 4, true>(d, ereg[ti], WmL + 64, ldw, lane);
          mm_k<4, 4, true>(hn[ti], hcur, WuL, ldw, lane);
        } else {
          mm_bf3_lean(d, ereg[ti], BFL + BF_HALF, lane);
          mm_bf3_lean(hn[ti], hcur, BFL + 2 * BF_HALF, lane);
        }
        if (layer == 0 && ti == 0) ECO_TS(11);
        if (mfma_first) gather_ri(ri, eg, Hs, (r / N) * N, s4, agg);
        if (layer == 0 && ti == 0) ECO_TS(12);
        // aggregation (A . h) / norm (mpnn.py:118), already in operand layout
        const float nf = (float)ri.norm;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          agg[c].x = agg[c].x / nf; agg[c].y = agg[c].y / nf; agg[c].z = agg[c].z / nf; agg[c].w = agg[c].w / nf;
        }
        if (SAVE && valid) {
          float* sa = a.sv + (size_t)(SV_AGG0 + layer) * RT * 64 + (R0 + r) * 64 + 4 * s4;
#pragma unroll
          for (int c = 0; c < 4; ++c) st4(sa + 16 * c, agg[c]);
        }
        // message = relu(Wm . [agg, e]) (mpnn.py:119)
        if constexpr (WLDS) mm_k<4, 4, true>(d, agg, WmL, ldw, lane);
        else mm_bf3_lean(d, agg, BFL, lane);
        float4 mrel[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) mrel[c] = relu4(d[c]);
        if (SAVE && valid) {
          float* sm = a.sv + (size_t)(SV_M0 + layer) * RT * 64 + (R0 + r) * 64 + 4 * s4;
#pragma unroll
          for (int c = 0; c < 4; ++c) st4(sm + 16 * c, mrel[c]);
        }
        // h' = relu(Wu . [h, m]) (mpnn.py:120)
        if constexpr (WLDS) mm_k<4, 4, true>(hn[ti], mrel, WuL + 64, ldw, lane);
        else mm_bf3_lean(hn[ti], mrel, BFL + 3 * BF_HALF, lane);
        if (layer == 0 && ti == 0) {
          ECO_TS(13);
#ifdef ECO_PHASE_TIMING
#ifdef ECO_PHASE_TIMING
          asm volatile("" ::"v"(hn[ti][3][3]));  // wait for the tile's last MFMA
#endif
#endif
          ECO_TS(14);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = SCH[w + ti * NW];
      if (t < ntiles) {
        const int r = t * 16 + c16;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const float4 hv = relu4(hn[ti][nt]);
          st4(Hs + r * LDH + 16 * nt + 4 * s4, hv);
          if (SAVE && r < rows_valid) st4(a.sv + (size_t)(SV_H0 + layer + 1) * RT * 64 + (R0 + r) * 64 + 16 * nt + 4 * s4, hv);
        }
      }
    }
    __syncthreads();
    ECO_TS(5 + layer);
  }

  // ---- phase E: ReadoutLayer (mpnn.py:143-159) + epsilon-greedy act, spread over all waves ----
  readout_act<SAVE, NW>(a, Hs, LDH, Es, a.gpb < NW, blk, g_valid, rows_valid, R0, RT);
  ECO_TS(8);
  ECO_TS(9);
}

// ============================================================== backward ====
// y[0..127] += W^T x for one 64-input transposed Linear from its two bf16x3 output-half fragment sets
__device__ __forceinline__ void bf3_t2(f32x4 (&d8)[8], const float4 (&x)[4], const uint16_t* WT, int lane) {
  f32x4 lo[4], hi[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) { lo[nt] = d8[nt]; hi[nt] = d8[4 + nt]; }
  mm_bf3_lean(lo, x, WT, lane);
  mm_bf3_lean(hi, x, WT + BF_HALF, lane);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) { d8[nt] = lo[nt]; d8[4 + nt] = hi[nt]; }
}

// Gradient of loss w.r.t. all MPNN parameters given dq = dLoss/dQ [B][N], for the
// forward saved in a.sv.  This kernel produces the activation gradients (the
// pre-activation gradients dY of every Linear, stored [R][64]) and the small
// per-graph / per-block partials; eco_train.hip reduces dW = sum_nodes dY^T X.
// LDS: G [rows_pad][LDH] (dq rows at the start) | Wl [2][128][LDH] (WLDS: Wu^T, Wm^T) | Xs [rows_pad][8] (WLDS) |
//      RI [rows_pad] int2 | GB [gpb] i64 | DMEAN [gpb][64] | RED [(gpb < NW ? gpb : 1)][NW][64]
template <int MAXT, int NW, bool WLDS>
__global__ __launch_bounds__(64 * NW, (NW == 8 && WLDS ? 2 : 1)) void mpnn_backward_kernel(MpnnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  ECO_TS(16);
  constexpr int NWAVE = NW;
  constexpr int NT = 64 * NW;
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int blk = blockIdx.x;
  const int N = a.N;
  const int g_valid = min(a.gpb, a.B - blk * a.gpb);
  const int rows_valid = g_valid * N;
  const int rows_pad = (a.gpb * N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  const bool split = a.gpb < NW;  // readout: all waves per graph
  float* G = lds;                                   // gathered-gradient source rows
  float* DQ = G;                                    // [rows_pad] dq of the block's rows (start only)
  float* Wl = G + rows_pad * LDH;                   // staged Wu^T | Wm^T, [128][LDH] each (WLDS)
  float* Xs = Wl + (WLDS ? 2 * 128 * LDH : 0);      // [rows_pad][8] (WLDS)
  int2* RI = reinterpret_cast<int2*>(Xs + (WLDS ? rows_pad * 8 : 0));
  int64_t* GB = reinterpret_cast<int64_t*>(RI + rows_pad);
  float* DMEAN = reinterpret_cast<float*>(GB + a.gpb);
  float* RED = DMEAN + a.gpb * 64;
  int* SCH = reinterpret_cast<int*>(RED + (a.gpb < NW ? a.gpb : 1) * NW * 64);  // [64] tile schedule
  const size_t R0 = (size_t)blk * a.gpb * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const float* sv = a.sv;
  float* gr = a.gr;
  const int s4 = lane >> 4;
  const int c16 = lane & 15;
  const uint32_t* __restrict__ edges = a.gs.edges;
  auto SV = [&](int t) { return sv + (size_t)t * RT * 64; };
  auto GR = [&](int t) { return gr + (size_t)t * RT * 64; };
  const float* MEAN = sv + (size_t)SV_NODE_TENSORS * RT * 64;
  const float* PP = MEAN + (size_t)a.B * 64;
  float* DP = gr + (size_t)GR_NODE_TENSORS * RT * 64;
  float* DWRA = DP + (size_t)a.B * 64;
  float* DWRB = DWRA + (size_t)a.B * 64;
  float* DBR = DWRB + (size_t)a.B * 64;
  float* DWA = DBR + ((a.B + 63) & ~63);  // [nblocks][64]

  // ---- staging: dq rows, row info, edge bases, x rows ----
  for (int r = threadIdx.x; r < rows_pad; r += NT) {
    DQ[r] = r < rows_valid ? a.dq[R0 + r] : 0.f;
    RI[r] = pack_row_info(a, blk, r, rows_valid);
  }
  for (int gl = threadIdx.x; gl < g_valid; gl += NT) GB[gl] = a.gs.edge_base[a.gids[blk * a.gpb + gl]];
  const bool xwide = a.xw == 16;  // features 8..15: read from global memory
  if (WLDS && !xwide) {
    for (int i = threadIdx.x; i < rows_pad * 2; i += NT) {
      const int r = i >> 1;
      st4(Xs + 8 * r + 4 * (i & 1), r < rows_valid ? f4(a.x + (R0 + r) * 8 + 4 * (i & 1)) : zero4());
    }
  }
  __syncthreads();
  if (w == 0) build_tile_schedule(SCH, RI, ntiles, NWAVE, MAXT);  // published by the barrier after the readout
  ECO_TS(17);

  // ---- readout backward (mpnn.py:143-159) ----
  // dWr[64:] = sum_v dq_v h3_v: spread over all waves when the block holds fewer graphs than waves
  if (split) {
    for (int gl = 0; gl < g_valid; ++gl) {
      const float* h3 = SV(SV_H3) + (R0 + (size_t)gl * N) * 64;
      float dwb = 0.f;
      for (int v = w; v < N; v += NWAVE) {
        const float dv = DQ[gl * N + v];
        if (dv != 0.f) dwb = fmaf(dv, h3[(size_t)v * 64 + lane], dwb);
      }
      RED[(gl * NWAVE + w) * 64 + lane] = dwb;
    }
    __syncthreads();
  }
  for (int gl = w; gl < g_valid; gl += NWAVE) {
    const int e = blk * a.gpb + gl;
    float s = 0.f;
    for (int v = lane; v < N; v += 64) s += DQ[gl * N + v];
    const float S = wave_sum_f(s);                       // d(sum_i q_i) / d br ...
    const float p = PP[(size_t)e * 64 + lane];
    const float wr = P[PK_WR + lane];
    const float dp = wr * S * (p > 0.f ? 1.f : 0.f);
    DP[(size_t)e * 64 + lane] = dp;
    DWRA[(size_t)e * 64 + lane] = relu(p) * S;
    if (lane == 0) DBR[e] = S;
    float dmean = 0.f;
#pragma unroll 16
    for (int k = 0; k < 64; ++k) dmean = fmaf(P[PK_WP + k * 64 + lane], __shfl(dp, k, 64), dmean);
    DMEAN[gl * 64 + lane] = dmean / (float)N;
    float dwb = 0.f;
    if (split) {
#pragma unroll
      for (int k = 0; k < NWAVE; ++k) dwb += RED[(gl * NWAVE + k) * 64 + lane];  // fixed order
    } else {
      const float* h3 = SV(SV_H3) + (R0 + (size_t)gl * N) * 64;
      for (int v = 0; v < N; ++v) {
        const float dv = DQ[gl * N + v];
        if (dv != 0.f) dwb = fmaf(dv, h3[(size_t)v * 64 + lane], dwb);
      }
    }
    DWRB[(size_t)e * 64 + lane] = dwb;
  }
  __syncthreads();
  ECO_TS(18);

  // dh3 (A layout): dq_i * wr[64+f] + dmean_f / N
  float4 dh[MAXT][4];
#pragma unroll
  for (int ti = 0; ti < MAXT; ++ti) {
    const int t = SCH[w + ti * NWAVE];
    const int r = t * 16 + c16;
#pragma unroll
    for (int c = 0; c < 4; ++c) dh[ti][c] = zero4();
    if (t < ntiles && r < rows_valid) {
      const int gl = r / N;
      const float dqi = DQ[r];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * c + 4 * s4;
        const float4 dm = f4(DMEAN + gl * 64 + f);
        dh[ti][c] = make_float4(fmaf(dqi, P[PK_WR + 64 + f + 0], dm.x), fmaf(dqi, P[PK_WR + 64 + f + 1], dm.y),
                                fmaf(dqi, P[PK_WR + 64 + f + 2], dm.z), fmaf(dqi, P[PK_WR + 64 + f + 3], dm.w));
      }
    }
  }
  // DQ (aliasing Mreg) is dead from here on; the next barrier orders it before the Z tiles

  // ---- update layers in reverse (mpnn.py:114-120) ----
  // Every Linear runs with the weight as the MFMA A operand (mm_k<.., true>): outputs arrive in the
  // node-operand layout (lane: node l&15, features 16c + 4(l>>4) + i), so the chain
  // duu -> [dh_direct, dm] -> dum -> [dagg, de] needs no transpose and rows are stored as float4.
  const uint16_t* BFP = reinterpret_cast<const uint16_t*>(P + PK_BF);
  for (int layer = 2; layer >= 0; --layer) {
    const float* WmT = P + PK_LAYERT + layer * 16384;  // [128][64]
    const float* WuT = WmT + 8192;                      // [128][64]
    // weights from L2 (no LDS staging): bf16x3-split transposed fragments, [out half][p][nt][kc2]
    const uint16_t* BFT = BFP + BFT_LAYER + layer * BF_LAYER_STRIDE;  // Wm^T halves, then Wu^T halves
    if constexpr (WLDS) {  // previous readers of Wl finished at the last barrier
      stage_rows<NT>(Wl, LDH, WuT, 64, 128, 64);
      stage_rows<NT>(Wl + 128 * LDH, LDH, WmT, 64, 128, 64);
      __syncthreads();
    }
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = SCH[w + ti * NWAVE];
      if (t < ntiles) {
        const int r = t * 16 + c16;
        const bool valid = r < rows_valid;
        const size_t ro = (R0 + r) * 64 + 4 * s4;
        // duu = dh' * [h' > 0]
        float4 duu[4], mv[4];
        const float* hnext = SV(SV_H0 + layer + 1) + ro;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 hv = valid ? f4(hnext + 16 * c) : zero4();
          mv[c] = valid ? f4(SV(SV_M0 + layer) + ro + 16 * c) : zero4();
          duu[c] = make_float4(hv.x > 0.f ? dh[ti][c].x : 0.f, hv.y > 0.f ? dh[ti][c].y : 0.f,
                               hv.z > 0.f ? dh[ti][c].z : 0.f, hv.w > 0.f ? dh[ti][c].w : 0.f);
          if (valid) st4(GR(GR_DUU0 + layer) + ro + 16 * c, duu[c]);
        }
        // [dh_direct, dm] = duu . Wu
        f32x4 d8[8];
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) d8[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (WLDS) mm_k<8, 4, true>(d8, duu, Wl, LDH, lane);
        else bf3_t2(d8, duu, BFT + 2 * BF_HALF, lane);
        // dum = dm * [m > 0]
        float4 dum[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          dum[c] = make_float4(mv[c].x > 0.f ? d8[4 + c][0] : 0.f, mv[c].y > 0.f ? d8[4 + c][1] : 0.f,
                               mv[c].z > 0.f ? d8[4 + c][2] : 0.f, mv[c].w > 0.f ? d8[4 + c][3] : 0.f);
          if (valid) {
            st4(GR(GR_DUM0 + layer) + ro + 16 * c, dum[c]);
            st4(GR(GR_DH) + ro + 16 * c, make_float4(d8[c][0], d8[c][1], d8[c][2], d8[c][3]));
          }
        }
        // [dagg, de] = dum . Wm;  G rows <- dagg / norm  (d(agg)/d(A.h) = 1/norm)
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) d8[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (WLDS) mm_k<8, 4, true>(d8, dum, Wl + 128 * LDH, LDH, lane);
        else bf3_t2(d8, dum, BFT, lane);
        const float nf = (float)row_info(RI, r).norm;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          st4(G + r * LDH + 16 * c + 4 * s4,
              valid ? make_float4(d8[c][0] / nf, d8[c][1] / nf, d8[c][2] / nf, d8[c][3] / nf) : zero4());
          if (valid) {
            float* de = GR(GR_DE) + ro + 16 * c;
            const float4 prev = layer == 2 ? zero4() : f4(de);
            st4(de, make_float4(prev.x + d8[4 + c][0], prev.y + d8[4 + c][1], prev.z + d8[4 + c][2],
                                prev.w + d8[4 + c][3]));
          }
        }
      }
    }
    __syncthreads();
    // dh_l = dh_direct + A^T . (dagg / norm)   (A symmetric: a gather over the node's own row)
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = SCH[w + ti * NWAVE];
      if (t < ntiles) {
        const int r = t * 16 + c16;
        const bool valid = r < rows_valid;
        const RowInfo ri = row_info(RI, r);
        float4 acc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = valid ? f4(GR(GR_DH) + (R0 + r) * 64 + 16 * c + 4 * s4) : zero4();
        gather_ri(ri, edges + (valid ? GB[r / N] : 0), G, (r / N) * N, s4, acc);
#pragma unroll
        for (int c = 0; c < 4; ++c) dh[ti][c] = acc[c];
      }
    }
    __syncthreads();
    ECO_TS(21 - layer);
  }

  // ---- h0 = relu(W0.x): du0 ----
#pragma unroll
  for (int ti = 0; ti < MAXT; ++ti) {
    const int t = SCH[w + ti * NWAVE];
    const int r = t * 16 + c16;
    if (t < ntiles && r < rows_valid) {
      const float* h0 = SV(SV_H0) + (R0 + r) * 64 + 4 * s4;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 hv = f4(h0 + 16 * c);
        st4(GR(GR_DU0) + (R0 + r) * 64 + 4 * s4 + 16 * c,
            make_float4(hv.x > 0.f ? dh[ti][c].x : 0.f, hv.y > 0.f ? dh[ti][c].y : 0.f,
                        hv.z > 0.f ? dh[ti][c].z : 0.f, hv.w > 0.f ? dh[ti][c].w : 0.f));
      }
    }
  }

  // ---- edge embedding (mpnn.py:89-104): due, dEagg ----
  if constexpr (WLDS) {  // Wf^T; the last layer's readers finished at the barrier above
    stage_rows<NT>(Wl, LDH, P + PK_WFT, 64, 64, 64);
    __syncthreads();
  }
#pragma unroll
  for (int ti = 0; ti < MAXT; ++ti) {
    const int t = SCH[w + ti * NWAVE];
    if (t < ntiles) {
      const int r = t * 16 + c16;
      const bool valid = r < rows_valid;
      float4 due[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const size_t off = (R0 + r) * 64 + 16 * c + 4 * s4;
        const float4 ev = valid ? f4(SV(SV_E) + off) : zero4();
        const float4 dv = valid ? f4(GR(GR_DE) + off) : zero4();
        due[c] = make_float4(ev.x > 0.f ? dv.x : 0.f, ev.y > 0.f ? dv.y : 0.f, ev.z > 0.f ? dv.z : 0.f,
                             ev.w > 0.f ? dv.w : 0.f);
        if (valid) st4(GR(GR_DUE) + off, due[c]);
      }
      f32x4 d4[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) d4[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (WLDS) mm_k<4, 4, true>(d4, due, Wl, LDH, lane);
      else mm_bf3_lean(d4, due, reinterpret_cast<const uint16_t*>(P + PK_BF) + BFT_WF, lane);
      const float nf = (float)row_info(RI, r).norm;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        st4(G + r * LDH + 16 * c + 4 * s4,
            valid ? make_float4(d4[c][0] / nf, d4[c][1] / nf, d4[c][2] / nf, d4[c][3] / nf) : zero4());
    }
  }
  __syncthreads();
  ECO_TS(22);
  // dz_j = sum_{i in N(j)} G_i * [w_ij wa + z_j > 0];  dwa += same * w_ij
  {
    float wa[16];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) wa[4 * c + i] = P[PK_WA + 16 * c + 4 * s4 + i];
    float dwa[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) dwa[i] = 0.f;
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = SCH[w + ti * NWAVE];
      if (t < ntiles) {
        const int r = t * 16 + c16;
        const bool valid = r < rows_valid;
        const RowInfo ri = row_info(RI, r);
        // z = Wx.x of the lane's node for its 16 features (same expression as forward phase A)
        float4 x0 = zero4(), x1 = zero4(), x2 = zero4(), x3 = zero4();
        if (valid) {
          const float* xr = (WLDS && !xwide) ? Xs + 8 * r : a.x + (R0 + r) * a.xw;
          x0 = f4(xr);
          x1 = f4(xr + 4);
          if (xwide) { x2 = f4(xr + 8); x3 = f4(xr + 12); }
        }
        float z[16], dz[16];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float* wx = P + PK_WX + (16 * c + 4 * s4 + i) * 8;
            const float4 w0 = f4(wx), w1 = f4(wx + 4);
            z[4 * c + i] = w0.x * x0.x + w0.y * x0.y + w0.z * x0.z + w0.w * x0.w + w1.x * x1.x + w1.y * x1.y +
                           w1.z * x1.z + w1.w * x1.w;
            if (xwide) {  // same left-to-right order as the forward's xdot_hi term
              const float* wh = P + PK_WXH + (16 * c + 4 * s4 + i) * 8;
              const float4 h0 = f4(wh), h1 = f4(wh + 4);
              z[4 * c + i] += h0.x * x2.x + h0.y * x2.y + h0.z * x2.z + h0.w * x2.w + h1.x * x3.x + h1.y * x3.y +
                              h1.z * x3.z + h1.w * x3.w;
            }
          }
#pragma unroll
        for (int i = 0; i < 16; ++i) dz[i] = 0.f;
        const int rbase = (r / N) * N;
        for_edges(edges + (valid ? GB[r / N] : 0), ri.e0, ri.e1, [&](uint32_t ex) {
          const float wv = (float)edge_w(ex);
          const float* gi = G + (rbase + edge_col(ex)) * LDH + 4 * s4;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float4 gv = f4(gi + 16 * c);
            const float g4[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int kk = 4 * c + i;
              const float gm = fmaf(wv, wa[kk], z[kk]) > 0.f ? g4[i] : 0.f;
              dz[kk] += gm;
              dwa[kk] = fmaf(gm, wv, dwa[kk]);
            }
          }
        });
        if (valid) {
          float* dzp = GR(GR_DZ) + (R0 + r) * 64 + 4 * s4;
#pragma unroll
          for (int c = 0; c < 4; ++c) st4(dzp + 16 * c, make_float4(dz[4 * c], dz[4 * c + 1], dz[4 * c + 2], dz[4 * c + 3]));
        }
      }
    }
    // reduce dwa over the 16 node lanes sharing s4, then over waves (fixed order)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float v = dwa[i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      dwa[i] = v;
    }
    if (c16 == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) RED[w * 64 + 16 * c + 4 * s4 + i] = dwa[4 * c + i];
    }
    __syncthreads();
    if (w == 0) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < NWAVE; ++k) s += RED[k * 64 + lane];
      DWA[(size_t)blk * 64 + lane] = s;
    }
  }
  ECO_TS(23);
}

// ======================================================== large graphs ====
// N > 512 (GSet G22, N = 2000; inference / best-cut search only): the node embeddings no longer fit
// LDS, so each episode's Z / h rows live in global memory (two ping-pong [rows][64] f32 buffers and the
// edge embedding e, in the forward workspace: per episode 3 x rows x 256 B, L2/MALL-resident while the
// workgroup runs).  One workgroup per episode; waves take 16-node tiles round-robin; the
// aggregations are CSR gathers from global rows in the MFMA operand layout; the Linears are the same
// exact-f32 MFMA tiles as the LDS kernels with both layer weights staged in LDS (8 waves: the gathers
// and the 8-chunk Linears need more than the 128 VGPRs of a 16-wave workgroup).
// LDS: Wl [2][64][LDW] | readout scratch
template <int NW>
__global__ __launch_bounds__(64 * NW, 2) void mpnn_forward_large_kernel(MpnnArgs a, float* hbuf) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  ws_invalidate_key(a.call_maxdeg);  // hbuf overwrites the cached shared-graph tables
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int e = blockIdx.x;
  const int N = a.N;
  const int rows_pad = (N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  const size_t R0 = (size_t)e * N;
  const size_t RT = (size_t)a.B * N;
  // Linears on the exact bf16x3-split weight fragments streamed from L2 (no LDS weight staging: the
  // LDS holds only the readout scratch, so two episodes share a CU and hide each other's gathers)
  const uint16_t* BFP = reinterpret_cast<const uint16_t*>(a.P + PK_BF);
  float* Scr = lds;
  float* HA = hbuf + (size_t)e * rows_pad * 64 * 3;
  float* HB = HA + (size_t)rows_pad * 64;
  float* EB = HB + (size_t)rows_pad * 64;
  const float* P = a.P;
  const int s4 = lane >> 4;
  const int c16 = lane & 15;
  const int gid = a.gids[e];
  const uint32_t* __restrict__ eg = a.gs.edges + a.gs.edge_base[gid];
  const float* x = a.x + R0 * 8;
  auto rinfo = [&](int r) { return row_info_packed(pack_row_info(a, e, r, N)); };

  // ---- phase A: Z = Wx . x into HB ----
  {
    float wx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) wx[k] = P[PK_WX + lane * 8 + k];
    for (int r = w; r < rows_pad; r += NW) {
      float z = 0.f;
      if (r < N) {
        const float4 x0 = f4(x + r * 8), x1 = f4(x + r * 8 + 4);
        z = wx[0] * x0.x + wx[1] * x0.y + wx[2] * x0.z + wx[3] * x0.w + wx[4] * x1.x + wx[5] * x1.y +
            wx[6] * x1.z + wx[7] * x1.w;
      }
      HB[(size_t)r * 64 + lane] = z;
    }
  }
  __threadfence();
  __syncthreads();
  // ---- phase B: edge embedding (mpnn.py:89-104) -> EB; phase C: h0 = relu(W0 . x) -> HA ----
  {
    const int maxdeg_call = a.norm_scope == ECO_NORM_PER_CALL ? *a.call_maxdeg : a.gs.max_deg[gid];
    float wa[16];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) wa[c * 4 + i] = P[PK_WA + 16 * c + 4 * s4 + i];
    for (int t = w; t < ntiles; t += NW) {
      const int r = t * 16 + c16;
      const bool valid = r < N;
      const RowInfo ri = rinfo(r);
      float4 acc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = zero4();
      for_edges(eg, ri.e0, ri.e1, [&](uint32_t ex) {
        const float wv = (float)edge_w(ex);
        const float* zr = HB + (size_t)edge_col(ex) * 64 + 4 * s4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 z = f4(zr + 16 * c);
          acc[c].x += relu(fmaf(wv, wa[4 * c + 0], z.x));
          acc[c].y += relu(fmaf(wv, wa[4 * c + 1], z.y));
          acc[c].z += relu(fmaf(wv, wa[4 * c + 2], z.z));
          acc[c].w += relu(fmaf(wv, wa[4 * c + 3], z.w));
        }
      });
      const float nf = (float)ri.norm;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c].x = acc[c].x / nf; acc[c].y = acc[c].y / nf; acc[c].z = acc[c].z / nf; acc[c].w = acc[c].w / nf;
      }
      if (s4 == 3) acc[3].w = nf / (float)maxdeg_call;  // norm / norm.max() (mpnn.py:102)
      if (!valid) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = zero4();
      }
      f32x4 d[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      mm_bf3_lean(d, acc, BFP + BF_WF, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) st4(EB + (size_t)r * 64 + 16 * nt + 4 * s4, relu4(d[nt]));
    }
    float w0[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w0[k] = P[PK_W0 + lane * 8 + k];
    for (int r = w; r < rows_pad; r += NW) {
      float h0 = 0.f;
      if (r < N) {
        const float4 x0 = f4(x + r * 8), x1 = f4(x + r * 8 + 4);
        h0 = relu(w0[0] * x0.x + w0[1] * x0.y + w0[2] * x0.z + w0[3] * x0.w + w0[4] * x1.x + w0[5] * x1.y +
                  w0[6] * x1.z + w0[7] * x1.w);
      }
      HA[(size_t)r * 64 + lane] = h0;
    }
  }
  __threadfence();
  __syncthreads();
  // ---- phase D: 3 x UpdateNodeEmbeddingLayer (mpnn.py:114-120), HA <-> HB ----
  float* Hc = HA;
  float* Hn = HB;
  for (int layer = 0; layer < 3; ++layer) {
    const uint16_t* BFL = BFP + BF_LAYER + layer * BF_LAYER_STRIDE;  // message halves, then update halves
    for (int t = w; t < ntiles; t += NW) {
      const int r = t * 16 + c16;
      const bool valid = r < N;
      const RowInfo ri = rinfo(r);
      float4 am[4], ev[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) am[c] = zero4();
      for_edges(eg, ri.e0, ri.e1, [&](uint32_t ex) {
        const float wv = (float)edge_w(ex);
        const float* hr = Hc + (size_t)edge_col(ex) * 64 + 4 * s4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 hv = f4(hr + 16 * c);
          am[c].x = fmaf(wv, hv.x, am[c].x);
          am[c].y = fmaf(wv, hv.y, am[c].y);
          am[c].z = fmaf(wv, hv.z, am[c].z);
          am[c].w = fmaf(wv, hv.w, am[c].w);
        }
      });
      const float nf = (float)ri.norm;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        am[c].x = am[c].x / nf; am[c].y = am[c].y / nf; am[c].z = am[c].z / nf; am[c].w = am[c].w / nf;
        ev[c] = f4(EB + (size_t)r * 64 + 16 * c + 4 * s4);
      }
      f32x4 d[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      mm_bf3_lean(d, am, BFL, lane);             // message = relu(Wm . [agg, e])
      mm_bf3_lean(d, ev, BFL + BF_HALF, lane);
      float4 hc[4], mr[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        hc[c] = f4(Hc + (size_t)r * 64 + 16 * c + 4 * s4);
        mr[c] = relu4(d[c]);
      }
      f32x4 hn[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) hn[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      mm_bf3_lean(hn, hc, BFL + 2 * BF_HALF, lane);  // h' = relu(Wu . [h, m])
      mm_bf3_lean(hn, mr, BFL + 3 * BF_HALF, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) st4(Hn + (size_t)r * 64 + 16 * nt + 4 * s4, valid ? relu4(hn[nt]) : zero4());
    }
    __threadfence();  // release the Hn rows and invalidate this CU's L1 before other waves read them
    __syncthreads();  // every wave done with Hc; Hn complete
    float* tmp = Hc;
    Hc = Hn;
    Hn = tmp;
  }
  // ---- phase E: readout + act over the h3 rows in global memory ----
  readout_act<false, NW>(a, Hc, 64, Scr, true, e, 1, N, R0, RT);
}

// norm.max() of the call (mpnn.py:102 over every graph of the batch): ONE workgroup reduces all B graph
// ids and writes the result (no zeroing memset, no atomics)
__global__ __launch_bounds__(1024) void call_maxdeg_kernel(const eco_graph_set gs, const int32_t* gids, int B,
                                                           int* out) {
  __shared__ int red[16];
  int m = 1;
  for (int i = threadIdx.x; i < B; i += blockDim.x) m = max(m, gs.max_deg[gids[i]]);
  m = wave_max_i(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    int r = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = max(r, red[w]);
    *out = r;
  }
}

static int prepare(MpnnArgs& a, const float* packed, int32_t n_obs_in, const eco_graph_set* gs,
                   const int32_t* graph_ids, int32_t batch, const float* obs_x, int32_t norm_scope) {
  if (!packed || !gs || !graph_ids || !obs_x) return fail(ECO_ERR_ARG, "null argument");
  if (n_obs_in < 1 || n_obs_in > ECO_MPNN_MAX_OBS) return fail(ECO_ERR_ARG, "n_obs_in out of range [1, 16]");
  if (batch < 1) return fail(ECO_ERR_ARG, "batch must be >= 1");
  const int N = gs->n_spins;
  if (N < 1 || N > MPNN_MAX_SPINS_LARGE) return fail(ECO_ERR_ARG, "mpnn supports 1 <= N <= 2048");
  if (norm_scope != ECO_NORM_PER_GRAPH && norm_scope != ECO_NORM_PER_CALL)
    return fail(ECO_ERR_ARG, "bad norm_scope");
  a = MpnnArgs{};
  a.P = packed; a.gs = *gs; a.gids = graph_ids; a.B = batch; a.N = N; a.gpb = graphs_per_block(N, batch);
  a.nobs = n_obs_in; a.xw = ECO_OBS_X_STRIDE(n_obs_in); a.x = obs_x; a.norm_scope = norm_scope;
  if (a.xw != 8 && N > MPNN_MAX_SPINS)
    return fail(ECO_ERR_ARG, "more than 8 node features need N <= 512 (the N > 512 kernel takes 8-float rows)");
  a.err = err_word();
  return ECO_OK;
}

}  // namespace eco

using namespace eco;

#ifdef ECO_PHASE_TIMING
extern "C" int eco_debug_phase_ts(unsigned long long* host, int32_t n) {
  if (n > ECO_TS_BLOCKS * 32) n = ECO_TS_BLOCKS * 32;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(eco_phase_ts), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" size_t eco_mpnn_param_count(int32_t n_obs_in) {
  if (n_obs_in < 1 || n_obs_in > ECO_MPNN_MAX_OBS) return 0;
  return (size_t)flat_offsets(n_obs_in).total;
}

extern "C" size_t eco_mpnn_packed_count(void) { return (size_t)PK_TOTAL; }

extern "C" int eco_mpnn_pack(const float* params, int32_t n_obs_in, float* packed, eco_stream_t stream) {
  if (!params || !packed) return fail(ECO_ERR_ARG, "null params/packed");
  if (n_obs_in < 1 || n_obs_in > ECO_MPNN_MAX_OBS) return fail(ECO_ERR_ARG, "n_obs_in out of range [1, 16]");
  pack_scale_kernel<<<FH_NMAT, PS_THREADS, 0, (hipStream_t)stream>>>(params, n_obs_in, packed);
  pack_kernel<<<(PK_TOTAL + 255) / 256, 256, 0, (hipStream_t)stream>>>(params, n_obs_in, packed);
  return check_launch("mpnn_pack");
}

extern "C" size_t eco_mpnn_workspace_bytes(int32_t n_spins, int32_t batch) {
  if (n_spins < 1 || batch < 1) return 0;
  if (n_spins > MPNN_MAX_SPINS) {  // + per episode Z/h ping-pong rows and e rows (mpnn_forward_large_kernel),
                                  // or the node-major buffers of the shared-graph path, whichever is larger
    const size_t per_ep = (size_t)batch * ((n_spins + 15) & ~15) * 64 * 3 * sizeof(float);
    const size_t shared = shared_ws_bytes(n_spins, batch);
    return 256 + (per_ep > shared ? per_ep : shared);
  }
  if (n_spins > DN_MAX_ROWS)  // + the edge embeddings of the dense kernels for 224 < N <= 512
    return 256 + (size_t)batch * n_spins * 64 * sizeof(float);
  return 256;  // the call-scope norm.max() slot
}

extern "C" size_t eco_mpnn_saved_bytes(int32_t n_spins, int32_t batch) {
  if (n_spins < 1 || batch < 1) return 0;
  const size_t RT = (size_t)n_spins * batch;
  return sv_mask_offset_floats(RT, batch) * sizeof(float) + RT * 4 * SM_TENSORS * sizeof(uint16_t);
}

static std::atomic<int> g_kernel_paths{0};
int eco::kernel_paths() { return g_kernel_paths.load(std::memory_order_relaxed); }

extern "C" int32_t eco_set_kernel_paths(int32_t mask) {
  return g_kernel_paths.exchange(mask & (ECO_PATH_NO_DENSE | ECO_PATH_NO_DL | ECO_PATH_NO_SHARED | ECO_PATH_NO_PAIR |
                                         ECO_PATH_DENSE2_FWD));
}

struct KCfg {
  int nw, maxt;
  bool wlds;
  size_t lds;
};
constexpr size_t LDS_MAX = 160 * 1024;

static size_t lds_bytes(int rows_pad, int gpb, int nw, bool wlds, bool backward) {
  size_t f = (size_t)rows_pad * LDH;
  if (backward) {
    if (wlds) f += (size_t)2 * 128 * LDH + (size_t)rows_pad * 8;  // Wu^T, Wm^T + x rows
    f += (size_t)rows_pad * 2 + 2 * (size_t)gpb;               // packed row info + per-graph edge base
    f += (size_t)gpb * 64 + (size_t)(gpb < nw ? gpb : 1) * nw * 64 + 64;  // + tile schedule
  } else {
    if (wlds) f += (size_t)2 * 64 * LDW;
    f += (size_t)fwd_mreg_floats(rows_pad, gpb, nw, wlds);
    f += (size_t)rows_pad * 2 + 3 * (size_t)gpb + 2 + 64;  // row info, edge base, max degree, tile schedule
  }
  return f * sizeof(float);
}

// 8 waves with LDS-staged weights when the block fits, else 4 waves (weights from L2).
static KCfg pick_cfg(int N, int gpb, bool backward) {
  const int rows_pad = (gpb * N + 15) & ~15;
  const int ntiles = rows_pad / 16;
  KCfg c;
  constexpr int force_nw = 0;  // (A/B builds of round 2 forced the wave count here)
  for (int nw : {16, 8, 4}) {
    if (force_nw && nw != force_nw && nw != 4) continue;
    if (backward && nw == 16) continue;  // the backward's 8-wide weight fragments need > 128 VGPRs
    c.nw = nw;
    c.wlds = true;
    c.lds = lds_bytes(rows_pad, gpb, nw, true, backward);
    c.maxt = (ntiles + nw - 1) / nw;
    if (c.lds <= LDS_MAX && c.maxt <= (nw == 16 ? 1 : 4)) return c;
  }
  // weights from L2, 8 waves (2 per SIMD: the block owns the CU through its LDS) when 4 tiles per
  // wave suffice; measured at BA-500: forward 15 % faster than 4 waves x 8 tiles, backward slower
  if (!force_nw || force_nw == 8) {
    c.nw = 8;
    c.wlds = false;
    c.lds = lds_bytes(rows_pad, gpb, 8, false, backward);
    c.maxt = (ntiles + 7) / 8;
    if (c.lds <= LDS_MAX && c.maxt <= 4) return c;
  }
  c.nw = 4;
  c.wlds = false;
  c.lds = lds_bytes(rows_pad, gpb, 4, false, backward);
  c.maxt = (ntiles + 3) / 4;
  return c;
}

extern "C" int eco_mpnn_forward_pair(const float* packed_a, const float* packed_b, int32_t n_obs_in,
                                     const eco_graph_set* gs, const int32_t* graph_ids, int32_t batch,
                                     const float* obs_x, int32_t norm_scope, float* q_a, const eco_act_config* act_a,
                                     int32_t* actions_a, float* q_b, const eco_act_config* act_b, int32_t* actions_b,
                                     void* workspace, eco_stream_t stream) {
  if (!packed_b) return fail(ECO_ERR_ARG, "null argument");
  const bool reuse_maxdeg = norm_scope == ECO_NORM_PER_CALL_REUSE;
  if (reuse_maxdeg) norm_scope = ECO_NORM_PER_CALL;
  MpnnArgs a;
  int rc = prepare(a, packed_a, n_obs_in, gs, graph_ids, batch, obs_x, norm_scope);
  if (rc) return rc;
  if (!workspace) return fail(ECO_ERR_ARG, "null workspace");
  if ((act_a && !actions_a) || (act_b && !actions_b)) return fail(ECO_ERR_ARG, "act config without actions buffer");
  if ((!q_a && !act_a) || (!q_b && !act_b)) return fail(ECO_ERR_ARG, "nothing to compute (q and act both null)");
  const int paths = kernel_paths();
  if ((paths & (ECO_PATH_NO_PAIR | ECO_PATH_NO_DENSE)) ||
      !(a.xw == 8 && dense_eligible(gs, a.gpb) && a.gpb == 1 && gs->adjbits)) {
    rc = eco_mpnn_forward(packed_a, n_obs_in, gs, graph_ids, batch, obs_x,
                          reuse_maxdeg ? ECO_NORM_PER_CALL_REUSE : norm_scope, q_a, act_a, actions_a, nullptr,
                          workspace, stream);
    if (rc) return rc;
    return eco_mpnn_forward(packed_b, n_obs_in, gs, graph_ids, batch, obs_x,
                            norm_scope == ECO_NORM_PER_GRAPH ? norm_scope : ECO_NORM_PER_CALL_REUSE, q_b, act_b,
                            actions_b, nullptr, workspace, stream);
  }
  hipStream_t st = (hipStream_t)stream;
  int* cmax = (int*)workspace;
  a.call_maxdeg = cmax;
  a.sv = nullptr;
  MpnnArgs b = a;
  a.q = q_a;
  a.has_act = act_a != nullptr;
  if (act_a) a.act = *act_a;
  a.actions = actions_a;
  b.P = packed_b;
  b.q = q_b;
  b.has_act = act_b != nullptr;
  if (act_b) b.act = *act_b;
  b.actions = actions_b;
  if (norm_scope == ECO_NORM_PER_CALL && !reuse_maxdeg)
    call_maxdeg_kernel<<<1, 1024, 0, st>>>(*gs, graph_ids, batch, cmax);
  if (paths & ECO_PATH_DENSE2_FWD) return mpnn_forward_dense2_pair_launch(a, b, st);
  return mpnn_forward_dense3_pair_launch(a, b, st);
}

extern "C" int eco_mpnn_forward(const float* packed, int32_t n_obs_in, const eco_graph_set* gs,
                                const int32_t* graph_ids, int32_t batch, const float* obs_x, int32_t norm_scope,
                                float* q, const eco_act_config* act, int32_t* actions, void* saved, void* workspace,
                                eco_stream_t stream) {
  const bool reuse_maxdeg = norm_scope == ECO_NORM_PER_CALL_REUSE;  // the workspace already holds the call max
  if (reuse_maxdeg) norm_scope = ECO_NORM_PER_CALL;
  MpnnArgs a;
  int rc = prepare(a, packed, n_obs_in, gs, graph_ids, batch, obs_x, norm_scope);
  if (rc) return rc;
  if (!workspace) return fail(ECO_ERR_ARG, "null workspace");
  if (act && !actions) return fail(ECO_ERR_ARG, "act config without actions buffer");
  if (!q && !act) return fail(ECO_ERR_ARG, "nothing to compute (q and act both null)");
  hipStream_t st = (hipStream_t)stream;
  const int N = a.N;
  a.q = q;
  int* cmax = (int*)workspace;
  a.call_maxdeg = cmax;
  a.sv = (float*)saved;
  a.has_act = act != nullptr;
  if (act) a.act = *act;
  a.actions = actions;
  if (norm_scope == ECO_NORM_PER_CALL && !reuse_maxdeg) {
    call_maxdeg_kernel<<<1, 1024, 0, st>>>(*gs, graph_ids, batch, cmax);
  }
  const int paths = kernel_paths();
  if (a.xw == 8 && dense_eligible(gs, a.gpb) && !(paths & ECO_PATH_NO_DENSE)) {
    if (paths & ECO_PATH_DENSE2_FWD) return mpnn_forward_dense2_launch(a, saved != nullptr, st);
    return mpnn_forward_dense3_launch(a, saved != nullptr, st);
  }
  if (a.xw == 8 && dl_eligible(gs, a.gpb) && !(paths & (ECO_PATH_NO_DL | ECO_PATH_NO_DENSE)))
    return mpnn_forward_dl_launch(a, saved != nullptr, workspace, st);
  if (N > MPNN_MAX_SPINS) {  // global-memory embeddings: inference only
    if (saved) return fail(ECO_ERR_ARG, "training forward (saved activations) supports N <= 512");
    // one graph shared by every episode (GSet best-cut search): node-major episode-batched kernels
    if (gs->n_graphs == 1 && gs->unit_weights && !(paths & ECO_PATH_NO_SHARED))
      return mpnn_forward_shared_launch(a, workspace, st);
    const int rows_pad = (N + 15) & ~15;
    const size_t lds = (size_t)readout_scratch_floats(rows_pad, 1, 8, true) * sizeof(float);
    (void)hipFuncSetAttribute((const void*)mpnn_forward_large_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    mpnn_forward_large_kernel<8><<<batch, 512, lds, st>>>(a, (float*)((char*)workspace + 256));
    return check_launch("mpnn_forward_large");
  }
  const int blocks = (batch + a.gpb - 1) / a.gpb;
  const KCfg k = pick_cfg(N, a.gpb, false);
  if (k.lds > LDS_MAX) return fail(ECO_ERR_ARG, "graph block exceeds the LDS budget");
#define ECO_LAUNCH_FWD(MT, SV, NW, WL)                                                                          \
  do {                                                                                                         \
    (void)hipFuncSetAttribute((const void*)mpnn_forward_kernel<MT, SV, NW, WL>,                                \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)k.lds);                        \
    mpnn_forward_kernel<MT, SV, NW, WL><<<blocks, 64 * NW, k.lds, st>>>(a);                                   \
  } while (0)
#define ECO_LAUNCH_FWD2(MT, NW, WL) \
  do { if (saved) ECO_LAUNCH_FWD(MT, true, NW, WL); else ECO_LAUNCH_FWD(MT, false, NW, WL); } while (0)
  if (k.wlds && k.nw == 16 && k.maxt <= 1) ECO_LAUNCH_FWD2(1, 16, true);
  else if (k.wlds && k.nw == 8 && k.maxt <= 2) ECO_LAUNCH_FWD2(2, 8, true);
  else if (k.wlds && k.nw == 8) ECO_LAUNCH_FWD2(4, 8, true);
  else if (k.wlds && k.maxt <= 4) ECO_LAUNCH_FWD2(4, 4, true);
  else if (k.nw == 8 && k.maxt <= 4) ECO_LAUNCH_FWD2(4, 8, false);
  else if (k.maxt <= 4) ECO_LAUNCH_FWD2(4, 4, false);
  else if (k.maxt <= 8) ECO_LAUNCH_FWD2(8, 4, false);
  else return fail(ECO_ERR_ARG, "graph block too large");
#undef ECO_LAUNCH_FWD2
#undef ECO_LAUNCH_FWD
  return check_launch("mpnn_forward");
}

size_t eco::mpnn_grad_ws_bytes(int32_t n_spins, int32_t batch) {
  if (n_spins < 1 || batch < 1) return 0;
  const int gpb = graphs_per_block(n_spins, batch);
  const size_t nblk = (batch + gpb - 1) / gpb;
  return ((size_t)GR_NODE_TENSORS * n_spins * batch * 64 + 3 * (size_t)batch * 64 + (((size_t)batch + 63) & ~63ull) +
          nblk * 64) * sizeof(float);
}

int eco::mpnn_backward_launch(const float* packed, int32_t n_obs_in, const eco_graph_set* gs,
                              const int32_t* graph_ids, int32_t batch, const float* obs_x, const void* saved,
                              const float* dq, void* gradws, hipStream_t st) {
  MpnnArgs a;
  int rc = prepare(a, packed, n_obs_in, gs, graph_ids, batch, obs_x, ECO_NORM_PER_CALL);
  if (rc) return rc;
  if (!saved || !dq || !gradws) return fail(ECO_ERR_ARG, "null saved/dq/workspace");
  if (a.N > MPNN_MAX_SPINS) return fail(ECO_ERR_ARG, "MPNN backward supports N <= 512");
  a.sv = (float*)saved;
  a.dq = dq;
  a.gr = (float*)gradws;
  const int paths = kernel_paths();
  if (a.xw == 8 && dense_eligible(gs, a.gpb) && !(paths & ECO_PATH_NO_DENSE)) {
    if (paths & ECO_PATH_DENSE2_FWD) return mpnn_backward_dense2_launch(a, st);
    return mpnn_backward_dense3_launch(a, st);
  }
  if (a.xw == 8 && dl_eligible(gs, a.gpb) && !(paths & (ECO_PATH_NO_DL | ECO_PATH_NO_DENSE)))
    return mpnn_backward_dl_launch(a, st);
  const int blocks = (batch + a.gpb - 1) / a.gpb;
  const KCfg k = pick_cfg(a.N, a.gpb, true);
  if (k.lds > LDS_MAX) return fail(ECO_ERR_ARG, "graph block exceeds the LDS budget");
#define ECO_LAUNCH_BWD(MT, NW, WL)                                                                              \
  do {                                                                                                         \
    (void)hipFuncSetAttribute((const void*)mpnn_backward_kernel<MT, NW, WL>,                                   \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)k.lds);                        \
    mpnn_backward_kernel<MT, NW, WL><<<blocks, 64 * NW, k.lds, st>>>(a);                                      \
  } while (0)
  if (k.wlds && k.nw == 8 && k.maxt <= 2) ECO_LAUNCH_BWD(2, 8, true);
  else if (k.wlds && k.nw == 8) ECO_LAUNCH_BWD(4, 8, true);
  else if (k.wlds && k.maxt <= 4) ECO_LAUNCH_BWD(4, 4, true);
  else if (k.nw == 8 && k.maxt <= 4) ECO_LAUNCH_BWD(4, 8, false);
  else if (k.maxt <= 4) ECO_LAUNCH_BWD(4, 4, false);
  else if (k.maxt <= 8) ECO_LAUNCH_BWD(8, 4, false);
  else return fail(ECO_ERR_ARG, "graph block too large");
#undef ECO_LAUNCH_BWD
  return check_launch("mpnn_backward");
}

// ---- split2_pk hazard probe (the v_fma_mix inline asm carries its own wait states) ----
namespace eco {
// One wave per 64 x 32 block of activations: the lane's four float4 split by split2_pk (inline asm) and fed to
// MFMAs exactly as mm_fh feeds them (order 0), with the lo fragment consumed first, straight after the asm (order
// 1), or with the split and that first MFMA in one asm block, the MFMA reading the register the last v_fma_mixhi
// wrote right after the product's wait states (order 2: the only schedule where nothing else can supply them, so
// a build without them -- ECO_SPLIT2_NEGATIVE_CONTROL -- must fail); the same products from the plain-conversion
// split (split2_ref).  out[2][block][4 x 16 outputs][64 lanes] fp32 accumulators, compared bitwise by the test.
template <bool REF>
__device__ __forceinline__ void probe_split_fh(const float4& a, const float4& b, float sf, f16x8& hi, f16x8& lo) {
  uint32_t h[4], l[4];
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (REF) split2_ref(v[2 * t], v[2 * t + 1], sf, h[t], l[t]);
    else split2_pk(v[2 * t], v[2 * t + 1], sf, h[t], l[t]);
  }
  const u32x4v hv = {h[0], h[1], h[2], h[3]}, lv = {l[0], l[1], l[2], l[3]};
  hi = __builtin_bit_cast(f16x8, hv);
  lo = __builtin_bit_cast(f16x8, lv);
}
template <bool REF, int ORDER>
__device__ __forceinline__ void probe_mm(f32x4 (&acc)[4], const float4 (&x)[4], float sf, const uint16_t* WH,
                                         int lane) {
  const uint16_t* wl = WH + lane * 8;
#pragma unroll
  for (int kc2 = 0; kc2 < 2; ++kc2) {
    f16x8 w1[4], w2[4];  // weight fragments read first: nothing but the split sits between it and the MFMAs
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      w1[nt] = *reinterpret_cast<const f16x8*>(wl + ((0 * 4 + nt) * 2 + kc2) * FH_FRAG);
      w2[nt] = *reinterpret_cast<const f16x8*>(wl + ((1 * 4 + nt) * 2 + kc2) * FH_FRAG);
    }
    if (ORDER >= 1) {
      // order 1 places the lo fragment's first reader straight after the split's last v_fma_mixhi: all loads
      // drained and earlier MFMAs retired first (nothing for the compiler to interleave), then that first
      // MFMA as inline asm (so no compiler-inserted wait state can separate it from the asm split), followed by
      // enough s_nop for every MFMA result hazard the recognizer cannot see through asm
      __builtin_amdgcn_s_waitcnt(0);
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    f16x8 xh, xl;
    if (ORDER == 2 && !REF) {
      // order 2: the split's eight v_fma_mix (the product's asm text and wait states, ECO_MIXLO / ECO_MIXHI /
      // ECO_SPLIT2_WAIT) and the first MFMA reading its lo fragment in ONE asm block with fixed registers, the MFMA
      // straight after the v_fma_mixhi that wrote its last operand register: nothing the compiler schedules can
      // separate them, so only ECO_SPLIT2_WAIT stands between the write and the read.  The lo pieces are then
      // copied out for the remaining MFMAs.
      const float v[8] = {x[2 * kc2].x, x[2 * kc2].y, x[2 * kc2].z, x[2 * kc2].w,
                          x[2 * kc2 + 1].x, x[2 * kc2 + 1].y, x[2 * kc2 + 1].z, x[2 * kc2 + 1].w};
      uint32_t h[4], l[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) h[t] = pk_f16(v[2 * t] * sf, v[2 * t + 1] * sf);
      asm volatile("s_nop 4\n\t"  // the compiler's VALU writes of h / v before this asm (reads by VALU: none needed)
                   ECO_MIXLO("v200", "%[a0]", "%[sf]", "%[h0]") "\n\t" ECO_MIXLO("v201", "%[a2]", "%[sf]", "%[h1]") "\n\t"
                   ECO_MIXLO("v202", "%[a4]", "%[sf]", "%[h2]") "\n\t" ECO_MIXLO("v203", "%[a6]", "%[sf]", "%[h3]") "\n\t"
                   ECO_MIXHI("v200", "%[a1]", "%[sf]", "%[h0]") "\n\t" ECO_MIXHI("v201", "%[a3]", "%[sf]", "%[h1]") "\n\t"
                   ECO_MIXHI("v202", "%[a5]", "%[sf]", "%[h2]") "\n\t" ECO_MIXHI("v203", "%[a7]", "%[sf]", "%[h3]")
                   ECO_SPLIT2_WAIT "\n\t"
                   "v_mfma_f32_16x16x32_f16 %[acc], %[w], v[200:203], %[acc]\n\t"
                   "v_mov_b32 %[l0], v200\n\tv_mov_b32 %[l1], v201\n\tv_mov_b32 %[l2], v202\n\tv_mov_b32 %[l3], v203\n\t"
                   "s_nop 7\n\ts_nop 7\n\ts_nop 3"
                   : [acc] "+v"(acc[0]), [l0] "=&v"(l[0]), [l1] "=&v"(l[1]), [l2] "=&v"(l[2]), [l3] "=&v"(l[3])
                   : [w] "v"(w1[0]), [sf] "v"(sf), [h0] "v"(h[0]), [h1] "v"(h[1]), [h2] "v"(h[2]), [h3] "v"(h[3]),
                     [a0] "v"(v[0]), [a1] "v"(v[1]), [a2] "v"(v[2]), [a3] "v"(v[3]), [a4] "v"(v[4]), [a5] "v"(v[5]),
                     [a6] "v"(v[6]), [a7] "v"(v[7])
                   : "v200", "v201", "v202", "v203");
      const u32x4v hv = {h[0], h[1], h[2], h[3]}, lv = {l[0], l[1], l[2], l[3]};
      xh = __builtin_bit_cast(f16x8, hv);
      xl = __builtin_bit_cast(f16x8, lv);
      __builtin_amdgcn_sched_barrier(0);
    } else {
      probe_split_fh<REF>(x[2 * kc2], x[2 * kc2 + 1], sf, xh, xl);
    }
    if (ORDER == 2 && REF) {  // the same first product from the plain split (compiler VALU: wait states written out)
      asm volatile("s_nop 4\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3"
                   : "+v"(acc[0])
                   : "v"(w1[0]), "v"(xl));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (ORDER == 1) {
      // (the plain-conversion reference split is compiler VALU code: its wait states before this asm MFMA are
      // written out here, the recognizer not knowing the asm is an MFMA; the asm split carries its own)
      if (REF)
        asm volatile("s_nop 4\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3"
                     : "+v"(acc[0])
                     : "v"(w1[0]), "v"(xl));
      else
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3"
                     : "+v"(acc[0])
                     : "v"(w1[0]), "v"(xl));
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      if (ORDER >= 1 && nt == 0) {
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[0], xh, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[0], xh, acc[0], 0, 0, 0);
      } else if (ORDER == 0) {  // mm_fh
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[nt], xh, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[nt], xl, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[nt], xh, acc[nt], 0, 0, 0);
      } else {
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[nt], xl, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[nt], xh, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[nt], xh, acc[nt], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
template <int ORDER>
__global__ __launch_bounds__(256) void split2_probe_kernel(const float* x, const float* sf, const uint16_t* W,
                                                           float* out, int n_blocks) {
  __shared__ __attribute__((aligned(16))) uint16_t sWH[FH_HALF];
  for (int i = threadIdx.x; i < FH_HALF / 8; i += 256)
    reinterpret_cast<uint4*>(sWH)[i] = reinterpret_cast<const uint4*>(W)[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= n_blocks) return;  // whole waves
  float4 xv[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) xv[c] = f4(x + ((size_t)blk * 64 + lane) * 16 + 4 * c);
  const float s = sf[blk];
  f32x4 a[4], r[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) a[nt] = r[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  probe_mm<false, ORDER>(a, xv, s, sWH, lane);
  probe_mm<true, ORDER>(r, xv, s, sWH, lane);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[(((size_t)0 * n_blocks + blk) * 16 + nt * 4 + i) * 64 + lane] = a[nt][i];
      out[(((size_t)1 * n_blocks + blk) * 16 + nt * 4 + i) * 64 + lane] = r[nt][i];
    }
}
}  // namespace eco

extern "C" int eco_probe_split2_mfma(const float* x, const float* sf, const uint16_t* w_frags, int32_t n_blocks,
                                     int32_t order, float* out, eco_stream_t stream) {
  using namespace eco;
  if (!x || !sf || !w_frags || !out || n_blocks < 1 || order < 0 || order > 2)
    return fail(ECO_ERR_ARG, "eco_probe_split2_mfma: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const int grid = (n_blocks + 3) / 4;
  if (order == 0) split2_probe_kernel<0><<<grid, 256, 0, st>>>(x, sf, w_frags, out, n_blocks);
  else if (order == 1) split2_probe_kernel<1><<<grid, 256, 0, st>>>(x, sf, w_frags, out, n_blocks);
  else split2_probe_kernel<2><<<grid, 256, 0, st>>>(x, sf, w_frags, out, n_blocks);
  return check_launch("split2_probe");
}
