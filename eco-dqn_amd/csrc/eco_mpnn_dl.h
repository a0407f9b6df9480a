// Dense-aggregation MPNN forward + backward (src/networks/mpnn.py:40-159; autograd of it, dqn.py:440-449) for ONE
// graph of 224 < N <= 512 vertices per workgroup with +-1 edge weights (BA-500, ER-500): the fp16x2 operands of
// eco_mpnn_dense2.h, re-laid for 32 node tiles.
//
// The CSR kernels of eco_mpnn.hip keep the block's f32 embeddings in LDS (147 KB at N = 500): one workgroup per CU,
// weights streamed from L2 in every wave, and gathers whose 16 lanes hit 16 random rows.  Here the aggregation is
// the dense fp16x2 MFMA product of eco_mpnn_dense2.h (the adjacency operand from bitmasks, two scaled planes per
// feature), which at N = 512 costs a fixed 16 chunks x 32 MFMAs per wave and half-layer:
//
//   * 8 waves, wave w owns tiles w, w + 8, w + 16, w + 24 (16 nodes each, h in registers); the aggregation of the
//     four tiles shares every plane fragment read (one ds_read_b64_tr_b16 pair per plane and feature block feeds
//     four MFMAs);
//   * LDS: the planes of ONE feature half (features 0..31, then 32..63: 2 planes x 2 blocks x 512 rows, 64 KB) --
//     two plane passes per aggregation -- so a whole layer's message and update Linears stay resident (2 x 32 KB,
//     prefetched by LDS-DMA a layer ahead) next to the edge Linear (16 KB); the edge layer's V planes use the two
//     Linear buffers;
//   * the edge embedding e lives in global memory (the saved-activation tensor, or the forward workspace), reread
//     per layer; the adjacency operand (gs.adjbits, pre-spread 16-bit chunks) stays in registers (8 words per tile).
// Numerics are those of eco_mpnn_dense2.h (22-bit fp16x2 operands, f32 accumulation, per-tile plane exponents);
// saved activations, ReLU masks and gradient outputs have its layouts, so the weight-gradient reduction is shared.
#pragma once
#include "eco_mpnn_dense2.h"

namespace eco {

#ifndef DL_NW_X
#define DL_NW_X 8  // A/B knob (with DL_MT_X = 32 / DL_NW_X): waves per workgroup
#define DL_MT_X 4
#endif
constexpr int DL_NW = DL_NW_X;                    // waves per workgroup
constexpr int DL_MT = DL_MT_X;                    // 16-node tiles per wave
constexpr int DL_MAX_ROWS = DL_NW * DL_MT * 16;   // 512
constexpr int DL_KC = DL_MAX_ROWS / 32;           // k-chunks of 32 nodes
constexpr int DL_AW = 8;                          // adjacency words per (node, lane quarter): 16 chunks x 16 bits
constexpr int DL_PLANE = 2 * DL_MAX_ROWS * 16;    // fp16 per plane: [2 feature blocks][512 rows][16] = 32 KB
static_assert(DL_PLANE == D2_WBUF, "a V plane fills one Linear buffer");

// sPL: the two planes of the current feature half (readout / scratch at the ends) | sW0, sW1: a 128-input Linear
// each (the edge layer's V planes) | sW2: the edge Linear (Wf / Wf^T) | sTE: tile exponents (U: 0..31, V: 32..63)
#define ECO_DL_LDS                                                 \
  __shared__ __attribute__((aligned(16))) uint16_t sPL[2 * DL_PLANE]; \
  __shared__ __attribute__((aligned(16))) uint16_t sW0[D2_WBUF];  \
  __shared__ __attribute__((aligned(16))) uint16_t sW1[D2_WBUF];  \
  __shared__ __attribute__((aligned(16))) uint16_t sW2[FH_HALF];  \
  __shared__ int sTE[64]

inline bool dl_eligible(const eco_graph_set* gs, int gpb) {
  const int rows_pad = (gs->n_spins + 15) & ~15;
  return gs->unit_weights && gs->adjbits != nullptr && gpb == 1 && rows_pad > DN_MAX_ROWS && rows_pad <= DL_MAX_ROWS;
}

// plane image of one feature half: [feature block ftl][row j][16] with the 8-B piece swizzle of plane_off
__device__ __forceinline__ int dl_plane_off(int ftl, int j, int k) {
  return ftl * (DL_MAX_ROWS * 16) + j * 16 + 4 * (k ^ ((j >> 2) & 3));
}
// the float4s c = 2hf, 2hf + 1 of node j (node-operand layout, lane quarter s4) scaled by 2^k into the planes
__device__ __forceinline__ void dl_planes_half(uint16_t* P0, uint16_t* P1, int j, int s4, const float4& v0,
                                               const float4& v1, int k) {
  const float sf = exp2i(k == D2_K_EMPTY ? 0 : k);
#pragma unroll
  for (int ftl = 0; ftl < 2; ++ftl) {
    const float4 v = ftl ? v1 : v0;
    uint32_t h0, l0, h1, l1;
    split2_pk(v.x, v.y, sf, h0, l0);
    split2_pk(v.z, v.w, sf, h1, l1);
    const int o = dl_plane_off(ftl, j, s4);
    *reinterpret_cast<uint2*>(P0 + o) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(P1 + o) = make_uint2(l0, l1);
  }
}
// zero the plane rows [rows_pad, KP) of both planes and both feature blocks (read by the last chunk, never written)
template <int NT>
__device__ __forceinline__ void dl_zero_pad(uint16_t* P0, uint16_t* P1, int rows_pad) {
  const int KP = (rows_pad + 31) & ~31;
  for (int i = threadIdx.x; i < (KP - rows_pad) * 2 * 2 * 4; i += NT) {
    const int k = i & 3, ftl = (i >> 2) & 1, p = (i >> 3) & 1, j = rows_pad + (i >> 4);
    *reinterpret_cast<uint2*>((p ? P1 : P0) + dl_plane_off(ftl, j, k)) = make_uint2(0u, 0u);
  }
}

// agg_scale of eco_mpnn_dense2.h over up to 32 tiles (lane t < 32: tile t)
__device__ __forceinline__ AggScale dl_agg_scale(const int* TE, int ntiles, int lane) {
  const int k = lane < ntiles ? TE[lane] : D2_K_EMPTY;
  int kmin = k;
  kmin = min(kmin, __builtin_amdgcn_update_dpp(kmin, kmin, 0x128, 0xF, 0xF, false));
  kmin = min(kmin, __builtin_amdgcn_update_dpp(kmin, kmin, 0x124, 0xF, 0xF, false));
  kmin = min(kmin, __builtin_amdgcn_update_dpp(kmin, kmin, 0x122, 0xF, 0xF, false));
  kmin = min(kmin, __builtin_amdgcn_update_dpp(kmin, kmin, 0x121, 0xF, 0xF, false));
  auto s16 = __builtin_amdgcn_permlane16_swap((uint32_t)kmin, (uint32_t)kmin, false, false);
  kmin = min((int)s16[0], (int)s16[1]);
  auto s32 = __builtin_amdgcn_permlane32_swap((uint32_t)kmin, (uint32_t)kmin, false, false);
  kmin = __builtin_amdgcn_readfirstlane(min((int)s32[0], (int)s32[1]));
  AggScale s;
  s.c = kmin == D2_K_EMPTY ? 0 : 15 + kmin;
  const int E = s.c - k;
  uint32_t p = 0u;
  if (k != D2_K_EMPTY) p = E >= -14 ? (uint32_t)(E + 15) << 10 : (E >= -21 ? 1u << (E + 24) : 0u);
  s.pat = p | (p << 16);
  return s;
}

// acc[i][ftl] += sum over chunks kc < KC and both planes of Hs[j][feature block ftl of the half] . B_i[j][node] for
// the wave's tiles i < ntw (products h 2^c); every plane fragment is read once for all tiles.  adj[i]: the tile's
// pre-spread adjacency words (word m: chunks 2m, 2m + 1), rotated by one word per chunk pair so the loop over pairs
// stays rolled (small code: the kernels call this at a dozen sites); back in place on return.  EXEC all ones
// (wave-uniform conditions only).
template <int MODE>
__device__ __forceinline__ void dl_agg(f32x4 (&acc)[DL_MT][2], const uint16_t* P0, const uint16_t* P1,
                                       uint32_t (&adj)[DL_MT][DL_AW], const AggScale& sc, int KC, int ntw,
                                       int lane) {
  const int q = lane >> 4;
  const int j_in = 4 * q + ((lane >> 2) & 3);
  const int pc = (lane & 3) ^ q;
  const int off0 = j_in * 16 + 4 * pc;
  // plane fragments of chunk kc (both planes, both feature blocks), double-buffered one chunk ahead
  f16x8 af[2][2][2];
  auto load = [&](f16x8 (&dst)[2][2], int kc) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int ftl = 0; ftl < 2; ++ftl) {
        const uint16_t* ap = (p ? P1 : P0) + off0 + 32 * 16 * kc + ftl * (DL_MAX_ROWS * 16);
        const v4s lo = tr_read(ap), hi = tr_read(ap + 16 * 16);
        const bf16x8 raw = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        dst[p][ftl] = __builtin_bit_cast(f16x8, raw);
      }
  };
  load(af[0], 0);
#pragma unroll 1
  for (int m = 0; m < DL_AW; ++m) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kc = 2 * m + h;
      if (kc < KC) {  // wave-uniform
        if (kc + 1 < KC) load(af[h ^ 1], kc + 1);
        const uint32_t plo = __builtin_amdgcn_readlane(sc.pat, 2 * kc);
        const uint32_t phi = __builtin_amdgcn_readlane(sc.pat, 2 * kc + 1);
#pragma unroll
        for (int i = 0; i < DL_MT; ++i) {
          if (i >= ntw) break;  // wave-uniform
          // the chunk's 16-bit word, its bytes spread to bits 0-7 and 16-23 (one v_perm_b32)
          const uint32_t W = __builtin_amdgcn_perm(0u, adj[i][m], h ? 0x0C030C02u : 0x0C010C00u);
          const f16x8 bf = adj_frag2<MODE>(W, plo, phi);
#pragma unroll
          for (int p = 1; p >= 0; --p)  // the small plane first
#pragma unroll
            for (int ftl = 0; ftl < 2; ++ftl)
              acc[i][ftl] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[h][p][ftl], bf, acc[i][ftl], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // bound the fragments in flight to the next chunk's
    }
  }
}

__device__ __forceinline__ float4 sel4(bool hi, const float4& a, const float4& b) {
  return make_float4(hi ? b.x : a.x, hi ? b.y : a.y, hi ? b.z : a.z, hi ? b.w : a.w);
}

// ================================================================================================ forward ====
// ebuf: [R][64] f32 edge embeddings (the saved SV_E tensor, or the forward workspace when nothing is saved).
// Barriers: edge layer 4, per update layer 4 (lo planes | lo read | hi planes + weights | Linears done), readout 1.
template <bool SAVE>
__global__ __launch_bounds__(64 * DL_NW, 1) void mpnn_forward_dl_kernel(MpnnArgs a, float* __restrict__ ebuf) {
  ECO_DL_LDS;
  ECO_TS(0);
  if (!SAVE) ws_invalidate_key(a.call_maxdeg);  // ebuf (the workspace) overwrites the cached shared-graph tables
  constexpr int NW = DL_NW;
  constexpr int MT = DL_MT;
  constexpr int NT = 64 * NW;
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int blk = blockIdx.x;
  const int N = a.N;
  const int rows_pad = (N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  const int KC = (rows_pad + 31) >> 5;
  const int ntw = (ntiles - w + NW - 1) / NW;  // this wave's tiles w, w + NW, ... (1..MT)
  const size_t R0 = (size_t)blk * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const uint16_t* PH = reinterpret_cast<const uint16_t*>(P + PK_FH);
  const int s4 = lane >> 4;
  const int c16 = lane & 15;
  uint16_t* PL0 = sPL;
  uint16_t* PL1 = sPL + DL_PLANE;
  int* TE = sTE;

  // ---- staging: Wf (LDS-DMA); per tile the row norm, adjacency operand and node features ----
  const int gid = a.gids[blk];  // first: the staging loads depend on it (waiting for it leaves the DMA in flight)
  __builtin_amdgcn_sched_barrier(0);
  glds_frags<NW>(sW2, PH + FH_WF, 16, w, lane);
  const int md_graph = a.gs.max_deg[gid];
  int rI[MT];
  bool vI[MT];
  float nf[MT], rnf[MT], xk0[MT], xk1[MT];
  uint32_t adj[MT][DL_AW];
  // unconditional loads (rows past the graph read row 0; degrees and bitmask words are masked below, after the
  // loop): a load skipped on some path made each tile's staging wait for the previous tile's (vmcnt(4) per tile)
  int dgr[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    rI[i] = (w + NW * i) * 16 + c16;
    vI[i] = i < ntw && rI[i] < N;
    const int rc = vI[i] ? rI[i] : 0;
    dgr[i] = a.gs.deg[(size_t)gid * N + rc];
    const uint4* ap = reinterpret_cast<const uint4*>(a.gs.adjbits + (((size_t)gid * N + rc) * 4 + s4) * DL_AW);
    const uint4 a0 = ap[0], a1 = ap[1];
    const float x0 = a.x[(R0 + rc) * 8 + s4], x1 = a.x[(R0 + rc) * 8 + 4 + s4];
    xk0[i] = vI[i] ? x0 : 0.f;
    xk1[i] = vI[i] ? x1 : 0.f;
    adj[i][0] = a0.x; adj[i][1] = a0.y; adj[i][2] = a0.z; adj[i][3] = a0.w;
    adj[i][4] = a1.x; adj[i][5] = a1.y; adj[i][6] = a1.z; adj[i][7] = a1.w;
  }
  dl_zero_pad<NT>(PL0, PL1, rows_pad);
  dl_zero_pad<NT>(sW0, sW1, rows_pad);  // V planes
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    nf[i] = vI[i] ? (float)max(dgr[i], 1) : 1.f;
    rnf[i] = 1.f / nf[i];
#pragma unroll
    for (int k = 0; k < DL_AW; ++k) adj[i][k] = vI[i] ? adj[i][k] : 0u;
  }
  ECO_TS(1);

  // ---- phases A + B: edge embedding (mpnn.py:89-104): (A+ . relu(Z + w_a) + A- . relu(Z - w_a)) / norm, per
  //      feature half: U planes in sPL, V planes in sW0 | sW1 ----
  float4 eg[MT][4];
  {
    float wx8[8];
    lin8_load(P + PK_WX, lane, wx8);
    float4 wa4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) wa4[c] = f4(P + PK_WA + 16 * c + 4 * s4);
    int teu[MT], tev[MT];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (i >= ntw) break;
        f32x4 z[4];
        lin8r(z, wx8, xk0[i], xk1[i]);
        float4 u[4], v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 wa = wa4[c];
          u[c] = vI[i] ? make_float4(relu(fmaf(1.f, wa.x, z[c][0])), relu(fmaf(1.f, wa.y, z[c][1])),
                                     relu(fmaf(1.f, wa.z, z[c][2])), relu(fmaf(1.f, wa.w, z[c][3])))
                       : zero4();
          v[c] = vI[i] ? make_float4(relu(fmaf(-1.f, wa.x, z[c][0])), relu(fmaf(-1.f, wa.y, z[c][1])),
                                     relu(fmaf(-1.f, wa.z, z[c][2])), relu(fmaf(-1.f, wa.w, z[c][3])))
                       : zero4();
        }
        if (hf == 0) {
          teu[i] = tile_exp(u);
          tev[i] = tile_exp(v);
          if (lane == 0) {
            TE[w + NW * i] = teu[i];
            TE[32 + w + NW * i] = tev[i];
          }
        }
        const bool h1 = hf != 0;
        dl_planes_half(PL0, PL1, rI[i], s4, sel4(h1, u[0], u[2]), sel4(h1, u[1], u[3]), teu[i]);
        dl_planes_half(sW0, sW1, rI[i], s4, sel4(h1, v[0], v[2]), sel4(h1, v[1], v[3]), tev[i]);
        __builtin_amdgcn_sched_barrier(0);  // one tile at a time (register budget)
      }
      lds_barrier();
      const AggScale su = dl_agg_scale(TE, ntiles, lane);
      const AggScale sv = dl_agg_scale(TE + 32, ntiles, lane);
      f32x4 ea[MT][2], ev[MT][2];
#pragma unroll
      for (int i = 0; i < MT; ++i) ea[i][0] = ea[i][1] = ev[i][0] = ev[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      dl_agg<1>(ea, PL0, PL1, adj, su, KC, ntw, lane);
      dl_agg<2>(ev, sW0, sW1, adj, sv, KC, ntw, lane);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int ftl = 0; ftl < 2; ++ftl) {
          float t4[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            t4[k] = (__builtin_ldexpf(ea[i][ftl][k], -su.c) + __builtin_ldexpf(ev[i][ftl][k], -sv.c)) * rnf[i];
          const float4 v = make_float4(t4[0], t4[1], t4[2], t4[3]);
          if (hf == 0) eg[i][ftl] = v;
          else eg[i][2 + ftl] = v;
        }
      if (hf == 1) glds_wait();  // Wf: published by the barrier below
      lds_barrier();             // planes read (U and V)
    }
  }
  ECO_TS(2);
  // layer-0 Linears into the freed buffers (landed by layer 0's hi-half barrier)
  glds_frags<NW>(sW0, PH + FH_LAYER, 32, w, lane);
  glds_frags<NW>(sW1, PH + FH_LAYER + 2 * FH_HALF, 32, w, lane);
  {
    const int maxdeg_call = a.norm_scope == ECO_NORM_PER_CALL ? *a.call_maxdeg : 0;
    const int md = a.norm_scope == ECO_NORM_PER_CALL ? maxdeg_call : md_graph;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (i >= ntw) break;
      float4 acc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = vI[i] ? eg[i][c] : zero4();
      if (s4 == 3 && vI[i]) acc[3].w = nf[i] / (float)md;  // feature 63 = norm / norm.max() (mpnn.py:102)
      const size_t ro = (R0 + rI[i]) * 64 + 4 * s4;
      if (SAVE && vI[i]) {
#pragma unroll
        for (int c = 0; c < 4; ++c) st4(a.sv + (size_t)SV_EAGG * RT * 64 + ro + 16 * c, acc[c]);
      }
      f32x4 d[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kx = node_exp<4>(acc);
      mm_fh(d, acc, exp2i(kx), sW2, lane);
      unscale(d, kx + fh_kw(P, 0));
      float4 e[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) e[nt] = relu4(d[nt]);
      if (vI[i]) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) st4(ebuf + ro + 16 * nt, e[nt]);
        if (SAVE) store_mask(a, RT, R0 + rI[i], s4, SM_E, pos_mask(e));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  ECO_TS(3);

  // ---- phase C: h0 = relu(W0 . x) (mpnn.py:20-23, :55) ----
  float4 hreg[MT][4];
  {
    float w08[8];
    lin8_load(P + PK_W0, lane, w08);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      f32x4 z[4];
      lin8r(z, w08, xk0[i], xk1[i]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        hreg[i][c] = vI[i] ? relu4(z[c]) : zero4();
        if (SAVE && vI[i]) st4(a.sv + (size_t)SV_H0 * RT * 64 + (R0 + rI[i]) * 64 + 16 * c + 4 * s4, hreg[i][c]);
      }
      if (SAVE && vI[i]) store_mask(a, RT, R0 + rI[i], s4, SM_H0, pos_mask(hreg[i]));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  ECO_TS(4);

  // the lane's row offset of tile i, recomputed from a laundered lane id inside the layer loop (see the backward)
  auto ro_of = [&](int i) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    return (R0 + (size_t)((w + NW * i) * 16 + (ln & 15))) * 64 + 4 * (ln >> 4);
  };
  // ---- phase D: 3 x UpdateNodeEmbeddingLayer (mpnn.py:114-120); Wm in sW0, Wu in sW1 ----
#pragma unroll 1
  for (int layer = 0; layer < 3; ++layer) {
    int th[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      th[i] = D2_K_EMPTY;
      if (i < ntw) {
        th[i] = tile_exp(hreg[i]);
        if (lane == 0) TE[w + NW * i] = th[i];
      }
    }
    float4 ag[MT][4];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const bool h1 = hf != 0;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (i >= ntw) break;
        dl_planes_half(PL0, PL1, rI[i], s4, sel4(h1, hreg[i][0], hreg[i][2]), sel4(h1, hreg[i][1], hreg[i][3]),
                       th[i]);
      }
      if (h1) glds_wait();  // this layer's Linears (DMA'd a layer ahead): published by this barrier
      lds_barrier();
      if (layer == 0 && hf == 0) ECO_TS(10);
      const AggScale sh = dl_agg_scale(TE, ntiles, lane);
      f32x4 acc[MT][2];
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      dl_agg<0>(acc, PL0, PL1, adj, sh, KC, ntw, lane);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const float sc = __builtin_ldexpf(rnf[i], -sh.c);
#pragma unroll
        for (int ftl = 0; ftl < 2; ++ftl) {
          const float4 v = make_float4(acc[i][ftl][0] * sc, acc[i][ftl][1] * sc, acc[i][ftl][2] * sc,
                                       acc[i][ftl][3] * sc);
          if (h1) ag[i][2 + ftl] = v;
          else ag[i][ftl] = v;
        }
      }
      if (layer == 0 && hf == 0) ECO_TS(11);
      if (!h1) lds_barrier();  // lo planes read before the hi planes overwrite them
    }
    if (layer == 0) ECO_TS(12);
    const float* ev = ebuf;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (i >= ntw) break;
      const size_t ro = ro_of(i);
      float4 e[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) e[c] = vI[i] ? f4(ev + ro + 16 * c) : zero4();
      if (SAVE && vI[i]) {
#pragma unroll
        for (int c = 0; c < 4; ++c) st4(a.sv + (size_t)(SV_AGG0 + layer) * RT * 64 + ro + 16 * c, ag[i][c]);
      }
      // message = relu(Wm . [agg, e])
      float4 mrel[4];
      {
        f32x4 d[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int kx = node_exp2(ag[i], e);
        const float sf = exp2i(kx);
        mm_fh(d, e, sf, sW0 + FH_HALF, lane);
        mm_fh(d, ag[i], sf, sW0, lane);
        unscale(d, kx + fh_kw(P, 1 + 2 * layer));
#pragma unroll
        for (int c = 0; c < 4; ++c) mrel[c] = relu4(d[c]);
      }
      if (SAVE && vI[i]) {
#pragma unroll
        for (int c = 0; c < 4; ++c) st4(a.sv + (size_t)(SV_M0 + layer) * RT * 64 + ro + 16 * c, mrel[c]);
        store_mask(a, RT, R0 + rI[i], s4, SM_M0 + layer, pos_mask(mrel));
      }
      // h' = relu(Wu . [h, m])
      {
        f32x4 hn[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) hn[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int kx = node_exp2(hreg[i], mrel);
        const float sf = exp2i(kx);
        mm_fh(hn, hreg[i], sf, sW1, lane);
        mm_fh(hn, mrel, sf, sW1 + FH_HALF, lane);
        unscale(hn, kx + fh_kw(P, 2 + 2 * layer));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          hreg[i][c] = vI[i] ? relu4(hn[c]) : zero4();
          if (SAVE && vI[i]) st4(a.sv + (size_t)(SV_H0 + layer + 1) * RT * 64 + ro + 16 * c, hreg[i][c]);
        }
      }
      if (SAVE && vI[i]) store_mask(a, RT, R0 + rI[i], s4, SM_H1 + layer, pos_mask(hreg[i]));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (layer == 0) ECO_TS(13);
    lds_barrier();  // hi planes read, this layer's Linears done: buffers free
    if (layer < 2) {
      glds_frags<NW>(sW0, PH + FH_LAYER + (layer + 1) * FH_LAYER_STRIDE, 32, w, lane);
      glds_frags<NW>(sW1, PH + FH_LAYER + (layer + 1) * FH_LAYER_STRIDE + 2 * FH_HALF, 32, w, lane);
    }
    ECO_TS(5 + layer);
  }

  // ---- phase E: readout (mpnn.py:143-159) + act: per node q_local = Wr[64:] . h3 and per tile the column sums of
  //      h3 (registers -> LDS), one barrier, wave 0 reduces the tiles in tile order ----
  float* COL = reinterpret_cast<float*>(sPL);  // [32][64]
  float* QL = COL + 32 * 64;                   // [512]
  float* MEANS = QL + DL_MAX_ROWS;             // [64]
  float* QB = MEANS + 64;                      // [512]
  {
    float4 wr[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) wr[c] = f4(P + PK_WR + 64 + 16 * c + 4 * s4);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (i >= ntw) break;
      float ql = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        ql = fmaf(hreg[i][c].x, wr[c].x, ql);
        ql = fmaf(hreg[i][c].y, wr[c].y, ql);
        ql = fmaf(hreg[i][c].z, wr[c].z, ql);
        ql = fmaf(hreg[i][c].w, wr[c].w, ql);
      }
      auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(ql), __float_as_uint(ql), false, false);
      ql = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
      auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(ql), __float_as_uint(ql), false, false);
      ql = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
      if (s4 == 0) QL[rI[i]] = ql;
      float cs[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        cs[4 * c] = row_sum16(hreg[i][c].x);
        cs[4 * c + 1] = row_sum16(hreg[i][c].y);
        cs[4 * c + 2] = row_sum16(hreg[i][c].z);
        cs[4 * c + 3] = row_sum16(hreg[i][c].w);
      }
      if (c16 == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          st4(COL + (w + NW * i) * 64 + 16 * c + 4 * s4,
              make_float4(cs[4 * c], cs[4 * c + 1], cs[4 * c + 2], cs[4 * c + 3]));
      }
    }
  }
  lds_barrier();
  if (w == 0) {
    float cs = 0.f;
    for (int t = 0; t < ntiles; ++t) cs += COL[t * 64 + lane];  // tile order
    const float mean = cs / (float)N;
    MEANS[lane] = mean;
    wave_lds_sync();
    const float* wp = P + PK_WP + lane * 64;
    float p = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float4 wv = f4(wp + 4 * k), mv = f4(MEANS + 4 * k);
      p = fmaf(wv.x, mv.x, p);
      p = fmaf(wv.y, mv.y, p);
      p = fmaf(wv.z, mv.z, p);
      p = fmaf(wv.w, mv.w, p);
    }
    if (SAVE) {
      a.sv[(size_t)SV_NODE_TENSORS * RT * 64 + (size_t)blk * 64 + lane] = mean;
      a.sv[(size_t)SV_NODE_TENSORS * RT * 64 + (size_t)a.B * 64 + (size_t)blk * 64 + lane] = p;
    }
    const float cg = wave_sum_f(relu(p) * P[PK_WR + lane]);
    const float br = P[PK_BR];
    for (int v = lane; v < N; v += 64) {
      const float qv = cg + QL[v] + br;
      QB[v] = qv;
      if (a.q) a.q[R0 + v] = qv;
    }
    if (a.has_act) {
      wave_lds_sync();
      graph_act<NW>(a, QB, blk, 1, R0);
    }
  }
  ECO_TS(8);
}

// =============================================================================================== backward ====
// Autograd of mpnn_forward_dl_kernel on the same operands (the per-layer structure of mpnn_backward_dense2_kernel):
// per layer the two transposed Linears (Wu^T in sW0, Wm^T in sW1, the next layer's pair DMA'd during the
// aggregation), G = dagg / norm as planes one feature half at a time, dh = dh_direct + A . G.  de accumulates in
// the GR_DE tensor (global), the edge layer's dEagg = Wf^T . due (sW2) feeds dz through A+ and A-.
__global__ __launch_bounds__(64 * DL_NW, 1) void mpnn_backward_dl_kernel(MpnnArgs a) {
  ECO_DL_LDS;
  ECO_TS(16);
  constexpr int NW = DL_NW;
  constexpr int MT = DL_MT;
  constexpr int NT = 64 * NW;
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int blk = blockIdx.x;
  const int N = a.N;
  const int rows_pad = (N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  const int KC = (rows_pad + 31) >> 5;
  const int ntw = (ntiles - w + NW - 1) / NW;
  const size_t R0 = (size_t)blk * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const uint16_t* PH = reinterpret_cast<const uint16_t*>(P + PK_FH);
  const float* sv = a.sv;
  float* gr = a.gr;
  const int s4 = lane >> 4;
  const int c16 = lane & 15;
  uint16_t* PL0 = sPL;
  uint16_t* PL1 = sPL + DL_PLANE;
  float* lds = reinterpret_cast<float*>(sPL);  // readout / dw_a scratch
  int* TE = sTE;
  auto GR = [&](int t) { return gr + (size_t)t * RT * 64; };
  const float* MEAN = sv + (size_t)SV_NODE_TENSORS * RT * 64;
  const float* PP = MEAN + (size_t)a.B * 64;
  float* DP = gr + (size_t)GR_NODE_TENSORS * RT * 64;
  float* DWRA = DP + (size_t)a.B * 64;
  float* DWRB = DWRA + (size_t)a.B * 64;
  float* DBR = DWRB + (size_t)a.B * 64;
  float* DWA = DBR + ((a.B + 63) & ~63);  // [nblocks][64]
  auto WUT = [&](int l) { return PH + FHT_LAYER + l * FH_LAYER_STRIDE + 2 * FH_HALF; };
  auto WMT = [&](int l) { return PH + FHT_LAYER + l * FH_LAYER_STRIDE; };

  // ---- staging: Wu^T / Wm^T of layer 2, Wf^T (LDS-DMA); per tile norm, adjacency operand, ReLU masks ----
  const int gid = a.gids[blk];  // first (see the forward)
  __builtin_amdgcn_sched_barrier(0);
  glds_frags<NW>(sW0, WUT(2), 32, w, lane);
  glds_frags<NW>(sW1, WMT(2), 32, w, lane);
  glds_frags<NW>(sW2, PH + FHT_WF, 16, w, lane);
  const uint16_t* Msk = reinterpret_cast<const uint16_t*>(sv + sv_mask_offset_floats(RT, a.B));
  int rI[MT];
  bool vI[MT];
  float rnf[MT];
  uint32_t adj[MT][DL_AW];
  uint4 rmask[MT];
  int dgr[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {  // unconditional loads, masked after the loop (see the forward)
    rI[i] = (w + NW * i) * 16 + c16;
    vI[i] = i < ntw && rI[i] < N;
    const int rc = vI[i] ? rI[i] : 0;
    dgr[i] = a.gs.deg[(size_t)gid * N + rc];
    const uint4* ap = reinterpret_cast<const uint4*>(a.gs.adjbits + (((size_t)gid * N + rc) * 4 + s4) * DL_AW);
    const uint4 a0 = ap[0], a1 = ap[1];
    rmask[i] = *reinterpret_cast<const uint4*>(Msk + ((R0 + rc) * 4 + s4) * SM_TENSORS);
    adj[i][0] = a0.x; adj[i][1] = a0.y; adj[i][2] = a0.z; adj[i][3] = a0.w;
    adj[i][4] = a1.x; adj[i][5] = a1.y; adj[i][6] = a1.z; adj[i][7] = a1.w;
  }
  ECO_TS(17);

  // ---- readout backward (mpnn.py:143-159), scratch in the plane region: dWr[64:] = sum_v dq_v h3_v over waves ----
  float* DQ = lds;              // [rows_pad]
  float* DMEAN = DQ + rows_pad;  // [64]
  float* RED = DMEAN + 64;       // [NW][64]
  for (int i = threadIdx.x; i < rows_pad; i += NT) DQ[i] = i < N ? a.dq[R0 + i] : 0.f;
  lds_barrier();
  {
    const float* h3 = sv + (size_t)SV_H3 * RT * 64 + R0 * 64;
    float dwb = 0.f;
    for (int v = w; v < N; v += NW) {
      const float dv = DQ[v];
      if (dv != 0.f) dwb = fmaf(dv, h3[(size_t)v * 64 + lane], dwb);
    }
    RED[w * 64 + lane] = dwb;
  }
  lds_barrier();
  if (w == 0) {
    const int e = blk;
    float sacc = 0.f;
    for (int v = lane; v < N; v += 64) sacc += DQ[v];
    const float S = wave_sum_f(sacc);
    const float p = PP[(size_t)e * 64 + lane];
    const float dp = P[PK_WR + lane] * S * (p > 0.f ? 1.f : 0.f);
    DP[(size_t)e * 64 + lane] = dp;
    DWRA[(size_t)e * 64 + lane] = relu(p) * S;
    if (lane == 0) DBR[e] = S;
    float dmean = 0.f;
#pragma unroll 16
    for (int k = 0; k < 64; ++k) dmean = fmaf(P[PK_WP + k * 64 + lane], __shfl(dp, k, 64), dmean);
    DMEAN[lane] = dmean / (float)N;
    float dwb = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) dwb += RED[k * 64 + lane];  // fixed order
    DWRB[(size_t)e * 64 + lane] = dwb;
  }
  lds_barrier();
  // dh3 (node-operand layout): dq_i * wr[64+f] + dmean_f / N
  float4 dh[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const float dqi = vI[i] ? DQ[rI[i]] : 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int f = 16 * c + 4 * s4;
      const float4 dm = vI[i] ? f4(DMEAN + f) : zero4();
      dh[i][c] = make_float4(fmaf(dqi, P[PK_WR + 64 + f + 0], dm.x), fmaf(dqi, P[PK_WR + 64 + f + 1], dm.y),
                             fmaf(dqi, P[PK_WR + 64 + f + 2], dm.z), fmaf(dqi, P[PK_WR + 64 + f + 3], dm.w));
    }
  }
  glds_wait();     // Wu^T / Wm^T of layer 2 and Wf^T
  lds_barrier();  // readout scratch dead
  // the staged degrees, bitmask words and ReLU masks of rows past the graph (loaded from row 0), first needed below
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    rnf[i] = vI[i] ? 1.f / (float)max(dgr[i], 1) : 1.f;
    if (!vI[i]) rmask[i] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < DL_AW; ++k) adj[i][k] = vI[i] ? adj[i][k] : 0u;
  }
  dl_zero_pad<NT>(PL0, PL1, rows_pad);
  ECO_TS(18);

  // the lane's row offset of tile i, recomputed from a laundered lane id inside the layer loop: hoisted out of it,
  // the per-tile row addresses stayed live through every layer and were spilled (scratch reloads wait for vmcnt(0))
  auto ro_of = [&](int i) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    return (R0 + (size_t)((w + NW * i) * 16 + (ln & 15))) * 64 + 4 * (ln >> 4);
  };
  // ---- update layers in reverse (mpnn.py:114-120) ----
#pragma unroll 1
  for (int layer = 2; layer >= 0; --layer) {
    float4 ghi[MT][2];
    int tg[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      tg[i] = D2_K_EMPTY;
      ghi[i][0] = ghi[i][1] = zero4();
      if (i >= ntw) continue;
      const size_t ro = ro_of(i);
      // duu = dh' * [h' > 0]
      float4 duu[4];
      {
        const uint32_t hmask = mask16(rmask[i], SM_H0 + layer + 1);
#pragma unroll
        for (int c = 0; c < 4; ++c) duu[c] = masked(f32x4{dh[i][c].x, dh[i][c].y, dh[i][c].z, dh[i][c].w}, hmask, c);
      }
      // [dh_direct, dm] = Wu^T . duu;  dum = dm * [m > 0]
      f32x4 dhd[4], dmm[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dhd[nt] = dmm[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      {
        const int kx = node_exp<4>(duu);
        mm_fh2(dhd, dmm, duu, exp2i(kx), sW0, sW0 + FH_HALF, lane);
        const int ku = kx + fh_kw(P, 2 + 2 * layer);
        unscale(dhd, ku);
        unscale(dmm, ku);
      }
      float4 dum[4];
      {
        const uint32_t mmask = mask16(rmask[i], SM_M0 + layer);
#pragma unroll
        for (int c = 0; c < 4; ++c) dum[c] = masked(dmm[c], mmask, c);
      }
      if (vI[i]) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          st4(GR(GR_DUU0 + layer) + ro + 16 * c, duu[c]);
          st4(GR(GR_DUM0 + layer) + ro + 16 * c, dum[c]);
        }
      }
      // [dagg, de] = Wm^T . dum;  G = dagg / norm -> planes
      f32x4 dg[4], dd[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dg[nt] = dd[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      {
        const int kx = node_exp<4>(dum);
        mm_fh2(dg, dd, dum, exp2i(kx), sW1, sW1 + FH_HALF, lane);
        const int km = kx + fh_kw(P, 1 + 2 * layer);
        unscale(dg, km);
        unscale(dd, km);
      }
      if (vI[i]) {
        float* dep = GR(GR_DE) + ro;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 prev = layer == 2 ? zero4() : f4(dep + 16 * c);
          st4(dep + 16 * c, make_float4(prev.x + dd[c][0], prev.y + dd[c][1], prev.z + dd[c][2], prev.w + dd[c][3]));
        }
      }
      float4 g[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        g[c] = vI[i] ? make_float4(dg[c][0] * rnf[i], dg[c][1] * rnf[i], dg[c][2] * rnf[i], dg[c][3] * rnf[i])
                     : zero4();
        dh[i][c] = make_float4(dhd[c][0], dhd[c][1], dhd[c][2], dhd[c][3]);  // dh_direct; + A . G below
      }
      tg[i] = tile_exp(g);
      if (lane == 0) TE[w + NW * i] = tg[i];
      dl_planes_half(PL0, PL1, rI[i], s4, g[0], g[1], tg[i]);
      ghi[i][0] = g[2];
      ghi[i][1] = g[3];
      __builtin_amdgcn_sched_barrier(0);
    }
    if (layer == 1) ECO_TS(24);
    lds_barrier();  // lo G planes + TE ready; this layer's Wu^T / Wm^T read by every wave
    if (layer > 0) {
      glds_frags<NW>(sW0, WUT(layer - 1), 32, w, lane);
      glds_frags<NW>(sW1, WMT(layer - 1), 32, w, lane);
    }
    const AggScale sg = dl_agg_scale(TE, ntiles, lane);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const bool h1 = hf != 0;
      if (h1) {
        lds_barrier();  // lo planes read
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          if (i >= ntw) break;
          dl_planes_half(PL0, PL1, rI[i], s4, ghi[i][0], ghi[i][1], tg[i]);
        }
        lds_barrier();
      }
      f32x4 acc[MT][2];
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      dl_agg<0>(acc, PL0, PL1, adj, sg, KC, ntw, lane);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int ftl = 0; ftl < 2; ++ftl) {
          const float4 d0 = h1 ? dh[i][2 + ftl] : dh[i][ftl];
          const float4 v = vI[i] ? make_float4(d0.x + __builtin_ldexpf(acc[i][ftl][0], -sg.c),
                                               d0.y + __builtin_ldexpf(acc[i][ftl][1], -sg.c),
                                               d0.z + __builtin_ldexpf(acc[i][ftl][2], -sg.c),
                                               d0.w + __builtin_ldexpf(acc[i][ftl][3], -sg.c))
                                 : zero4();
          if (h1) dh[i][2 + ftl] = v;
          else dh[i][ftl] = v;
        }
    }
    glds_wait();
    lds_barrier();  // planes free; the next layer's Wu^T / Wm^T landed
    ECO_TS(21 - layer);
  }

  // ---- du0 = dh0 * [h0 > 0];  edge embedding (mpnn.py:89-104): due = de * [e > 0], G = (Wf^T . due) / norm ----
  float4 ghi[MT][2];
  int tg[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    tg[i] = D2_K_EMPTY;
    ghi[i][0] = ghi[i][1] = zero4();
    if (i >= ntw) continue;
    const size_t ro = (R0 + rI[i]) * 64 + 4 * s4;
    const uint32_t h0m = mask16(rmask[i], SM_H0), em = mask16(rmask[i], SM_E);
    float4 due[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 de = vI[i] ? f4(GR(GR_DE) + ro + 16 * c) : zero4();
      due[c] = masked(f32x4{de.x, de.y, de.z, de.w}, em, c);
      if (vI[i]) {
        st4(GR(GR_DU0) + ro + 16 * c, masked(f32x4{dh[i][c].x, dh[i][c].y, dh[i][c].z, dh[i][c].w}, h0m, c));
        st4(GR(GR_DUE) + ro + 16 * c, due[c]);
      }
    }
    f32x4 dg[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dg[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kx = node_exp<4>(due);
    mm_fh(dg, due, exp2i(kx), sW2, lane);
    unscale(dg, kx + fh_kw(P, 0));
    float4 g[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
      g[c] = vI[i] ? make_float4(dg[c][0] * rnf[i], dg[c][1] * rnf[i], dg[c][2] * rnf[i], dg[c][3] * rnf[i])
                   : zero4();
    tg[i] = tile_exp(g);
    if (lane == 0) TE[w + NW * i] = tg[i];
    dl_planes_half(PL0, PL1, rI[i], s4, g[0], g[1], tg[i]);
    ghi[i][0] = g[2];
    ghi[i][1] = g[3];
  }
  lds_barrier();
  ECO_TS(22);
  // dz_j = [z_j + w_a > 0] (A+ . G)_j + [z_j - w_a > 0] (A- . G)_j;  dw_a = sum_j of the same with signs
  {
    float wx8[8];
    lin8_load(P + PK_WX, lane, wx8);
    float xk0[MT], xk1[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      xk0[i] = vI[i] ? a.x[(R0 + rI[i]) * 8 + s4] : 0.f;
      xk1[i] = vI[i] ? a.x[(R0 + rI[i]) * 8 + 4 + s4] : 0.f;
    }
    float dwacc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) dwacc[k] = 0.f;
    const AggScale sg = dl_agg_scale(TE, ntiles, lane);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const bool h1 = hf != 0;
      if (h1) {
        lds_barrier();
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          if (i >= ntw) break;
          dl_planes_half(PL0, PL1, rI[i], s4, ghi[i][0], ghi[i][1], tg[i]);
        }
        lds_barrier();
      }
      f32x4 gp[MT][2], gm[MT][2];
#pragma unroll
      for (int i = 0; i < MT; ++i) gp[i][0] = gp[i][1] = gm[i][0] = gm[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      dl_agg<1>(gp, PL0, PL1, adj, sg, KC, ntw, lane);
      dl_agg<2>(gm, PL0, PL1, adj, sg, KC, ntw, lane);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (i >= ntw) break;
        f32x4 zz[4];
        lin8r(zz, wx8, xk0[i], xk1[i]);  // Z exactly as the forward computed it
#pragma unroll
        for (int ftl = 0; ftl < 2; ++ftl) {
          const int c = 2 * hf + ftl;
          const f32x4 z = h1 ? zz[2 + ftl] : zz[ftl];
          const float4 wa = f4(P + PK_WA + 16 * c + 4 * s4);
          const float wav[4] = {wa.x, wa.y, wa.z, wa.w};
          float dz4[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float tp = fmaf(1.f, wav[k], z[k]) > 0.f ? __builtin_ldexpf(gp[i][ftl][k], -sg.c) : 0.f;
            const float tm = fmaf(-1.f, wav[k], z[k]) > 0.f ? __builtin_ldexpf(gm[i][ftl][k], -sg.c) : 0.f;
            dz4[k] = vI[i] ? tp + tm : 0.f;
            const float dwv = vI[i] ? tp - tm : 0.f;
            if (h1) dwacc[8 + 4 * ftl + k] += dwv;
            else dwacc[4 * ftl + k] += dwv;
          }
          if (vI[i]) st4(GR(GR_DZ) + (R0 + rI[i]) * 64 + 16 * c + 4 * s4, make_float4(dz4[0], dz4[1], dz4[2], dz4[3]));
        }
      }
    }
    // reduce dw_a over the 16 node lanes sharing s4, then over waves (fixed order)
#pragma unroll
    for (int k = 0; k < 16; ++k) dwacc[k] = row_sum16(dwacc[k]);
    lds_barrier();  // every wave is done reading the G planes: the region becomes the dwa scratch
    float* REDW = lds;  // [NW][64]
    if (c16 == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        st4(REDW + w * 64 + 16 * c + 4 * s4,
            make_float4(dwacc[4 * c], dwacc[4 * c + 1], dwacc[4 * c + 2], dwacc[4 * c + 3]));
    }
    lds_barrier();
    if (w == 0) {
      float sacc = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) sacc += REDW[k * 64 + lane];
      DWA[(size_t)blk * 64 + lane] = sacc;
    }
  }
  ECO_TS(23);
}

static int mpnn_forward_dl_launch(const MpnnArgs& a, bool save, void* workspace, hipStream_t st) {
  float* ebuf = save ? a.sv + (size_t)SV_E * a.B * a.N * 64 : reinterpret_cast<float*>((char*)workspace + 256);
  if (save) mpnn_forward_dl_kernel<true><<<a.B, 64 * DL_NW, 0, st>>>(a, ebuf);
  else mpnn_forward_dl_kernel<false><<<a.B, 64 * DL_NW, 0, st>>>(a, ebuf);
  return check_launch("mpnn_forward_dl");
}

static int mpnn_backward_dl_launch(const MpnnArgs& a, hipStream_t st) {
  mpnn_backward_dl_kernel<<<a.B, 64 * DL_NW, 0, st>>>(a);
  return check_launch("mpnn_backward_dl");
}

}  // namespace eco
