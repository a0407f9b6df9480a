// Dense-aggregation MPNN forward (src/networks/mpnn.py:40-159) on the fp16x2 operands of eco_mpnn_dense2.h, laid
// out for TWO 16-node tiles per wave: 8 waves (2 per SIMD, 256 VGPRs each) per block of whole graphs, wave w owning
// tiles 2w and 2w + 1 (h and e of both in registers).
//
// Why (round-5 ISA and SQ counters of the 16-wave dense2 kernel): with one tile per wave and the
// 128-VGPR budget of 16 waves, every aggregation MFMA waited on a plane fragment read issued one MFMA earlier
// (lgkmcnt(2) after each pair of ds_read_b64_tr_b16) and every Linear MFMA group on a weight fragment read issued
// right before it (lgkmcnt(0)): the LDS latency was exposed on each 16-cycle MFMA, and 13 waves re-read the same
// plane and weight fragments.  Here each fragment read feeds the MFMAs of both tiles (half the LDS traffic per MFMA),
// the two tiles' chains interleave (no dependent back-to-back MFMAs), and the 256-VGPR budget keeps a whole chunk's
// plane fragments and a whole Linear half's weight fragments in flight.
//
// Numerics are those of mpnn_forward_dense2_kernel operation by operation: every accumulator receives the same
// MFMAs with the same operands in the same order (tile pairs whose chunk ranges differ -- several graphs per block --
// run the union range; the extra chunks carry all-zero adjacency fragments and add +-0 to a sum that starts at +0),
// the same scales, splits and f32 epilogues, so the two kernels are bitwise equal
// (tests/test_dense_gpu.py::test_dense3_matches_dense2_bitwise).  Saved activations, masks and the readout are
// written in dense2's layout (the backward is shared).
#pragma once
#include "eco_mpnn_dense2.h"

namespace eco {

constexpr int D3_NW = 8;  // waves per workgroup
// Priority checkpoints inside a forward layer (A/B: D3_SETPRIO): the priority drops at each checkpoint a wave
// passes and is restored after each barrier, so of the two waves of a SIMD the one behind is issued first and they
// reach the barrier together (the arbiter's oldest-first choice otherwise lets one run ahead and wait)
#ifndef D3_SETPRIO
#define D3_SETPRIO 1
#endif
#define D3_PRIO(k)                                     \
  do {                                                 \
    if (D3_SETPRIO) __builtin_amdgcn_s_setprio(k);     \
  } while (0)
#ifndef D3_LIN_SPLIT_AHEAD
#define D3_LIN_SPLIT_AHEAD 1  // A/B: the inference forward's Linears split one step ahead
#endif

// Transposed fragment reads of the planes through LDS pointers derived from the plane array itself (address-space
// casts and element offsets), not integer byte addresses: the compiler's alias analysis then sees that they cannot
// touch a weight buffer an LDS-DMA is filling, and does not make them wait for the DMA (an integer-built address --
// round 5's opaque base, ~220 VALU fewer -- forced s_waitcnt vmcnt(0) before each layer's first plane reads, i.e.
// waited for the next weights' DMA instead of landing it under the aggregation).
typedef __attribute__((address_space(3))) v4s lds_v4s;
__device__ __forceinline__ v4s tr_read_p(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}
// the (lo, hi) fragment pair of plane base b (the lane part included), chunk kc, feature block ft
__device__ __forceinline__ f16x8 plane_frag(const uint16_t* b, int kc, int ft) {
  const int o = 32 * kc * 16 + ft * (DN_KPMAX * 16);
  const v4s lo = tr_read_p(b + o), hi = tr_read_p(b + o + 16 * 16);
  const bf16x8 raw = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(f16x8, raw);
}
// aggregation of the wave's two tiles: the pipelined straight-line form when every chunk is live
#define AGG3(M, acc, P0, P1, adjw, sc, kc0, kc1, lane)                                        \
  do {                                                                                      \
    if (kc0 == 0 && kc1 == DN_KC) agg3f<M>(acc, P0, P1, adjw, sc, lane);                    \
    else agg3<M>(acc, P0, P1, adjw, sc, kc0, kc1, lane);                                    \
  } while (0)

// acc[t][ft] += sum over chunks kc in [kc0, kc1) and both planes of Hs[j][16ft + ..] . B_t[j][node] for the wave's
// two tiles t = 0, 1 (products h 2^c); each plane fragment read feeds both tiles' MFMAs.  adjw[t][kc]: spread
// adjacency words of tile t; sc: agg_scale of the planes.  EXEC all ones (wave-uniform branches only).
template <int MODE>
__device__ __forceinline__ void agg3(f32x4 (&acc)[2][4], const uint16_t* P0, const uint16_t* P1,
                                     const uint32_t (&adjw)[2][DN_KC], const AggScale& sc, int kc0, int kc1,
                                     int lane) {
  const int q = lane >> 4;
  const int j_in = 4 * q + ((lane >> 2) & 3);
  const int pc = (lane & 3) ^ q;
  const uint16_t* pb[2] = {P0 + j_in * 16 + 4 * pc, P1 + j_in * 16 + 4 * pc};
#pragma unroll
  for (int kc = 0; kc < DN_KC; ++kc) {
    if (kc < kc0 || kc >= kc1) continue;  // wave-uniform
    const uint32_t plo = __builtin_amdgcn_readlane(sc.pat, 2 * kc);
    const uint32_t phi = __builtin_amdgcn_readlane(sc.pat, 2 * kc + 1);
    const f16x8 b0 = adj_frag2<MODE>(adjw[0][kc], plo, phi);
    const f16x8 b1 = adj_frag2<MODE>(adjw[1][kc], plo, phi);
    f16x8 af[2][4];
#pragma unroll
    for (int p = 1; p >= 0; --p) {
#pragma unroll
      for (int ft = 0; ft < 4; ++ft) af[p][ft] = plane_frag(pb[p], kc, ft);
    }
#pragma unroll
    for (int p = 1; p >= 0; --p) {  // the small plane first (dense2's order per accumulator)
#pragma unroll
      for (int ft = 0; ft < 4; ++ft) {
        acc[0][ft] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[p][ft], b0, acc[0][ft], 0, 0, 0);
        acc[1][ft] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[p][ft], b1, acc[1][ft], 0, 0, 0);
      }
    }
  }
}

// agg3 software-pipelined for blocks whose every wave runs chunks 0 .. DN_KC - 1 (one graph of 193 .. 224 rows:
// ER-200): straight-line code, chunk kc + 1's 16 plane reads and adjacency fragments issued into the other register
// set while chunk kc's 16 MFMAs run, interleaved one MFMA / one read / two VALU by sched_group_barrier (the
// compiler's own schedule waited on every pair of fragments: lgkmcnt(0) before each group of four MFMAs).  Same
// MFMAs per accumulator in the same order as agg3.
template <int MODE>
__device__ __forceinline__ void agg3f(f32x4 (&acc)[2][4], const uint16_t* P0, const uint16_t* P1,
                                      const uint32_t (&adjw)[2][DN_KC], const AggScale& sc, int lane) {
  const int q = lane >> 4;
  const int j_in = 4 * q + ((lane >> 2) & 3);
  const int pc = (lane & 3) ^ q;
  const uint16_t* pb[2] = {P0 + j_in * 16 + 4 * pc, P1 + j_in * 16 + 4 * pc};
  f16x8 fa[2][8], fb[2][2];
  auto issue = [&](int kc, int buf) {
#pragma unroll
    for (int p = 1; p >= 0; --p) {
#pragma unroll
      for (int ft = 0; ft < 4; ++ft) fa[buf][(1 - p) * 4 + ft] = plane_frag(pb[p], kc, ft);
    }
    const uint32_t plo = __builtin_amdgcn_readlane(sc.pat, 2 * kc);
    const uint32_t phi = __builtin_amdgcn_readlane(sc.pat, 2 * kc + 1);
    fb[buf][0] = adj_frag2<MODE>(adjw[0][kc], plo, phi);
    fb[buf][1] = adj_frag2<MODE>(adjw[1][kc], plo, phi);
  };
  issue(0, 0);
#pragma unroll
  for (int kc = 0; kc < DN_KC; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < DN_KC) issue(kc + 1, cur ^ 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // i = (1 - p) * 4 + ft: the small plane first
      acc[0][i & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[cur][i], fb[cur][0], acc[0][i & 3], 0, 0, 0);
      acc[1][i & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[cur][i], fb[cur][1], acc[1][i & 3], 0, 0, 0);
    }
    if (kc + 1 < DN_KC) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // chunk kc + 1's reads stay in this group (ahead of their MFMAs)
  }
}

// acc[t][nt] += W[16nt + .][one 64-input half] . x_t for both tiles, x_t = hi + lo (split_fh with the tile's node
// scale sf[t]); every weight fragment read feeds both tiles.  Per accumulator the products of mm_fh in its order.
__device__ __forceinline__ void mm_fh_2t(f32x4 (&acc)[2][4], const float4 (&x0)[4], const float4 (&x1)[4],
                                         const float (&sf)[2], const uint16_t* WH, int lane) {
  const uint16_t* wl = WH + lane * 8;
#pragma unroll
  for (int kc2 = 0; kc2 < 2; ++kc2) {
    f16x8 wf1[4], wf2[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      wf1[nt] = *reinterpret_cast<const f16x8*>(wl + ((0 * 4 + nt) * 2 + kc2) * FH_FRAG);
      wf2[nt] = *reinterpret_cast<const f16x8*>(wl + ((1 * 4 + nt) * 2 + kc2) * FH_FRAG);
    }
    f16x8 xh0, xl0, xh1, xl1;
    split_fh(x0[2 * kc2], x0[2 * kc2 + 1], sf[0], xh0, xl0);
    split_fh(x1[2 * kc2], x1[2 * kc2 + 1], sf[1], xh1, xl1);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf2[nt], xh0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf2[nt], xh1, acc[1][nt], 0, 0, 0);
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[nt], xl0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[nt], xl1, acc[1][nt], 0, 0, 0);
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[nt], xh0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[nt], xh1, acc[1][nt], 0, 0, 0);
    }
  }
}

// A whole 128-input Linear for both tiles, as mm_fh_2t(x_a, W_a) then mm_fh_2t(x_b, W_b) (the same products per
// accumulator in the same order), software-pipelined over its four 32-input steps: step s + 1's eight weight
// fragments are read while step s's inputs are split and its 24 MFMAs run (sched_barrier keeps each step's reads
// ahead of their MFMAs instead of right before them).
template <bool AHEAD>
__device__ __forceinline__ void lin128_2t(f32x4 (&acc)[2][4], const float4 (&xa0)[4], const float4 (&xa1)[4],
                                          const uint16_t* WA, const float4 (&xb0)[4], const float4 (&xb1)[4],
                                          const uint16_t* WB, const float (&sf)[2], int lane) {
  f16x8 w1[2][4], w2[2][4];
  auto issue = [&](int s, int buf) {
    const uint16_t* wl = (s < 2 ? WA : WB) + lane * 8;
    const int kc2 = s & 1;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      w1[buf][nt] = *reinterpret_cast<const f16x8*>(wl + ((0 * 4 + nt) * 2 + kc2) * FH_FRAG);
      w2[buf][nt] = *reinterpret_cast<const f16x8*>(wl + ((1 * 4 + nt) * 2 + kc2) * FH_FRAG);
    }
  };
if constexpr (AHEAD) {
  // the inputs of step s + 1 are split while step s's MFMAs run (VALU under the matrix core, one wave); the
  // second split set costs 16 VGPRs: the inference forward only (the saving and the paired kernels would spill)
  f16x8 xs[2][4];  // [buf][xh0, xl0, xh1, xl1]
  auto split_step = [&](int s, int buf) {
    const int kc2 = s & 1;
    if (s < 2) {
      split_fh(xa0[2 * kc2], xa0[2 * kc2 + 1], sf[0], xs[buf][0], xs[buf][1]);
      split_fh(xa1[2 * kc2], xa1[2 * kc2 + 1], sf[1], xs[buf][2], xs[buf][3]);
    } else {
      split_fh(xb0[2 * kc2], xb0[2 * kc2 + 1], sf[0], xs[buf][0], xs[buf][1]);
      split_fh(xb1[2 * kc2], xb1[2 * kc2 + 1], sf[1], xs[buf][2], xs[buf][3]);
    }
  };
  issue(0, 0);
  split_step(0, 0);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int cur = s & 1;
    if (s + 1 < 4) {
      issue(s + 1, cur ^ 1);
      split_step(s + 1, cur ^ 1);
    }
    const f16x8 xh0 = xs[cur][0], xl0 = xs[cur][1], xh1 = xs[cur][2], xl1 = xs[cur][3];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[cur][nt], xh0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[cur][nt], xh1, acc[1][nt], 0, 0, 0);
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[cur][nt], xl0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[cur][nt], xl1, acc[1][nt], 0, 0, 0);
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[cur][nt], xh0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[cur][nt], xh1, acc[1][nt], 0, 0, 0);
    }
    if (s + 1 < 4) {
#pragma unroll
      for (int i = 0; i < 24; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU (the next step's split)
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
} else {
  issue(0, 0);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int cur = s & 1;
    if (s + 1 < 4) issue(s + 1, cur ^ 1);
    const int kc2 = s & 1;
    f16x8 xh0, xl0, xh1, xl1;
    if (s < 2) {
      split_fh(xa0[2 * kc2], xa0[2 * kc2 + 1], sf[0], xh0, xl0);
      split_fh(xa1[2 * kc2], xa1[2 * kc2 + 1], sf[1], xh1, xl1);
    } else {
      split_fh(xb0[2 * kc2], xb0[2 * kc2 + 1], sf[0], xh0, xl0);
      split_fh(xb1[2 * kc2], xb1[2 * kc2 + 1], sf[1], xh1, xl1);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[cur][nt], xh0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2[cur][nt], xh1, acc[1][nt], 0, 0, 0);
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[cur][nt], xl0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[cur][nt], xl1, acc[1][nt], 0, 0, 0);
      acc[0][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[cur][nt], xh0, acc[0][nt], 0, 0, 0);
      acc[1][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[cur][nt], xh1, acc[1][nt], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
}

// The seven matrix scales kw (PK_FHS: Wf, then (Wm, Wu) per layer) as vector loads issued early; each use makes its
// value wave-uniform (readfirstlane), so the load latency is waited for at the first use, not at the kernel start.
// Seven separate members, not an array: with an array the per-layer select became a dynamically indexed private
// array (scratch memory), whose store at the staging and load at the top of every layer each forced a vmcnt(0) --
// waiting for every load and weight DMA in flight (the layer weights meant to land under the aggregation).
struct KwLoad {
  int v0, v1, v2, v3, v4, v5, v6;  // as loaded (VGPRs, in flight until ECO_KW_SCALARS reads them)
  __device__ __forceinline__ explicit KwLoad(const float* P)
      : v0(fh_kw(P, 0)), v1(fh_kw(P, 1)), v2(fh_kw(P, 2)), v3(fh_kw(P, 3)), v4(fh_kw(P, 4)), v5(fh_kw(P, 5)),
        v6(fh_kw(P, 6)) {
    static_assert(FH_NMAT == 7, "one member per packed matrix scale");
  }
};
// The scales as wave-uniform scalars, read once the staging's loads have landed (after its vmcnt(0)): seven SGPRs
// instead of seven VGPRs live through the layers (the paired kernel spilled with them), selected per layer from
// separate values (kept out of any array, which the compiler would index in scratch memory)
#define ECO_KW_SCALARS(kw)                                                                                  \
  const int kw_f = __builtin_amdgcn_readfirstlane((kw).v0), kw_m0 = __builtin_amdgcn_readfirstlane((kw).v1), \
            kw_u0 = __builtin_amdgcn_readfirstlane((kw).v2), kw_m1 = __builtin_amdgcn_readfirstlane((kw).v3), \
            kw_u1 = __builtin_amdgcn_readfirstlane((kw).v4), kw_m2 = __builtin_amdgcn_readfirstlane((kw).v5), \
            kw_u2 = __builtin_amdgcn_readfirstlane((kw).v6)
#define ECO_KW_MESSAGE(layer) ((layer) == 0 ? kw_m0 : ((layer) == 1 ? kw_m1 : kw_m2))
#define ECO_KW_UPDATE(layer) ((layer) == 0 ? kw_u0 : ((layer) == 1 ? kw_u1 : kw_u2))

__device__ __forceinline__ void zero_acc2(f32x4 (&d)[2][4]) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) d[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Staging of the wave's two tiles (d2_stage per tile): row norms, max degrees and spread adjacency words.  One
// graph per block with a prepared gs.adjbits: per-lane loads; otherwise row info / edge bases / max degrees in LDS
// and the block bitmask built once (barriers: uniform over the workgroup).
template <int NT, bool PREP>
__device__ __forceinline__ void d3_stage_raw(const MpnnArgs& a, int blk, int rows_pad, int rows_valid,
                                             const int (&r)[2], const bool (&valid)[2], int s4, int2* RI, int64_t* GB,
                                             int* MD, uint32_t* ADJ, float (&nf)[2], int (&md)[2],
                                             uint32_t (&adjb)[2][4], int gid_v) {
  const int N = a.N;
  if constexpr (PREP) {  // one graph per block with a prepared gs.adjbits (the launch decides: mpnn_dense3_prep)
    // gid_v: the block's graph id, loaded by the caller ahead of its other loads.  Every load here is unconditional
    // (rows clamped, results selected): a load skipped on some path turns each later wait into vmcnt(0), which
    // serialised the prologue's round trips (graph id, degrees, bitmask, node features)
    const int gid = uniform_i(gid_v);
    const int mdg = a.gs.max_deg[gid];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      // rows past the graph read row 0 (their degree only scales rows that are zeroed; their bitmask words are
      // masked by d3_spread, after the loads have long landed: a select here became a predicated load)
      const int rc = valid[t] ? r[t] : 0;
      const int dl = a.gs.deg[(size_t)gid * N + rc];
      const uint4 v = *reinterpret_cast<const uint4*>(a.gs.adjbits + (((size_t)gid * N + rc) * 4 + s4) * 4);
      adjb[t][0] = v.x; adjb[t][1] = v.y; adjb[t][2] = v.z; adjb[t][3] = v.w;
      nf[t] = (float)max(dl, 1);
      md[t] = mdg;
    }
  } else {
    const int g_valid = min(a.gpb, a.B - blk * a.gpb);
    for (int r2 = threadIdx.x; r2 < rows_pad; r2 += NT) RI[r2] = pack_row_info(a, blk, r2, rows_valid);
    for (int gl = threadIdx.x; gl < g_valid; gl += NT) {
      const int gid = a.gids[blk * a.gpb + gl];
      GB[gl] = a.gs.edge_base[gid];
      MD[gl] = a.gs.max_deg[gid];
    }
    lds_barrier();
    const bool built = adj_build<NT>(a, ADJ, RI, GB, rows_pad, rows_valid);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int rr = min(r[t], rows_pad - 1);
      nf[t] = (float)row_info(RI, rr).norm;
      md[t] = valid[t] ? MD[r[t] / N] : 1;
      adj_lane(a, ADJ, built, blk, r[t], rr, valid[t], s4, adjb[t]);
    }
    if (built) __syncthreads();
  }
}
// the bitmask words as the spread words of agg3 (the first use of the staged adjacency: placing it late lets the
// adjacency / degree loads of the prepared-bitmask path run under the forward's phase A)
__device__ __forceinline__ void d3_spread(const uint32_t (&adjb)[2][4], const bool (&valid)[2],
                                          uint32_t (&adjw)[2][DN_KC]) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kc = 0; kc < DN_KC; ++kc)
      adjw[t][kc] = valid[t] ? adj_spread((adjb[t][kc >> 1] >> (16 * (kc & 1))) & 0xFFFFu) : 0u;
}

// LDS (ECO_D2_LDS), as mpnn_forward_dense2_kernel.  NNET = 2: the online and the target network on the same graphs
// and features (a0 then a1), sharing the staging.
template <bool SAVE, int NNET, bool PREP>
__global__ __launch_bounds__(64 * D3_NW, 1) void mpnn_forward_dense3_kernel(MpnnArgs a0, MpnnArgs a1) {
  ECO_D2_LDS;
  const MpnnArgs& a = a0;  // the staging reads the graph fields, equal in a0 and a1
  ECO_TS(0);
  constexpr int NW = D3_NW;
  constexpr int NT = 64 * NW;
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int blk = blockIdx.x;
  const int N = a.N;
  const int g_valid = min(a.gpb, a.B - blk * a.gpb);
  const int rows_valid = g_valid * N;
  const int rows_pad = (a.gpb * N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  uint16_t* PL = sPL;
  uint16_t* PL1 = sPL + D2_PLANE;
  uint16_t* WB0 = sW0;
  uint16_t* WB1 = sW1;
  uint16_t* WB2 = sW2;
  int* TE = sTE;
  uint32_t* ADJ = reinterpret_cast<uint32_t*>(sPL);  // [rows_pad][DN_ADJW] while a bitmask is built
  const size_t R0 = (size_t)blk * a.gpb * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const uint16_t* PH = reinterpret_cast<const uint16_t*>(P + PK_FH);
  const int s4 = lane >> 4;
  const int c16 = lane & 15;

  const bool act = 2 * w < ntiles;  // the wave computes both of its tiles (a padding tile on zeros)
  int tl[2], r[2];
  bool has[2], valid[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    tl[t] = 2 * w + t;
    has[t] = tl[t] < ntiles;
    r[t] = tl[t] * 16 + c16;
    valid[t] = has[t] && r[t] < rows_valid;
  }
  // ---- staging: the graph id (first: the degree / bitmask loads depend on it); Wf fragments (LDS-DMA); node
  //      features, the 8-input Linears' weights and w_a; row norms, max degrees and adjacency operands of the
  //      lane's two rows.  Unconditional loads (rows clamped, results selected): see d3_stage_raw ----
  const int gid_v = a.gids[min(blk * a.gpb, a.B - 1)];
  __builtin_amdgcn_sched_barrier(0);  // issued before the loads below (waiting for it then leaves them in flight)
  glds_frags<NW>(WB0, PH + FH_WF, 16, w, lane);
  float xk0[2], xk1[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const size_t row = R0 + (valid[t] ? r[t] : 0);
    const float x0 = a.x[row * 8 + s4], x1 = a.x[row * 8 + 4 + s4];
    xk0[t] = valid[t] ? x0 : 0.f;
    xk1[t] = valid[t] ? x1 : 0.f;
  }
  float wx8[8], w08[8];
  lin8_load(P + PK_WX, lane, wx8);
  lin8_load(P + PK_W0, lane, w08);
  float4 wa4[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) wa4[c] = f4(P + PK_WA + 16 * c + 4 * s4);
  float nf[2];
  int md_graph[2];
  uint32_t adjb[2][4], adjw[2][DN_KC];
  d3_stage_raw<NT, PREP>(a, blk, rows_pad, rows_valid, r, valid, s4, sRI, sGB, sMD, ADJ, nf, md_graph, adjb, gid_v);
  ECO_TS(1);
  float rnf[2];
  // aggregation chunks of the wave's rows (the union of its two tiles' ranges)
  // a tile row recomputed from a laundered lane id where it is used after the staging, so the compiler does not keep
  // r[] live through the layers (the paired kernel spilled it and reloaded it with vmcnt(0), i.e. waiting for the
  // weight DMA in flight)
  auto row_of = [&](int t) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    return tl[t] * 16 + (ln & 15);
  };
  const int g_lo = min(w * 32, rows_pad - 1) / N, g_hi = min(w * 32 + 31, rows_pad - 1) / N;
  const int kc0 = (g_lo * N) >> 5;
  const int kc1 = (min((g_hi + 1) * N, rows_pad) + 31) >> 5;
  // one network (a: its weights and outputs); next: the network that runs after it in this launch, or null.
  // Called once per network with its own argument struct (no per-field selects between a0 and a1).
  auto net_body = [&](const MpnnArgs& a, const MpnnArgs* next, bool first) __attribute__((always_inline)) {
  const float* P = a.P;
  const uint16_t* PH = reinterpret_cast<const uint16_t*>(P + PK_FH);
  KwLoad kw(P);  // the matrix scales: loaded here, made wave-uniform where they are used
  if (!first) {
    lin8_load(P + PK_WX, lane, wx8);
    lin8_load(P + PK_W0, lane, w08);
#pragma unroll
    for (int c = 0; c < 4; ++c) wa4[c] = f4(P + PK_WA + 16 * c + 4 * s4);
  }
  zero_pad_rows2<NT>(PL, PL1, rows_pad);
  zero_pad_rows2<NT>(WB1, WB2, rows_pad);  // V planes

  // ---- phase A: Z = Wx . x (f32 MFMA); U = relu(Z + w_a) and V = relu(Z - w_a) planes ----
  if (act) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 z[4];
      lin8r(z, wx8, xk0[t], xk1[t]);
      float4 u[4], v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 wa = wa4[c];
        u[c] = valid[t] ? make_float4(relu(fmaf(1.f, wa.x, z[c][0])), relu(fmaf(1.f, wa.y, z[c][1])),
                                      relu(fmaf(1.f, wa.z, z[c][2])), relu(fmaf(1.f, wa.w, z[c][3])))
                        : zero4();
        v[c] = valid[t] ? make_float4(relu(fmaf(-1.f, wa.x, z[c][0])), relu(fmaf(-1.f, wa.y, z[c][1])),
                                      relu(fmaf(-1.f, wa.z, z[c][2])), relu(fmaf(-1.f, wa.w, z[c][3])))
                        : zero4();
      }
      if (has[t]) {
        tile_planes(PL, PL1, TE, tl[t], r[t], s4, u, lane);
        tile_planes(WB1, WB2, TE + 16, tl[t], r[t], s4, v, lane);
      }
    }
  }
  ECO_TS(9);
  glds_wait();  // Wf fragments
  ECO_TS(15);
  lds_barrier();
  D3_PRIO(3);
  ECO_TS(2);
  ECO_KW_SCALARS(kw);
  if (first) {  // the staged adjacency and degrees, first needed here
    d3_spread(adjb, valid, adjw);
#pragma unroll
    for (int t = 0; t < 2; ++t) rnf[t] = 1.f / nf[t];
  }

  // ---- phase B: edge embedding (mpnn.py:89-104): (A+ . relu(Z + w_a) + A- . relu(Z - w_a)) / norm; Wf ----
  float4 ereg[2][4];
  {
    const AggScale su = agg_scale(TE, ntiles, lane);
    const AggScale sv = agg_scale(TE + 16, ntiles, lane);
    f32x4 ea[2][4], ev[2][4];
    zero_acc2(ea);
    zero_acc2(ev);
    AGG3(1, ea, PL, PL1, adjw, su, kc0, kc1, lane);
    AGG3(2, ev, WB1, WB2, adjw, sv, kc0, kc1, lane);
    D3_PRIO(2);
    const int maxdeg_call = a.norm_scope == ECO_NORM_PER_CALL ? *a.call_maxdeg : 0;
    float4 acc[2][4];
    float sfx[2];
    int kx[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float t4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          t4[i] = (__builtin_ldexpf(ea[t][c][i], -su.c) + __builtin_ldexpf(ev[t][c][i], -sv.c)) * rnf[t];
        acc[t][c] = make_float4(t4[0], t4[1], t4[2], t4[3]);
      }
      // feature 63 = norm / norm.max()  (mpnn.py:102)
      const int md = a.norm_scope == ECO_NORM_PER_CALL ? maxdeg_call : (valid[t] ? md_graph[t] : 1);
      if (s4 == 3) acc[t][3].w = nf[t] / (float)md;
      if (!valid[t]) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[t][c] = zero4();
      } else if (SAVE) {
        float* eap = a.sv + (size_t)SV_EAGG * RT * 64 + (R0 + r[t]) * 64 + 4 * s4;
#pragma unroll
        for (int c = 0; c < 4; ++c) st4(eap + 16 * c, acc[t][c]);
      }
      kx[t] = node_exp<4>(acc[t]);
      sfx[t] = exp2i(kx[t]);
    }
    f32x4 d[2][4];
    zero_acc2(d);
    mm_fh_2t(d, acc[0], acc[1], sfx, WB0, lane);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      unscale(d[t], kx[t] + kw_f);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        ereg[t][nt] = relu4(d[t][nt]);
        if (SAVE && valid[t])
          st4(a.sv + (size_t)SV_E * RT * 64 + (R0 + r[t]) * 64 + 16 * nt + 4 * s4, ereg[t][nt]);
      }
      if (SAVE && valid[t]) store_mask(a, RT, R0 + r[t], s4, SM_E, pos_mask(ereg[t]));
    }
  }
  D3_PRIO(1);
  lds_barrier();  // every wave is done with the U / V planes and with Wf
  D3_PRIO(3);
  ECO_TS(3);
  // layer weights: Wm0 -> WB1, Wu0 -> WB2, Wm1 -> WB0 (landed by layer 0's first barrier)
  glds_frags<NW>(WB1, PH + FH_LAYER, 32, w, lane);
  glds_frags<NW>(WB2, PH + FH_LAYER + 2 * FH_HALF, 32, w, lane);
  glds_frags<NW>(WB0, PH + FH_LAYER + FH_LAYER_STRIDE, 32, w, lane);

  // ---- phase C: h0 = relu(W0 . x) (mpnn.py:20-23, :55), in registers + planes ----
  float4 hreg[2][4];
  if (act) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 z[4];
      lin8r(z, w08, xk0[t], xk1[t]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        hreg[t][c] = valid[t] ? relu4(z[c]) : zero4();
        if (SAVE && valid[t])
          st4(a.sv + (size_t)SV_H0 * RT * 64 + (R0 + r[t]) * 64 + 16 * c + 4 * s4, hreg[t][c]);
      }
      if (has[t]) tile_planes(PL, PL1, TE, tl[t], row_of(t), s4, hreg[t], lane);
      if (SAVE && valid[t]) store_mask(a, RT, R0 + r[t], s4, SM_H0, pos_mask(hreg[t]));
    }
  } else {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int c = 0; c < 4; ++c) hreg[t][c] = zero4();
  }
  lds_barrier();
  D3_PRIO(3);
  ECO_TS(4);

  // ---- phase D: 3 x UpdateNodeEmbeddingLayer (mpnn.py:114-120) ----
  for (int layer = 0; layer < 3; ++layer) {
    const uint16_t* WM = layer == 0 ? WB1 : (layer == 1 ? WB0 : WB2);
    const uint16_t* WU = layer == 0 ? WB2 : (layer == 1 ? WB1 : WB0);
    const int kwm = ECO_KW_MESSAGE(layer);  // scalar selects (KwLoad)
    const int kwu = ECO_KW_UPDATE(layer);
    if (layer == 1) {
      glds_frags<NW>(WB1, PH + FH_LAYER + FH_LAYER_STRIDE + 2 * FH_HALF, 32, w, lane);  // Wu1
      glds_frags<NW>(WB2, PH + FH_LAYER + 2 * FH_LAYER_STRIDE, 32, w, lane);            // Wm2
    } else if (layer == 2) {
      glds_frags<NW>(WB0, PH + FH_LAYER + 2 * FH_LAYER_STRIDE + 2 * FH_HALF, 32, w, lane);  // Wu2
    }
    const AggScale sh = agg_scale(TE, ntiles, lane);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int kc = 0; kc < DN_KC; ++kc) asm volatile("" : "+v"(adjw[t][kc]));  // no hoisting of the fragment masks
    f32x4 ag[2][4];
    zero_acc2(ag);
    AGG3(0, ag, PL, PL1, adjw, sh, kc0, kc1, lane);
    float4 agg[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float sc = __builtin_ldexpf(rnf[t], -sh.c);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        agg[t][c] = make_float4(ag[t][c][0] * sc, ag[t][c][1] * sc, ag[t][c][2] * sc, ag[t][c][3] * sc);
    }
    D3_PRIO(2);
    if (layer == 0) ECO_TS(10);
    glds_wait();
    lds_barrier();  // B1: planes read by every wave; this layer's weights landed
    D3_PRIO(3);
    if (layer == 0) ECO_TS(11);
    if (SAVE) {  // after the wait: stores count in vmcnt with the weight DMA
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (!valid[t]) continue;
        float* sa = a.sv + (size_t)(SV_AGG0 + layer) * RT * 64 + (R0 + r[t]) * 64 + 4 * s4;
#pragma unroll
        for (int c = 0; c < 4; ++c) st4(sa + 16 * c, agg[t][c]);
      }
    }
    // message = relu(Wm . [agg, e])
    float4 mrel[2][4];
    {
      f32x4 d[2][4];
      zero_acc2(d);
      int kx[2];
      float sf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        kx[t] = node_exp2(agg[t], ereg[t]);
        sf[t] = exp2i(kx[t]);
      }
        lin128_2t<D3_LIN_SPLIT_AHEAD && !SAVE && NNET == 1>(d, ereg[0], ereg[1], WM + FH_HALF, agg[0], agg[1], WM, sf, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        unscale(d[t], kx[t] + kwm);
#pragma unroll
        for (int c = 0; c < 4; ++c) mrel[t][c] = relu4(d[t][c]);
      }
    }
    if (SAVE) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (!valid[t]) continue;
        float* sm = a.sv + (size_t)(SV_M0 + layer) * RT * 64 + (R0 + r[t]) * 64 + 4 * s4;
#pragma unroll
        for (int c = 0; c < 4; ++c) st4(sm + 16 * c, mrel[t][c]);
        store_mask(a, RT, R0 + r[t], s4, SM_M0 + layer, pos_mask(mrel[t]));
      }
    }
    D3_PRIO(2);
    if (layer == 0) ECO_TS(12);
    // h' = relu(Wu . [h, m])
    {
      f32x4 hn[2][4];
      zero_acc2(hn);
      int kx[2];
      float sf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        kx[t] = node_exp2(hreg[t], mrel[t]);
        sf[t] = exp2i(kx[t]);
      }
        lin128_2t<D3_LIN_SPLIT_AHEAD && !SAVE && NNET == 1>(hn, hreg[0], hreg[1], WU, mrel[0], mrel[1], WU + FH_HALF, sf, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        unscale(hn[t], kx[t] + kwu);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          hreg[t][c] = valid[t] ? relu4(hn[t][c]) : zero4();
          if (SAVE && valid[t])
            st4(a.sv + (size_t)(SV_H0 + layer + 1) * RT * 64 + (R0 + r[t]) * 64 + 16 * c + 4 * s4, hreg[t][c]);
        }
        if (SAVE && valid[t]) store_mask(a, RT, R0 + r[t], s4, SM_H1 + layer, pos_mask(hreg[t]));
      }
    }
    D3_PRIO(1);
    if (layer == 0) ECO_TS(13);
    if (layer < 2) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (has[t]) tile_planes(PL, PL1, TE, tl[t], row_of(t), s4, hreg[t], lane);
    }
    D3_PRIO(0);
    if (layer == 0) ECO_TS(14);
    lds_barrier();  // B2: planes of h_{layer+1} complete; this layer's weight buffers free
    D3_PRIO(3);
    ECO_TS(5 + layer);
  }
  if (next)  // the next network's Wf into the free buffer, landing while this readout runs
    glds_frags<NW>(WB0, reinterpret_cast<const uint16_t*>(next->P + PK_FH) + FH_WF, 16, w, lane);

  // ---- phase E: readout (mpnn.py:143-159) + act ----
  if (a.gpb == 1) {
    // one graph: per node q_local = Wr[64:] . h3 and per tile the column sums of h3 go to LDS from registers; one
    // barrier; wave 0 reduces the tile partials in tile order, forms p = Wp . mean, relu(p) . Wr[:64], q and acts
    float* COL = reinterpret_cast<float*>(sPL);  // [ntiles][64]
    float* QL = COL + 16 * 64;                    // [rows_pad] q_local
    float* MEANS = QL + DN_MAX_ROWS;              // [64]
    float* QB = MEANS + 64;                       // [rows_pad] q
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (!has[t]) continue;
      float ql = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 wr = f4(P + PK_WR + 64 + 16 * c + 4 * s4);
        ql = fmaf(hreg[t][c].x, wr.x, ql);
        ql = fmaf(hreg[t][c].y, wr.y, ql);
        ql = fmaf(hreg[t][c].z, wr.z, ql);
        ql = fmaf(hreg[t][c].w, wr.w, ql);
      }
      auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(ql), __float_as_uint(ql), false, false);
      ql = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
      auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(ql), __float_as_uint(ql), false, false);
      ql = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
      if (s4 == 0) QL[row_of(t)] = ql;
      float cs[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        cs[4 * c] = row_sum16(hreg[t][c].x);
        cs[4 * c + 1] = row_sum16(hreg[t][c].y);
        cs[4 * c + 2] = row_sum16(hreg[t][c].z);
        cs[4 * c + 3] = row_sum16(hreg[t][c].w);
      }
      if (c16 == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          st4(COL + tl[t] * 64 + 16 * c + 4 * s4, make_float4(cs[4 * c], cs[4 * c + 1], cs[4 * c + 2], cs[4 * c + 3]));
      }
    }
    // wave 0's readout weights (its Wp row, Wr[lane], b) in flight across the barrier
    float4 wpv[16];
    float wr_l = 0.f, br = 0.f;
    if (w == 0) {
      const float* wp = P + PK_WP + lane * 64;
#pragma unroll
      for (int k = 0; k < 16; ++k) wpv[k] = f4(wp + 4 * k);
      wr_l = P[PK_WR + lane];
      br = P[PK_BR];
    }
    lds_barrier();
    if (w == 0) {
      float cs = 0.f;
      for (int t = 0; t < ntiles; ++t) cs += COL[t * 64 + lane];  // tile order
      const float mean = cs / (float)N;
      MEANS[lane] = mean;
      wave_lds_sync();
      float p = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float4 wv = wpv[k], mv = f4(MEANS + 4 * k);
        p = fmaf(wv.x, mv.x, p);
        p = fmaf(wv.y, mv.y, p);
        p = fmaf(wv.z, mv.z, p);
        p = fmaf(wv.w, mv.w, p);
      }
      if (SAVE) {
        a.sv[(size_t)SV_NODE_TENSORS * RT * 64 + (size_t)blk * 64 + lane] = mean;
        a.sv[(size_t)SV_NODE_TENSORS * RT * 64 + (size_t)a.B * 64 + (size_t)blk * 64 + lane] = p;
      }
      const float cg = wave_sum_f(relu(p) * wr_l);
      for (int i = lane; i < N; i += 64) {
        const float qv = cg + QL[i] + br;
        QB[i] = qv;
        if (a.q) a.q[R0 + i] = qv;
      }
      if (a.has_act) {
        wave_lds_sync();
        graph_act<NW>(a, QB, blk, 1, R0);
      }
    }
    ECO_TS(8);
    if (next) lds_barrier();  // wave 0's readout scratch (the plane array) before the next planes
    return;
  }
  // several graphs per block: h3 rows staged as fp32 [rows][D2_HS_LD] in the plane array
  float* Hs = reinterpret_cast<float*>(sPL);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (!has[t]) continue;
#pragma unroll
    for (int c = 0; c < 4; ++c) st4(Hs + row_of(t) * D2_HS_LD + 16 * c + 4 * s4, hreg[t][c]);
  }
  lds_barrier();
  float* Scr = reinterpret_cast<float*>(sW1);
  // the readout's column sums in dense2's order: 16 strided partials (DN_NW virtual waves) when split
  const bool split = a.gpb < DN_NW && readout_scratch_floats(rows_pad, a.gpb, DN_NW, true) * 4 <= D2_WBUF_BYTES;
  if (!split && readout_scratch_floats(rows_pad, a.gpb, DN_NW, false) * 4 > D2_WBUF_BYTES) return;  // launch checks
  readout_act<SAVE, NW, DN_NW>(a, Hs, D2_HS_LD, Scr, split, blk, g_valid, rows_valid, R0, RT);
  ECO_TS(8);
  if (next) lds_barrier();
  };  // net_body
  net_body(a0, NNET == 2 ? &a1 : nullptr, true);
  if constexpr (NNET == 2) net_body(a1, nullptr, false);
}

static int dense3_check(const MpnnArgs& a) {
  const int rows_pad = (a.gpb * a.N + 15) & ~15;
  if (rows_pad > DN_MAX_ROWS || a.gpb > D2_MAX_GPB) return fail(ECO_ERR_ARG, "dense MPNN block exceeds the LDS tables");
  if (readout_scratch_floats(rows_pad, a.gpb, DN_NW, false) * 4 > D2_WBUF_BYTES)
    return fail(ECO_ERR_ARG, "dense MPNN readout scratch exceeds its buffer");
  return ECO_OK;
}

// the staging path of the launch (one graph per block with a prepared gs.adjbits: per-lane loads) as a template
// argument: a run-time branch merged the two paths' registers and turned every staging wait into vmcnt(0)
inline bool mpnn_dense3_prep(const MpnnArgs& a) { return a.gpb == 1 && a.gs.adjbits != nullptr; }
static int mpnn_forward_dense3_launch(const MpnnArgs& a, bool save, hipStream_t st) {
  if (const int rc = dense3_check(a)) return rc;
  const int blocks = (a.B + a.gpb - 1) / a.gpb;
  const bool prep = mpnn_dense3_prep(a);
  if (save && prep) mpnn_forward_dense3_kernel<true, 1, true><<<blocks, 64 * D3_NW, 0, st>>>(a, a);
  else if (save) mpnn_forward_dense3_kernel<true, 1, false><<<blocks, 64 * D3_NW, 0, st>>>(a, a);
  else if (prep) mpnn_forward_dense3_kernel<false, 1, true><<<blocks, 64 * D3_NW, 0, st>>>(a, a);
  else mpnn_forward_dense3_kernel<false, 1, false><<<blocks, 64 * D3_NW, 0, st>>>(a, a);
  return check_launch("mpnn_forward_dense3");
}
static int mpnn_forward_dense3_pair_launch(const MpnnArgs& a, const MpnnArgs& b, hipStream_t st) {
  if (const int rc = dense3_check(a)) return rc;
  if (a.gpb != 1) return fail(ECO_ERR_ARG, "paired dense forward: one graph per block only");
  if (mpnn_dense3_prep(a)) mpnn_forward_dense3_kernel<false, 2, true><<<a.B, 64 * D3_NW, 0, st>>>(a, b);
  else mpnn_forward_dense3_kernel<false, 2, false><<<a.B, 64 * D3_NW, 0, st>>>(a, b);
  return check_launch("mpnn_forward_dense3_pair");
}


// ============================================================== backward ====
// Two output halves (fragment sets WH0, WH1) of one 64-input transposed Linear for both tiles, sharing each tile's
// split of x and every weight fragment read (mm_fh2's products per accumulator, in its order).
__device__ __forceinline__ void mm_fh2_2t(f32x4 (&acc0)[2][4], f32x4 (&acc1)[2][4], const float4 (&x0)[4],
                                          const float4 (&x1)[4], const float (&sf)[2], const uint16_t* WH0,
                                          const uint16_t* WH1, int lane) {
#pragma unroll
  for (int kc2 = 0; kc2 < 2; ++kc2) {
    f16x8 xh0, xl0, xh1, xl1;
    split_fh(x0[2 * kc2], x0[2 * kc2 + 1], sf[0], xh0, xl0);
    split_fh(x1[2 * kc2], x1[2 * kc2 + 1], sf[1], xh1, xl1);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const uint16_t* wl = (hh ? WH1 : WH0) + lane * 8;
      f16x8 wf1[4], wf2[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        wf1[nt] = *reinterpret_cast<const f16x8*>(wl + ((0 * 4 + nt) * 2 + kc2) * FH_FRAG);
        wf2[nt] = *reinterpret_cast<const f16x8*>(wl + ((1 * 4 + nt) * 2 + kc2) * FH_FRAG);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        f32x4& a0 = hh ? acc1[0][nt] : acc0[0][nt];
        f32x4& a1 = hh ? acc1[1][nt] : acc0[1][nt];
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf2[nt], xh0, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf2[nt], xh1, a1, 0, 0, 0);
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[nt], xl0, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[nt], xl1, a1, 0, 0, 0);
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[nt], xh0, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf1[nt], xh1, a1, 0, 0, 0);
      }
    }
  }
}

// Autograd of the forward (dqn.py:440-449): mpnn_backward_dense2_kernel's operations, laid out as the forward here
// (8 waves, tiles 2w and 2w + 1 per wave, shared fragment reads).  Every sum keeps dense2's order -- the readout's
// strided node sums run over 16 virtual waves, dw_a's per-tile partials are summed in tile order over 16 slots --
// so the gradients are bitwise those of mpnn_backward_dense2_kernel (tests/test_dense_gpu.py).
// LDS (ECO_D2_LDS): sPL 2 planes (readout scratch first) | sW0, sW1, sW2 | TE | RI | GB
template <bool PREP>
__global__ __launch_bounds__(64 * D3_NW, 1) void mpnn_backward_dense3_kernel(MpnnArgs a) {
  ECO_D2_LDS;
  ECO_TS(16);
  constexpr int NW = D3_NW;
  constexpr int NT = 64 * NW;
  constexpr int VNW = 16;  // dense2's wave count: the order of the readout's strided sums and of dw_a
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int blk = blockIdx.x;
  const int N = a.N;
  const int g_valid = min(a.gpb, a.B - blk * a.gpb);
  const int rows_valid = g_valid * N;
  const int rows_pad = (a.gpb * N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  uint16_t* PL = sPL;
  uint16_t* PL1 = sPL + D2_PLANE;
  uint32_t* ADJ = reinterpret_cast<uint32_t*>(sPL);
  float* lds = reinterpret_cast<float*>(sPL);  // readout / dw_a scratch
  uint16_t* WB0 = sW0;
  uint16_t* WB1 = sW1;
  uint16_t* WB2 = sW2;
  int* TE = sTE;
  const size_t R0 = (size_t)blk * a.gpb * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const uint16_t* PH = reinterpret_cast<const uint16_t*>(P + PK_FH);
  const float* sv = a.sv;
  float* gr = a.gr;
  const int s4 = lane >> 4;
  const int c16 = lane & 15;
  auto SV = [&](int t) { return sv + (size_t)t * RT * 64; };
  auto GR = [&](int t) { return gr + (size_t)t * RT * 64; };
  const float* MEAN = sv + (size_t)SV_NODE_TENSORS * RT * 64;
  const float* PP = MEAN + (size_t)a.B * 64;
  float* DP = gr + (size_t)GR_NODE_TENSORS * RT * 64;
  float* DWRA = DP + (size_t)a.B * 64;
  float* DWRB = DWRA + (size_t)a.B * 64;
  float* DBR = DWRB + (size_t)a.B * 64;
  float* DWA = DBR + ((a.B + 63) & ~63);  // [nblocks][64]
  auto WUT = [&](int l) { return PH + FHT_LAYER + l * FH_LAYER_STRIDE + 2 * FH_HALF; };  // Wu^T: 2 output halves
  auto WMT = [&](int l) { return PH + FHT_LAYER + l * FH_LAYER_STRIDE; };                // Wm^T: dagg, de halves
  KwLoad kw(P);  // the matrix scales: loaded here, made wave-uniform where they are used

  // ---- staging: the graph id (see the forward), Wu^T / Wm^T of layer 2 and Wu^T of layer 1 (LDS-DMA), row info,
  //      edge bases ----
  const int gid_v = a.gids[min(blk * a.gpb, a.B - 1)];
  __builtin_amdgcn_sched_barrier(0);
  glds_frags<NW>(WB0, WUT(2), 32, w, lane);
  glds_frags<NW>(WB1, WMT(2), 32, w, lane);
  glds_frags<NW>(WB2, WUT(1), 32, w, lane);
  const bool act = 2 * w < ntiles;
  int tl[2], rw[2], rr[2];
  bool has[2], valid[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    tl[t] = 2 * w + t;
    has[t] = tl[t] < ntiles;
    rw[t] = tl[t] * 16 + c16;
    valid[t] = has[t] && rw[t] < rows_valid;
    rr[t] = min(rw[t], rows_pad - 1);
  }
  float nf[2], rnf[2];
  int md_unused[2];
  uint32_t adjb[2][4], adjw[2][DN_KC];
  d3_stage_raw<NT, PREP>(a, blk, rows_pad, rows_valid, rw, valid, s4, sRI, sGB, sMD, ADJ, nf, md_unused, adjb, gid_v);
  const int g_lo = min(w * 32, rows_pad - 1) / N, g_hi = min(w * 32 + 31, rows_pad - 1) / N;
  const int kc0 = (g_lo * N) >> 5;
  const int kc1 = (min((g_hi + 1) * N, rows_pad) + 31) >> 5;
  const uint16_t* Msk = reinterpret_cast<const uint16_t*>(sv + sv_mask_offset_floats(RT, a.B));
  uint4 rmask[2];  // unconditional loads (row clamped), masked after the readout (see d3_stage_raw)
#pragma unroll
  for (int t = 0; t < 2; ++t)
    rmask[t] = *reinterpret_cast<const uint4*>(Msk + ((R0 + min(rw[t], rows_valid - 1)) * 4 + s4) * SM_TENSORS);
  ECO_TS(17);

  // ---- readout backward (mpnn.py:143-159), scratch in the plane region ----
  float* DQ = lds;                       // [rows_pad]
  float* DMEAN = DQ + rows_pad;          // [gpb][64]
  float* RED = DMEAN + a.gpb * 64;       // [gpb][VNW][64] (split)
  const bool split = a.gpb < VNW && (size_t)(rows_pad + a.gpb * 64 + a.gpb * VNW * 64) * 4 <= (size_t)D2_PL_BYTES;
  for (int i = threadIdx.x; i < rows_pad; i += NT) DQ[i] = i < rows_valid ? a.dq[R0 + i] : 0.f;
  // the per-graph waves' Wp columns (Wp[k][lane], k < 64) and p, loaded ahead: the dmean chain below then runs on
  // registers instead of waiting on 64 dependent-order L2 reads (same FMAs, same order)
  float wpk[64], p_pre = 0.f;
  if (w < g_valid) {
#pragma unroll
    for (int k = 0; k < 64; ++k) wpk[k] = P[PK_WP + k * 64 + lane];
    p_pre = PP[(size_t)(blk * a.gpb + w) * 64 + lane];
  }
  lds_barrier();
  if (split) {  // dWr[64:] = sum_v dq_v h3_v, over dense2's 16 strided partial sums (virtual waves w, w + 8)
    ECO_TS(29);
    for (int gl = 0; gl < g_valid; ++gl) {
      const float* h3 = SV(SV_H3) + (R0 + (size_t)gl * N) * 64;
      float dwb0 = 0.f, dwb1 = 0.f;  // virtual waves w and w + NW, interleaved
      for (int v = w; v < N; v += VNW) {
        const float dv0 = DQ[gl * N + v];
        const float dv1 = v + NW < N ? DQ[gl * N + v + NW] : 0.f;
        if (dv0 != 0.f) dwb0 = fmaf(dv0, h3[(size_t)v * 64 + lane], dwb0);
        if (dv1 != 0.f) dwb1 = fmaf(dv1, h3[(size_t)(v + NW) * 64 + lane], dwb1);
      }
      RED[(gl * VNW + w) * 64 + lane] = dwb0;
      RED[(gl * VNW + w + NW) * 64 + lane] = dwb1;
    }
    lds_barrier();
    ECO_TS(30);
  }
  for (int gl = w; gl < g_valid; gl += NW) {
    const int e = blk * a.gpb + gl;
    float sacc = 0.f;
    for (int v = lane; v < N; v += 64) sacc += DQ[gl * N + v];
    const float S = wave_sum_f(sacc);
    const float p = gl == w ? p_pre : PP[(size_t)e * 64 + lane];
    const float dp = P[PK_WR + lane] * S * (p > 0.f ? 1.f : 0.f);
    DP[(size_t)e * 64 + lane] = dp;
    DWRA[(size_t)e * 64 + lane] = relu(p) * S;
    if (lane == 0) DBR[e] = S;
    float dmean = 0.f;
    if (gl == w) {  // the prefetched columns (the wave's first graph)
#pragma unroll
      for (int k = 0; k < 64; ++k)
        dmean = fmaf(wpk[k], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dp), k)), dmean);
    } else {
#pragma unroll 16
      for (int k = 0; k < 64; ++k)
        dmean = fmaf(P[PK_WP + k * 64 + lane], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dp), k)),
                     dmean);
    }
    DMEAN[gl * 64 + lane] = dmean / (float)N;
    float dwb = 0.f;
    if (split) {
#pragma unroll
      for (int k = 0; k < VNW; ++k) dwb += RED[(gl * VNW + k) * 64 + lane];  // fixed order
    } else {
      const float* h3 = SV(SV_H3) + (R0 + (size_t)gl * N) * 64;
      for (int v = 0; v < N; ++v) {
        const float dv = DQ[gl * N + v];
        if (dv != 0.f) dwb = fmaf(dv, h3[(size_t)v * 64 + lane], dwb);
      }
    }
    DWRB[(size_t)e * 64 + lane] = dwb;
  }
  lds_barrier();
  ECO_TS(31);
  // dh3 (node-operand layout): dq_i * wr[64+f] + dmean_f / N
  float4 dh[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float dqi = valid[t] ? DQ[rw[t]] : 0.f;
    const int gl = rr[t] / N;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int f = 16 * c + 4 * s4;
      const float4 dm = valid[t] ? f4(DMEAN + gl * 64 + f) : zero4();
      dh[t][c] = make_float4(fmaf(dqi, P[PK_WR + 64 + f + 0], dm.x), fmaf(dqi, P[PK_WR + 64 + f + 1], dm.y),
                             fmaf(dqi, P[PK_WR + 64 + f + 2], dm.z), fmaf(dqi, P[PK_WR + 64 + f + 3], dm.w));
    }
  }
  glds_wait();     // Wu^T / Wm^T of layer 2 and Wu^T of layer 1 (staged at the start) are read from here on
  lds_barrier();  // readout scratch dead: zero the plane rows [rows_pad, KP) no tile writes
  ECO_KW_SCALARS(kw);
  zero_pad_rows2<NT>(PL, PL1, rows_pad);
  // the staged adjacency and degrees, first needed by the layers (their loads ran under the readout backward)
  d3_spread(adjb, valid, adjw);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    rnf[t] = 1.f / nf[t];
    if (!valid[t]) rmask[t] = make_uint4(0u, 0u, 0u, 0u);
  }
  ECO_TS(18);

  // ---- update layers in reverse (mpnn.py:114-120) ----
  float4 de[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) de[t][c] = zero4();
  for (int layer = 2; layer >= 0; --layer) {
    const uint16_t* WU = layer == 2 ? WB0 : (layer == 1 ? WB2 : WB1);
    const uint16_t* WM = layer == 2 ? WB1 : (layer == 1 ? WB0 : WB2);
    const int kwm = ECO_KW_MESSAGE(layer);
    const int kwu = ECO_KW_UPDATE(layer);
    // duu = dh' * [h' > 0]  (in place in dh)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t hmask = mask16(rmask[t], SM_H0 + layer + 1);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        dh[t][c] = masked(f32x4{dh[t][c].x, dh[t][c].y, dh[t][c].z, dh[t][c].w}, hmask, c);
    }
    // [dh_direct, dm] = Wu^T . duu;  dum = dm * [m > 0]
    f32x4 dhd[2][4];
    float4 dum[2][4];
    {
      f32x4 dmm[2][4];
      zero_acc2(dhd);
      zero_acc2(dmm);
      int kx[2];
      float sf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        kx[t] = node_exp<4>(dh[t]);
        sf[t] = exp2i(kx[t]);
      }
      mm_fh2_2t(dhd, dmm, dh[0], dh[1], sf, WU, WU + FH_HALF, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ku = kx[t] + kwu;
        unscale(dhd[t], ku);
        unscale(dmm[t], ku);
        const uint32_t mmask = mask16(rmask[t], SM_M0 + layer);
#pragma unroll
        for (int c = 0; c < 4; ++c) dum[t][c] = masked(dmm[t][c], mmask, c);
      }
    }
    D3_PRIO(2);
    if (layer == 1) ECO_TS(24);
    glds_wait();
    lds_barrier();  // B0: Wm^T landed
    D3_PRIO(3);
    if (layer == 1) ECO_TS(25);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (!valid[t]) continue;  // stored after the wait: stores count in vmcnt with the weight DMA
      const size_t ro = (R0 + rr[t]) * 64 + 4 * s4;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        st4(GR(GR_DUU0 + layer) + ro + 16 * c, dh[t][c]);
        st4(GR(GR_DUM0 + layer) + ro + 16 * c, dum[t][c]);
      }
    }
    // [dagg, de] = Wm^T . dum;  G = dagg / norm -> planes
    {
      f32x4 dg[2][4], dd[2][4];
      zero_acc2(dg);
      zero_acc2(dd);
      int kx[2];
      float sf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        kx[t] = node_exp<4>(dum[t]);
        sf[t] = exp2i(kx[t]);
      }
      mm_fh2_2t(dg, dd, dum[0], dum[1], sf, WM, WM + FH_HALF, lane);
      D3_PRIO(2);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int km = kx[t] + kwm;
        unscale(dg[t], km);
        unscale(dd[t], km);
        float4 g[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          de[t][c].x += dd[t][c][0]; de[t][c].y += dd[t][c][1]; de[t][c].z += dd[t][c][2]; de[t][c].w += dd[t][c][3];
          g[c] = valid[t] ? make_float4(dg[t][c][0] * rnf[t], dg[t][c][1] * rnf[t], dg[t][c][2] * rnf[t],
                                        dg[t][c][3] * rnf[t])
                          : zero4();
        }
        if (has[t]) tile_planes(PL, PL1, TE, tl[t], rw[t], s4, g, lane);
      }
    }
    D3_PRIO(1);
    if (layer == 1) ECO_TS(26);
    lds_barrier();  // B1: G planes complete; every wave is past both Linears: this layer's weight buffers free
    D3_PRIO(3);
    if (layer == 2) {
      glds_frags<NW>(WB0, WMT(1), 32, w, lane);
      glds_frags<NW>(WB1, WUT(0), 32, w, lane);
    } else if (layer == 1) {
      glds_frags<NW>(WB2, WMT(0), 32, w, lane);
      glds_frags<NW>(WB0, PH + FHT_WF, 16, w, lane);  // Wf^T for the edge layer
    }
    if (layer == 1) ECO_TS(27);
    // dh_layer = dh_direct + A^T . G  (A symmetric: the forward aggregation)
    {
      const AggScale sg = agg_scale(TE, ntiles, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int kc = 0; kc < DN_KC; ++kc) asm volatile("" : "+v"(adjw[t][kc]));
      f32x4 ag[2][4];
      zero_acc2(ag);
      AGG3(0, ag, PL, PL1, adjw, sg, kc0, kc1, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float t4[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) t4[i] = dhd[t][c][i] + __builtin_ldexpf(ag[t][c][i], -sg.c);
          dh[t][c] = valid[t] ? make_float4(t4[0], t4[1], t4[2], t4[3]) : zero4();
        }
    }
    D3_PRIO(2);
    if (layer == 1) ECO_TS(28);
    lds_barrier();  // B2: planes read
    D3_PRIO(3);
    ECO_TS(21 - layer);
  }

  // ---- h0 = relu(W0.x): du0;  edge embedding (mpnn.py:89-104): due, dEagg = Wf^T . due -> G planes ----
  glds_wait();
  lds_barrier();  // Wf^T landed
  {
    float4 due[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const size_t ro = (R0 + rr[t]) * 64 + 4 * s4;
      const uint32_t h0m = mask16(rmask[t], SM_H0), em = mask16(rmask[t], SM_E);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (valid[t])
          st4(GR(GR_DU0) + ro + 16 * c, masked(f32x4{dh[t][c].x, dh[t][c].y, dh[t][c].z, dh[t][c].w}, h0m, c));
        due[t][c] = masked(f32x4{de[t][c].x, de[t][c].y, de[t][c].z, de[t][c].w}, em, c);
        if (valid[t]) st4(GR(GR_DUE) + ro + 16 * c, due[t][c]);
      }
    }
    f32x4 dg[2][4];
    zero_acc2(dg);
    int kx[2];
    float sf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      kx[t] = node_exp<4>(due[t]);
      sf[t] = exp2i(kx[t]);
    }
    mm_fh_2t(dg, due[0], due[1], sf, WB0, lane);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      unscale(dg[t], kx[t] + kw_f);
      float4 g[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        g[c] = valid[t] ? make_float4(dg[t][c][0] * rnf[t], dg[t][c][1] * rnf[t], dg[t][c][2] * rnf[t],
                                      dg[t][c][3] * rnf[t])
                        : zero4();
      if (has[t]) tile_planes(PL, PL1, TE, tl[t], rw[t], s4, g, lane);
    }
  }
  lds_barrier();
  ECO_TS(22);
  // dz_j = [z_j + w_a > 0] (A+ . G)_j + [z_j - w_a > 0] (A- . G)_j;  dw_a = sum_j of the same with signs
  {
    float xk0[2], xk1[2];  // inputs of Z, loaded ahead of the aggregations (row clamped: invalid rows masked below)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const size_t row = R0 + min(rw[t], rows_valid - 1);
      xk0[t] = a.x[row * 8 + s4];
      xk1[t] = a.x[row * 8 + 4 + s4];
    }
    float wx8[8];
    lin8_load(P + PK_WX, lane, wx8);
    float4 wa4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) wa4[c] = f4(P + PK_WA + 16 * c + 4 * s4);
    const AggScale sg = agg_scale(TE, ntiles, lane);
    f32x4 gp[2][4], gm[2][4];
    zero_acc2(gp);
    zero_acc2(gm);
    AGG3(1, gp, PL, PL1, adjw, sg, kc0, kc1, lane);
    AGG3(2, gm, PL, PL1, adjw, sg, kc0, kc1, lane);
    float dwacc[2][16];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 zz[4];
      lin8r(zz, wx8, xk0[t], xk1[t]);  // Z exactly as the forward computed it
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float dz4[4];
        const float wav[4] = {wa4[c].x, wa4[c].y, wa4[c].z, wa4[c].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float z = zz[c][i];
          const float wa = wav[i];
          const float tp = fmaf(1.f, wa, z) > 0.f ? __builtin_ldexpf(gp[t][c][i], -sg.c) : 0.f;
          const float tm = fmaf(-1.f, wa, z) > 0.f ? __builtin_ldexpf(gm[t][c][i], -sg.c) : 0.f;
          dz4[i] = valid[t] ? tp + tm : 0.f;
          dwacc[t][4 * c + i] = valid[t] ? 0.f + (tp - tm) : 0.f;  // dense2: 0 + (tp - tm) per wave = tile
        }
        if (valid[t])
          st4(GR(GR_DZ) + (R0 + rw[t]) * 64 + 16 * c + 4 * s4, make_float4(dz4[0], dz4[1], dz4[2], dz4[3]));
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) dwacc[t][i] = row_sum16(dwacc[t][i]);
    }
    lds_barrier();  // every wave is done reading the G planes: the region becomes the dwa scratch
    float* REDW = lds;  // [VNW][64]: one partial per tile slot (dense2: per wave = tile), zero past the tiles
    if (c16 == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          st4(REDW + tl[t] * 64 + 16 * c + 4 * s4,
              make_float4(dwacc[t][4 * c], dwacc[t][4 * c + 1], dwacc[t][4 * c + 2], dwacc[t][4 * c + 3]));
    }
    lds_barrier();
    if (w == 0) {
      float sacc = 0.f;
#pragma unroll
      for (int k = 0; k < VNW; ++k) sacc += REDW[k * 64 + lane];
      DWA[(size_t)blk * 64 + lane] = sacc;
    }
  }
  ECO_TS(23);
}

static int mpnn_backward_dense3_launch(const MpnnArgs& a, hipStream_t st) {
  if (const int rc = dense3_check(a)) return rc;
  const int blocks = (a.B + a.gpb - 1) / a.gpb;
  if (mpnn_dense3_prep(a)) mpnn_backward_dense3_kernel<true><<<blocks, 64 * D3_NW, 0, st>>>(a);
  else mpnn_backward_dense3_kernel<false><<<blocks, 64 * D3_NW, 0, st>>>(a);
  return check_launch("mpnn_backward_dense3");
}

}  // namespace eco
