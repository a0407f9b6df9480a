// Dense-aggregation MPNN forward on fp16x2 operands (src/networks/mpnn.py:40-159) for blocks of <= 224 rows
// with +-1 edge weights (ER-20 ... ER-200): the successor of eco_mpnn_dense.h's bf16x3 kernel.
//
// Every MFMA operand that is not exactly representable is carried as TWO fp16 pieces of a power-of-two-scaled
// value: v 2^k = V1 + V2, V1 = fp16(v 2^k), V2 = fp16(v 2^k - V1) (round to nearest, 22 significand bits:
// representation error <= 2^-22 |v|), on v_mfma_f32_16x16x32_f16 with f32 accumulation.  The scale 2^k puts the
// operand's block maximum into [2^14, 2^15), inside fp16's normal range whatever the magnitudes (activations of a
// std-0.01 network fall by ~10x per layer).  Against the bf16x3 forms of eco_mpnn_dense.h this needs 2/3 of the
// aggregation MFMAs and LDS reads (two planes instead of three) and half of the Linear MFMAs (three products
// W1.X1 + W1.X2 + W2.X1 instead of six).  The dropped W2.X2 is 2^-22 of the largest product; measured against
// float64 the products are closer than torch's own fp32 matmul (tools: /tmp f16 emulation in DESIGN.md §5).
//
//   * Aggregation agg[f][i] = sum_j H[j][f] A[j][i]: the planes hold H of tile t (16 rows) scaled by 2^k_t (k_t
//     from the tile's max |h|, written by the wave that owns the tile next to its planes); the adjacency operand,
//     built in registers from bitmasks, carries +-2^(c - k_t) instead of +-1 (exact in fp16 for
//     c - k_t in [-21, 15]; c = 15 + min_t k_t per aggregation), so every product is h 2^c and the f32 sum is
//     scaled back by 2^-c -- folded into the 1/norm multiply.  Rows of a tile more than 2^36 below the block's
//     largest tile get a zero operand (they contribute < 2^-36 of the largest term).
//   * Linears: weights pre-split per matrix (PK_FH, scale 2^kw); activations scaled per node by 2^kx (node max
//     over the Linear's 64 or 128 inputs: four lanes hold one node, combined with permlane swaps), unscaled by
//     2^-(kx + kw) after the f32 accumulation.
//
// One 1024-thread workgroup (16 waves) per block of whole graphs, wave w owns 16-node tile w (h and e in
// registers), as eco_mpnn_dense.h.  LDS keeps a whole layer's weights resident (three rotating 32-KB buffers:
// message and update Linear of the layer + the next layer's message Linear prefetched by LDS-DMA), so a layer
// has two barriers (planes ready -> aggregation; aggregation done + weights landed -> Linears -> next planes)
// instead of four; the edge layer writes the U and V planes at once (V into the two idle weight buffers).
// Saved activations and ReLU masks have the layout of eco_mpnn_dense.h (the backward reads them unchanged).
#pragma once
#include "eco_mpnn_dense.h"

namespace eco {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

constexpr int D2_PLANE = 4 * DN_KPMAX * 16;           // fp16 per plane: [4 feature blocks][224 rows][16]
constexpr int D2_PL_BYTES = 2 * D2_PLANE * 2;          // two planes: 57,344 B
constexpr int D2_WBUF = 2 * FH_HALF;                   // fp16 per weight buffer: one 128-input Linear (32 KB)
constexpr int D2_WBUF_BYTES = D2_WBUF * 2;
constexpr int D2_TE_INTS = 32;                         // tile exponents: [0..15] current planes, [16..31] V planes
constexpr int D2_K_EMPTY = 127;                        // tile exponent of an all-zero tile
constexpr int D2_HS_LD = 68;                           // fp32 row stride of the readout's h3 rows (conflict-free)
constexpr int D2_PL_U16 = DN_MAX_ROWS * D2_HS_LD * 2;  // plane array: 2 planes (57,344 B) or the h3 rows (60,928 B)
constexpr int D2_MAX_GPB = 52;                         // graphs per block (N >= 4, <= 208 rows)
static_assert(2 * D2_PLANE <= D2_PL_U16, "planes fit the plane array");
// The LDS is declared as separate static arrays (planes, three weight buffers, small tables) rather than one
// dynamic block: the waitcnt pass then knows that an LDS-DMA into one weight buffer cannot alias the planes or
// another buffer, and does not make the aggregation's plane reads wait for weight fragments still in flight.
#define ECO_D2_LDS                                                                   \
  __shared__ __attribute__((aligned(16))) uint16_t sPL[D2_PL_U16];                  \
  __shared__ __attribute__((aligned(16))) uint16_t sW0[D2_WBUF];                    \
  __shared__ __attribute__((aligned(16))) uint16_t sW1[D2_WBUF];                    \
  __shared__ __attribute__((aligned(16))) uint16_t sW2[D2_WBUF];                    \
  __shared__ int sTE[D2_TE_INTS];                                                    \
  __shared__ int2 sRI[DN_MAX_ROWS];                                                  \
  __shared__ int64_t sGB[D2_MAX_GPB];                                                \
  __shared__ int sMD[D2_MAX_GPB]

// ---- fp16x2 splitting -------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pk_f16(float a, float b) {
  const f32x2v v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2v));  // v_cvt_pk_f16_f32 (RNE)
}
// (a, b) scaled by the power of two sf into fp16 range -> hi and lo fp16 pairs with a sf = hi + lo to 2^-22.
// lo = fp16(a sf - hi) in ONE v_fma_mix{lo,hi}_f16 per value (f32 a and sf, f16 hi, single rounding: a sf - hi
// is exact, so the result is bitwise that of converting hi back, subtracting and converting: 4 VALU per pair
// instead of 6, the per-layer split being the largest VALU item of the dense kernels)
// The asm text, shared with the hazard probe (eco_probe_split2_mfma order 2, which places an MFMA reading the
// register straight after the last v_fma_mixhi): d = a sf - h, written to the low / high half of d.
#define ECO_MIXLO(d, a, s, h) "v_fma_mixlo_f16 " d ", " a ", " s ", -" h " op_sel_hi:[0,0,1]"
#define ECO_MIXHI(d, a, s, h) "v_fma_mixhi_f16 " d ", " a ", " s ", -" h " op_sel:[0,0,1] op_sel_hi:[0,0,1]"
// the trailing wait states: the hazard recognizer does not see inside inline asm, and an MFMA reading a VGPR
// written by VALU needs 2 (without them the fragments fed to the MFMAs were stale in some schedules)
#ifndef ECO_SPLIT2_NEGATIVE_CONTROL
#define ECO_SPLIT2_WAIT "\n\ts_nop 1"
#else  // tests/test_split2_hazard_gpu.py's negative control (a tools build only): the wait states removed
#define ECO_SPLIT2_WAIT ""
#endif
__device__ __forceinline__ void split2_pk(float a, float b, float sf, uint32_t& hi, uint32_t& lo) {
  hi = pk_f16(a * sf, b * sf);
  uint32_t l;  // mixlo writes bits 15:0 (16:31 kept, then written by mixhi)
  asm(ECO_MIXLO("%0", "%1", "%2", "%3") : "=v"(l) : "v"(a), "v"(sf), "v"(hi));
  asm(ECO_MIXHI("%0", "%1", "%2", "%3") ECO_SPLIT2_WAIT : "+v"(l) : "v"(b), "v"(sf), "v"(hi));
  lo = l;
}
// the same split by plain conversions (v_cvt_pk_f16_f32, f32 subtract, convert): the reference of
// eco_probe_split2_mfma (bitwise equal to split2_pk by construction: a sf - hi is exact in f32)
__device__ __forceinline__ void split2_ref(float a, float b, float sf, uint32_t& hi, uint32_t& lo) {
  hi = pk_f16(a * sf, b * sf);
  const f16x2v h = __builtin_bit_cast(f16x2v, hi);
  lo = pk_f16(a * sf - (float)h[0], b * sf - (float)h[1]);
}
// 2^k as a float (k clamped to the normal range)
__device__ __forceinline__ float exp2i(int k) {
  k = k < -126 ? -126 : (k > 127 ? 127 : k);
  return __int_as_float((k + 127) << 23);
}

// wave-wide max of non-negative floats (DPP row rotations, then across rows with permlane swaps)
__device__ __forceinline__ float wave_max_nonneg(float m) {
  int v = __float_as_int(m);
  v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x128, 0xF, 0xF, false));  // row_ror:8
  v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x124, 0xF, 0xF, false));  // row_ror:4
  v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x122, 0xF, 0xF, false));  // row_ror:2
  v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x121, 0xF, 0xF, false));  // row_ror:1
  auto s16 = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
  v = max((int)s16[0], (int)s16[1]);
  auto s32 = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
  return __int_as_float(max((int)s32[0], (int)s32[1]));  // non-negative floats order as ints
}
// max over the four lanes l, l^16, l^32, l^48 (one node of the node-operand layout) of a non-negative float
__device__ __forceinline__ float node_max_nonneg(float m) {
  // integer max: non-negative floats order as their bit patterns (fmaxf canonicalised both operands first)
  auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  const uint32_t a = max(s16[0], s16[1]);
  auto s32 = __builtin_amdgcn_permlane32_swap(a, a, false, false);
  return __uint_as_float(max(s32[0], s32[1]));
}
// scale exponent k with max 2^k in [2^14, 2^15) (0 for an all-zero / non-finite max)
__device__ __forceinline__ int scale_exp(float mx) {
  if (!(mx > 0.f) || mx == INFINITY) return 0;
  int k = 15 - __builtin_amdgcn_frexp_expf(mx);
  return k < -110 ? -110 : (k > 110 ? 110 : k);
}
__device__ __forceinline__ float absmax4(const float4& v, float m) {
  return fmaxf(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))), m);
}

// 8 activations (float4 c = 2kc2, 2kc2+1 of a 64-input half) scaled by sf, as hi / lo fp16 B fragments
__device__ __forceinline__ void split_fh(const float4& a, const float4& b, float sf, f16x8& hi, f16x8& lo) {
  uint32_t h0, h1, h2, h3, l0, l1, l2, l3;
  split2_pk(a.x, a.y, sf, h0, l0);
  split2_pk(a.z, a.w, sf, h1, l1);
  split2_pk(b.x, b.y, sf, h2, l2);
  split2_pk(b.z, b.w, sf, h3, l3);
  const u32x4v h = {h0, h1, h2, h3}, l = {l0, l1, l2, l3};
  hi = __builtin_bit_cast(f16x8, h);
  lo = __builtin_bit_cast(f16x8, l);
}

// acc[nt] += W[16nt + .][one 64-input half] . x for x = hi + lo (split_fh of the half's four float4), three
// products (smallest first).  WH: the half's 16 fragments [p][nt][kc2] in LDS.
__device__ __forceinline__ void mm_fh(f32x4 (&acc)[4], const float4 (&x)[4], float sf, const uint16_t* WH, int lane) {
  const uint16_t* wl = WH + lane * 8;
#pragma unroll
  for (int kc2 = 0; kc2 < 2; ++kc2) {
    f16x8 xh, xl;
    split_fh(x[2 * kc2], x[2 * kc2 + 1], sf, xh, xl);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const f16x8 w1 = *reinterpret_cast<const f16x8*>(wl + ((0 * 4 + nt) * 2 + kc2) * FH_FRAG);
      const f16x8 w2 = *reinterpret_cast<const f16x8*>(wl + ((1 * 4 + nt) * 2 + kc2) * FH_FRAG);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2, xh, acc[nt], 0, 0, 0);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, xl, acc[nt], 0, 0, 0);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, xh, acc[nt], 0, 0, 0);
    }
  }
}

// Workgroup barrier for LDS data only: waits for this wave's LDS operations (lgkmcnt), not for its global loads,
// stores or LDS-DMA (vmcnt).  __syncthreads() would drain vmcnt whenever an LDS-DMA is pending (the fence covers
// the DMA's LDS writes), which exposes every weight prefetch and global load in flight at the first barrier; here
// each barrier that publishes DMA-staged weights is preceded by an explicit glds_wait() instead.  The "memory"
// clobber keeps the compiler from moving memory operations across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// the lane's 8 weights of lin8 (W[16 nt + (l & 15)][l >> 4 | 4 + (l >> 4)], nt = 0..3), loaded ahead of use
__device__ __forceinline__ void lin8_load(const float* W, int lane, float (&wv)[8]) {
  const float* wl = W + (lane & 15) * 8 + (lane >> 4);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    wv[2 * nt] = wl[nt * 128];
    wv[2 * nt + 1] = wl[nt * 128 + 4];
  }
}
// lin8 of eco_mpnn_dense.h on preloaded weights (same products, same order)
__device__ __forceinline__ void lin8r(f32x4 (&d)[4], const float (&wv)[8], float xk0, float xk1) {
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    d[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[2 * nt], xk0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    d[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[2 * nt + 1], xk1, d[nt], 0, 0, 0);
  }
}
// sum over the 16 lanes of a row (the lanes l with equal l >> 4), every lane of the row gets it
__device__ __forceinline__ float row_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x128, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x124, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x122, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x121, 0xF, 0xF, false));
  return v;
}

// node scale of a Linear's inputs (the lane's float4s of every half)
template <int NC>
__device__ __forceinline__ int node_exp(const float4 (&x)[NC]) {
  float m = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) m = absmax4(x[c], m);
  return scale_exp(node_max_nonneg(m));
}
__device__ __forceinline__ int node_exp2(const float4 (&x)[4], const float4 (&y)[4]) {
  float m = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) m = absmax4(y[c], absmax4(x[c], m));
  return scale_exp(node_max_nonneg(m));
}
__device__ __forceinline__ void unscale(f32x4 (&acc)[4], int k) {
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[nt][i] = __builtin_ldexpf(acc[nt][i], -k);
}
// scale exponent of packed matrix m: a SCALAR load through the constant address space (P and m are uniform, the
// packed parameters are read-only during every kernel), so its wait is lgkmcnt and never vmcnt -- a vector load
// here, used right away, made the wave wait for every older vector load and weight DMA in flight
__device__ __forceinline__ int fh_kw(const float* P, int m) {
  return ((const __attribute__((address_space(4))) int*)(P + PK_FHS))[m];
}

// ---- planes ---------------------------------------------------------------------------------------------------
// tile scale exponent of the wave's 16 nodes x 64 features (identical in every lane; D2_K_EMPTY for all zero)
__device__ __forceinline__ int tile_exp(const float4 (&v)[4]) {
  float m = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) m = absmax4(v[c], m);
  const float mx = wave_max_nonneg(m);
  return mx > 0.f ? scale_exp(mx) : D2_K_EMPTY;
}
// features 16ft + 4k .. +3 of node j, scaled by sf, as two fp16 planes
__device__ __forceinline__ void plane2_store4(uint16_t* P0, uint16_t* P1, int ft, int j, int k, float4 v, float sf) {
  uint32_t h0, l0, h1, l1;
  split2_pk(v.x, v.y, sf, h0, l0);
  split2_pk(v.z, v.w, sf, h1, l1);
  const int o = plane_off(ft, j, k);
  *reinterpret_cast<uint2*>(P0 + o) = make_uint2(h0, h1);
  *reinterpret_cast<uint2*>(P1 + o) = make_uint2(l0, l1);
}
// the tile's four float4 (node-operand layout) scaled by 2^k into the planes; lane 0 records k in TE[tile]
__device__ __forceinline__ void tile_planes(uint16_t* P0, uint16_t* P1, int* TE, int tile, int r, int s4,
                                            const float4 (&v)[4], int lane) {
  const int k = tile_exp(v);
  const float sf = exp2i(k == D2_K_EMPTY ? 0 : k);
#pragma unroll
  for (int c = 0; c < 4; ++c)
    plane2_store4(P0, P1, c, r, s4, v[c], sf);
  if (lane == 0) TE[tile] = k;
}

// Per aggregation: from the tile exponents TE[0 .. ntiles) -> c (products are h 2^c) and, per tile t, the fp16
// pattern of the adjacency magnitude 2^(c - k_t) replicated in both halves of a dword (0: dropped / empty tile).
// Lane t < 16 works on tile t; the caller reads pattern t with readlane.
struct AggScale {
  uint32_t pat;  // lane t: pattern of tile t
  int c;
};
__device__ __forceinline__ AggScale agg_scale(const int* TE, int ntiles, int lane) {
  const int t = lane & 15;
  const int k = t < ntiles ? TE[t] : D2_K_EMPTY;
  int kmin = k;  // min over the row (lanes 0..15 hold tiles 0..15)
  kmin = min(kmin, __builtin_amdgcn_update_dpp(kmin, kmin, 0x128, 0xF, 0xF, false));
  kmin = min(kmin, __builtin_amdgcn_update_dpp(kmin, kmin, 0x124, 0xF, 0xF, false));
  kmin = min(kmin, __builtin_amdgcn_update_dpp(kmin, kmin, 0x122, 0xF, 0xF, false));
  kmin = min(kmin, __builtin_amdgcn_update_dpp(kmin, kmin, 0x121, 0xF, 0xF, false));
  kmin = __builtin_amdgcn_readfirstlane(kmin);
  AggScale s;
  s.c = kmin == D2_K_EMPTY ? 0 : 15 + kmin;
  const int E = s.c - k;  // <= 15 by the choice of c
  uint32_t p = 0u;
  if (k != D2_K_EMPTY) p = E >= -14 ? (uint32_t)(E + 15) << 10 : (E >= -21 ? 1u << (E + 24) : 0u);
  s.pat = p | (p << 16);
  return s;
}

// B fragment (8 fp16 adjacency entries of the lane's node for the chunk's k slots) from a spread word; PPlo / PPhi:
// magnitude patterns of the chunk's two tiles.  MODE 0: A (signed); 1: A+ = [A = +1]; 2: A- = [A = -1] as +1.
// Per dword t: the 0/1 edge bits of the two halves times the magnitude pattern in one v_pk_mul_lo_u16, and (MODE 0)
// the sign bits moved to bits 15 / 31 in one v_and_or: 5 VALU per dword instead of 7 (the adjacency fragments are
// the largest VALU item of the aggregations; bitwise the same fragments)
typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
template <int MODE>
__device__ __forceinline__ f16x8 adj_frag2(uint32_t W, uint32_t PPlo, uint32_t PPhi) {
  const uint32_t Wm = MODE == 0 ? W : (MODE == 1 ? (W & ~(W >> 4)) : (W >> 4));  // bit t: edge (+1 edge, -1 edge)
  u32x4v d;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    // the edge bit stays at bit t (value 2^t) and the pattern is shifted down instead (scalar, uniform): exact, the
    // patterns having no bit below bit 3 (agg_scale: normal fp16 powers of two, subnormals down to 2^-21 only)
    const uint32_t PP = (t < 2 ? PPlo : PPhi) >> t;
    const u16x2v on = __builtin_bit_cast(u16x2v, Wm & (0x10001u << t));
    uint32_t v = __builtin_bit_cast(uint32_t, on * __builtin_bit_cast(u16x2v, PP));
    if (MODE == 0) v |= (W << (11 - t)) & 0x80008000u;  // -1 edge bits t + 4, t + 20 -> signs 15, 31
    d[t] = v;
  }
  return __builtin_bit_cast(f16x8, d);
}

// acc[ft] += sum over chunks kc in [kc0, kc1) and both planes of Hs[j][16ft + ..] . B[j][node] (products h 2^c);
// adjw[kc]: spread adjacency words; sc: agg_scale of the planes.  EXEC all ones (wave-uniform branches only).
template <int MODE>
__device__ __forceinline__ void agg2(f32x4 (&acc)[4], const uint16_t* P0, const uint16_t* P1,
                                     const uint32_t (&adjw)[DN_KC], const AggScale& sc, int kc0, int kc1, int lane) {
  const int q = lane >> 4;
  const int j_in = 4 * q + ((lane >> 2) & 3);
  const int pc = (lane & 3) ^ q;
#pragma unroll
  for (int kc = 0; kc < DN_KC; ++kc) {
    if (kc < kc0 || kc >= kc1) continue;  // wave-uniform
    const uint32_t plo = __builtin_amdgcn_readlane(sc.pat, 2 * kc);
    const uint32_t phi = __builtin_amdgcn_readlane(sc.pat, 2 * kc + 1);
    const f16x8 bf = adj_frag2<MODE>(adjw[kc], plo, phi);
    const int off = (32 * kc + j_in) * 16 + 4 * pc;
#pragma unroll
    for (int p = 1; p >= 0; --p) {  // the small plane first
#pragma unroll
      for (int ft = 0; ft < 4; ++ft) {
        const uint16_t* a = (p ? P1 : P0) + off + ft * (DN_KPMAX * 16);
        const v4s lo = tr_read(a), hi = tr_read(a + 16 * 16);
        const bf16x8 raw = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const f16x8 af = __builtin_bit_cast(f16x8, raw);
        acc[ft] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, acc[ft], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // bound the plane reads in flight (16-wave VGPR budget)
  }
}

// zero the plane rows [rows_pad, KP) (read as zeros by the last k-chunk; no tile writes them)
template <int NT>
__device__ __forceinline__ void zero_pad_rows2(uint16_t* P0, uint16_t* P1, int rows_pad) {
  const int KP = (rows_pad + 31) & ~31;
  for (int i = threadIdx.x; i < (KP - rows_pad) * 2 * 4 * 4; i += NT) {
    const int k = i & 3, ft = (i >> 2) & 3, p = (i >> 4) & 1, j = rows_pad + (i >> 5);
    *reinterpret_cast<uint2*>((p ? P1 : P0) + plane_off(ft, j, k)) = make_uint2(0u, 0u);
  }
}


// Per-lane staging of the block: the row's norm (deg clamped 0 -> 1, mpnn.py:34-38), its graph's max degree and
// the adjacency operand as spread words.  One graph per block with a prepared gs.adjbits (ER-200 ... ER-224): the
// lane loads its own degree and bitmask right after the block's graph id (two dependent global round trips, no
// LDS table and no barrier); otherwise the row-info table, edge bases and max degrees are staged in LDS and the
// bitmask is built from the CSR rows (dense_adjacency, with its barriers).
template <int NT>
__device__ __forceinline__ void d2_stage(const MpnnArgs& a, int blk, int rows_pad, int rows_valid, int r, bool valid,
                                         int s4, int2* RI, int64_t* GB, int* MD, uint32_t* ADJ, float& nf, int& md,
                                         uint32_t (&adjw)[DN_KC]) {
  const int N = a.N;
  const int rr = min(r, rows_pad - 1);
  uint32_t adjb[4];
  if (a.gpb == 1 && a.gs.adjbits != nullptr) {
    const int gid = a.gids[blk];  // uniform: scalar load
    const int dg = valid ? a.gs.deg[(size_t)gid * N + r] : 1;
    md = a.gs.max_deg[gid];
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (valid) v = *reinterpret_cast<const uint4*>(a.gs.adjbits + (((size_t)gid * N + r) * 4 + s4) * 4);
    adjb[0] = v.x; adjb[1] = v.y; adjb[2] = v.z; adjb[3] = v.w;
    nf = (float)max(dg, 1);
  } else {
    const int g_valid = min(a.gpb, a.B - blk * a.gpb);
    for (int r2 = threadIdx.x; r2 < rows_pad; r2 += NT) RI[r2] = pack_row_info(a, blk, r2, rows_valid);
    for (int gl = threadIdx.x; gl < g_valid; gl += NT) {
      const int gid = a.gids[blk * a.gpb + gl];
      GB[gl] = a.gs.edge_base[gid];
      MD[gl] = a.gs.max_deg[gid];
    }
    lds_barrier();
    nf = (float)row_info(RI, rr).norm;
    md = valid ? MD[r / N] : 1;
    dense_adjacency<NT>(a, ADJ, RI, GB, blk, rows_pad, rows_valid, r, rr, valid, s4, adjb);
  }
#pragma unroll
  for (int kc = 0; kc < DN_KC; ++kc) adjw[kc] = adj_spread((adjb[kc >> 1] >> (16 * (kc & 1))) & 0xFFFFu);
}

// LDS (ECO_D2_LDS): sPL the 2 fp16 planes (the readout's fp32 h3 rows at the end) | sW0, sW1, sW2 32-KB Linear
//      fragment buffers (sW1 / sW2 hold the V planes of the edge layer; sW1 is the readout scratch) | TE | RI | GB | MD
// NNET = 2 (one graph per block, no saved activations): the block runs TWO networks on the same graphs and node
// features -- the online and the target network on a train step's s' -- a0 then a1, sharing the staging (graph
// id -> degrees, adjacency words; node features), with a1's Wf DMA'd while a0's readout runs.
template <bool SAVE, int NNET>
__global__ __launch_bounds__(64 * DN_NW, 1) void mpnn_forward_dense2_kernel(MpnnArgs a0, MpnnArgs a1) {
  ECO_D2_LDS;
  const MpnnArgs& a = a0;  // the staging reads the graph fields, equal in a0 and a1
  ECO_TS(0);
  constexpr int NW = DN_NW;
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
  int2* RI = sRI;
  int64_t* GB = sGB;
  int* MD = sMD;
  uint32_t* ADJ = reinterpret_cast<uint32_t*>(sPL);  // [rows_pad][DN_ADJW] while a bitmask is built
  const size_t R0 = (size_t)blk * a.gpb * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const uint16_t* PH = reinterpret_cast<const uint16_t*>(P + PK_FH);
  const int s4 = lane >> 4;
  const int c16 = lane & 15;

  const bool has_tile = w < ntiles;
  const int r = w * 16 + c16;
  const bool valid = has_tile && r < rows_valid;
  // ---- staging: Wf fragments (LDS-DMA); node features, the 8-input Linears' weights and w_a; row norm, max
  //      degree and adjacency operand of the lane (d2_stage) ----
  glds_frags<NW>(WB0, PH + FH_WF, 16, w, lane);
  float xk0 = 0.f, xk1 = 0.f;
  if (valid) {
    xk0 = a.x[(R0 + r) * 8 + s4];
    xk1 = a.x[(R0 + r) * 8 + 4 + s4];
  }
  float wx8[8], w08[8];
  lin8_load(P + PK_WX, lane, wx8);
  lin8_load(P + PK_W0, lane, w08);
  float4 wa4[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) wa4[c] = f4(P + PK_WA + 16 * c + 4 * s4);
  float nf;
  int md_graph;
  uint32_t adjw[DN_KC];
  d2_stage<NT>(a, blk, rows_pad, rows_valid, r, valid, s4, RI, GB, MD, ADJ, nf, md_graph, adjw);
  ECO_TS(1);
  const float rnf = 1.f / nf;
  const int g_lo = min(w * 16, rows_pad - 1) / N, g_hi = min(w * 16 + 15, rows_pad - 1) / N;
  const int kc0 = (g_lo * N) >> 5;
  const int kc1 = (min((g_hi + 1) * N, rows_pad) + 31) >> 5;
#pragma unroll
  for (int net = 0; net < NNET; ++net) {
  const MpnnArgs& a = net == 0 ? a0 : a1;  // this network's weights and outputs
  const float* P = a.P;
  const uint16_t* PH = reinterpret_cast<const uint16_t*>(P + PK_FH);
  if (net > 0) {  // the 8-input Linears' weights and w_a of this network
    lin8_load(P + PK_WX, lane, wx8);
    lin8_load(P + PK_W0, lane, w08);
#pragma unroll
    for (int c = 0; c < 4; ++c) wa4[c] = f4(P + PK_WA + 16 * c + 4 * s4);
  }
  zero_pad_rows2<NT>(PL, PL1, rows_pad);
  zero_pad_rows2<NT>(WB1, WB2, rows_pad);  // V planes

  // ---- phase A: Z = Wx . x (f32 MFMA); U = relu(Z + w_a) and V = relu(Z - w_a) planes ----
  if (has_tile) {
    f32x4 z[4];
    lin8r(z, wx8, xk0, xk1);
    float4 u[4], v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 wa = wa4[c];
      u[c] = valid ? make_float4(relu(fmaf(1.f, wa.x, z[c][0])), relu(fmaf(1.f, wa.y, z[c][1])),
                                 relu(fmaf(1.f, wa.z, z[c][2])), relu(fmaf(1.f, wa.w, z[c][3])))
                   : zero4();
      v[c] = valid ? make_float4(relu(fmaf(-1.f, wa.x, z[c][0])), relu(fmaf(-1.f, wa.y, z[c][1])),
                                 relu(fmaf(-1.f, wa.z, z[c][2])), relu(fmaf(-1.f, wa.w, z[c][3])))
                   : zero4();
    }
    tile_planes(PL, PL1, TE, w, r, s4, u, lane);
    tile_planes(WB1, WB2, TE + 16, w, r, s4, v, lane);
  }
  glds_wait();  // Wf fragments
  lds_barrier();
  ECO_TS(2);

  // ---- phase B: edge embedding (mpnn.py:89-104): (A+ . relu(Z + w_a) + A- . relu(Z - w_a)) / norm; Wf ----
  float4 ereg[4];
  {
    const AggScale su = agg_scale(TE, ntiles, lane);
    const AggScale sv = agg_scale(TE + 16, ntiles, lane);
    f32x4 ea[4], ev[4];
#pragma unroll
    for (int ft = 0; ft < 4; ++ft) ea[ft] = ev[ft] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (has_tile) {
      agg2<1>(ea, PL, PL1, adjw, su, kc0, kc1, lane);
      agg2<2>(ev, WB1, WB2, adjw, sv, kc0, kc1, lane);
    }
    const int maxdeg_call = a.norm_scope == ECO_NORM_PER_CALL ? *a.call_maxdeg : 0;
    float4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float t4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        t4[i] = (__builtin_ldexpf(ea[c][i], -su.c) + __builtin_ldexpf(ev[c][i], -sv.c)) * rnf;
      acc[c] = make_float4(t4[0], t4[1], t4[2], t4[3]);
    }
    // feature 63 = norm / norm.max()  (mpnn.py:102)
    const int md = a.norm_scope == ECO_NORM_PER_CALL ? maxdeg_call : (valid ? md_graph : 1);
    if (s4 == 3) acc[3].w = nf / (float)md;
    if (!valid) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = zero4();
    } else if (SAVE) {
      float* eap = a.sv + (size_t)SV_EAGG * RT * 64 + (R0 + r) * 64 + 4 * s4;
#pragma unroll
      for (int c = 0; c < 4; ++c) st4(eap + 16 * c, acc[c]);
    }
    f32x4 d[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kx = node_exp<4>(acc);
    if (has_tile) mm_fh(d, acc, exp2i(kx), WB0, lane);
    unscale(d, kx + fh_kw(P, 0));
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      ereg[nt] = relu4(d[nt]);
      if (SAVE && valid) st4(a.sv + (size_t)SV_E * RT * 64 + (R0 + r) * 64 + 16 * nt + 4 * s4, ereg[nt]);
    }
    if (SAVE && valid) store_mask(a, RT, R0 + r, s4, SM_E, pos_mask(ereg));
  }
  lds_barrier();  // every wave is done with the U / V planes and with Wf
  ECO_TS(3);
  // layer weights: Wm0 -> WB1, Wu0 -> WB2, Wm1 -> WB0 (landed by layer 0's first barrier)
  glds_frags<NW>(WB1, PH + FH_LAYER, 32, w, lane);
  glds_frags<NW>(WB2, PH + FH_LAYER + 2 * FH_HALF, 32, w, lane);
  glds_frags<NW>(WB0, PH + FH_LAYER + FH_LAYER_STRIDE, 32, w, lane);

  // ---- phase C: h0 = relu(W0 . x) (mpnn.py:20-23, :55), in registers + planes ----
  float4 hreg[4];
  {
    f32x4 z[4];
    lin8r(z, w08, xk0, xk1);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      hreg[c] = valid ? relu4(z[c]) : zero4();
      if (SAVE && valid) st4(a.sv + (size_t)SV_H0 * RT * 64 + (R0 + r) * 64 + 16 * c + 4 * s4, hreg[c]);
    }
    if (has_tile) tile_planes(PL, PL1, TE, w, r, s4, hreg, lane);
  }
  if (SAVE && valid) store_mask(a, RT, R0 + r, s4, SM_H0, pos_mask(hreg));
  lds_barrier();
  ECO_TS(4);

  // ---- phase D: 3 x UpdateNodeEmbeddingLayer (mpnn.py:114-120) ----
  // per layer: [planes h_l + TE ready] (DMA of later weights) aggregation | wait + [B1] message, update (both
  //            Linears resident), h' planes | [B2]
  for (int layer = 0; layer < 3; ++layer) {
    const uint16_t* WM = layer == 0 ? WB1 : (layer == 1 ? WB0 : WB2);
    const uint16_t* WU = layer == 0 ? WB2 : (layer == 1 ? WB1 : WB0);
    if (layer == 1) {
      glds_frags<NW>(WB1, PH + FH_LAYER + FH_LAYER_STRIDE + 2 * FH_HALF, 32, w, lane);  // Wu1
      glds_frags<NW>(WB2, PH + FH_LAYER + 2 * FH_LAYER_STRIDE, 32, w, lane);            // Wm2
    } else if (layer == 2) {
      glds_frags<NW>(WB0, PH + FH_LAYER + 2 * FH_LAYER_STRIDE + 2 * FH_HALF, 32, w, lane);  // Wu2
    }
    const AggScale sh = agg_scale(TE, ntiles, lane);
#pragma unroll
    for (int kc = 0; kc < DN_KC; ++kc) asm volatile("" : "+v"(adjw[kc]));  // no hoisting of the 56 fragment masks
    f32x4 ag[4];
#pragma unroll
    for (int ft = 0; ft < 4; ++ft) ag[ft] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (has_tile) agg2<0>(ag, PL, PL1, adjw, sh, kc0, kc1, lane);
    float4 agg[4];
    {
      const float sc = __builtin_ldexpf(rnf, -sh.c);
#pragma unroll
      for (int c = 0; c < 4; ++c) agg[c] = make_float4(ag[c][0] * sc, ag[c][1] * sc, ag[c][2] * sc, ag[c][3] * sc);
    }
    if (layer == 0) ECO_TS(10);
    glds_wait();
    lds_barrier();  // B1: planes read by every wave; this layer's weights landed
    if (layer == 0) ECO_TS(11);
    if (SAVE && valid) {  // after the wait: stores count in vmcnt with the weight DMA
      float* sa = a.sv + (size_t)(SV_AGG0 + layer) * RT * 64 + (R0 + r) * 64 + 4 * s4;
#pragma unroll
      for (int c = 0; c < 4; ++c) st4(sa + 16 * c, agg[c]);
    }
    // message = relu(Wm . [agg, e])
    float4 mrel[4];
    {
      f32x4 d[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kx = node_exp2(agg, ereg);
      const float sf = exp2i(kx);
      if (has_tile) {
        mm_fh(d, ereg, sf, WM + FH_HALF, lane);
        mm_fh(d, agg, sf, WM, lane);
      }
      unscale(d, kx + fh_kw(P, 1 + 2 * layer));
#pragma unroll
      for (int c = 0; c < 4; ++c) mrel[c] = relu4(d[c]);
    }
    if (SAVE && valid) {
      float* sm = a.sv + (size_t)(SV_M0 + layer) * RT * 64 + (R0 + r) * 64 + 4 * s4;
#pragma unroll
      for (int c = 0; c < 4; ++c) st4(sm + 16 * c, mrel[c]);
      store_mask(a, RT, R0 + r, s4, SM_M0 + layer, pos_mask(mrel));
    }
    if (layer == 0) ECO_TS(12);
    // h' = relu(Wu . [h, m])
    {
      f32x4 hn[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) hn[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kx = node_exp2(hreg, mrel);
      const float sf = exp2i(kx);
      if (has_tile) {
        mm_fh(hn, hreg, sf, WU, lane);
        mm_fh(hn, mrel, sf, WU + FH_HALF, lane);
      }
      unscale(hn, kx + fh_kw(P, 2 + 2 * layer));
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        hreg[c] = valid ? relu4(hn[c]) : zero4();
        if (SAVE && valid) st4(a.sv + (size_t)(SV_H0 + layer + 1) * RT * 64 + (R0 + r) * 64 + 16 * c + 4 * s4, hreg[c]);
      }
    }
    if (SAVE && valid) store_mask(a, RT, R0 + r, s4, SM_H1 + layer, pos_mask(hreg));
    if (layer == 0) ECO_TS(13);
    if (layer < 2 && has_tile) tile_planes(PL, PL1, TE, w, r, s4, hreg, lane);
    if (layer == 0) ECO_TS(14);
    lds_barrier();  // B2: planes of h_{layer+1} complete; this layer's weight buffers free
    ECO_TS(5 + layer);
  }
  if (net + 1 < NNET)  // the next network's Wf into the free buffer, landing while this readout runs
    glds_frags<NW>(WB0, reinterpret_cast<const uint16_t*>(a1.P + PK_FH) + FH_WF, 16, w, lane);

  // ---- phase E: readout (mpnn.py:143-159) + act ----
  if (a.gpb == 1) {
    // one graph: per node q_local = Wr[64:] . h3 (the lane's 16 features, summed over the node's four lanes) and per
    // tile the column sums of h3 (DPP sums over the 16 nodes of a lane row) go to LDS from registers; one barrier;
    // wave 0 reduces the tile partials in tile order, forms p = Wp . mean, relu(p) . Wr[:64], the q values and acts
    float* COL = reinterpret_cast<float*>(sPL);  // [ntiles][64]
    float* QL = COL + 16 * 64;                    // [rows_pad] q_local
    float* MEANS = QL + DN_MAX_ROWS;              // [64]
    float* QB = MEANS + 64;                       // [rows_pad] q
    if (has_tile) {
      float ql = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 wr = f4(P + PK_WR + 64 + 16 * c + 4 * s4);
        ql = fmaf(hreg[c].x, wr.x, ql);
        ql = fmaf(hreg[c].y, wr.y, ql);
        ql = fmaf(hreg[c].z, wr.z, ql);
        ql = fmaf(hreg[c].w, wr.w, ql);
      }
      auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(ql), __float_as_uint(ql), false, false);
      ql = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
      auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(ql), __float_as_uint(ql), false, false);
      ql = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
      if (s4 == 0) QL[r] = ql;
      float cs[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        cs[4 * c] = row_sum16(hreg[c].x);
        cs[4 * c + 1] = row_sum16(hreg[c].y);
        cs[4 * c + 2] = row_sum16(hreg[c].z);
        cs[4 * c + 3] = row_sum16(hreg[c].w);
      }
      if (c16 == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          st4(COL + w * 64 + 16 * c + 4 * s4, make_float4(cs[4 * c], cs[4 * c + 1], cs[4 * c + 2], cs[4 * c + 3]));
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
    if (net + 1 < NNET) lds_barrier();  // wave 0's readout scratch (the plane array) before the next planes
    continue;
  }
  // several graphs per block: h3 rows staged as fp32 [rows][D2_HS_LD] in the plane array
  float* Hs = reinterpret_cast<float*>(sPL);
  if (has_tile) {
#pragma unroll
    for (int c = 0; c < 4; ++c) st4(Hs + r * D2_HS_LD + 16 * c + 4 * s4, hreg[c]);
  }
  lds_barrier();
  float* Scr = reinterpret_cast<float*>(sW1);
  const bool split = a.gpb < NW && readout_scratch_floats(rows_pad, a.gpb, NW, true) * 4 <= D2_WBUF_BYTES;
  if (!split && readout_scratch_floats(rows_pad, a.gpb, NW, false) * 4 > D2_WBUF_BYTES) return;  // launch checks
  readout_act<SAVE, NW>(a, Hs, D2_HS_LD, Scr, split, blk, g_valid, rows_valid, R0, RT);
  ECO_TS(8);
  if (net + 1 < NNET) lds_barrier();
  }  // networks
}

static int dense2_check(const MpnnArgs& a) {
  const int rows_pad = (a.gpb * a.N + 15) & ~15;
  if (rows_pad > DN_MAX_ROWS || a.gpb > D2_MAX_GPB) return fail(ECO_ERR_ARG, "dense MPNN block exceeds the LDS tables");
  if (readout_scratch_floats(rows_pad, a.gpb, DN_NW, false) * 4 > D2_WBUF_BYTES)
    return fail(ECO_ERR_ARG, "dense MPNN readout scratch exceeds its buffer");
  return ECO_OK;
}

static int mpnn_forward_dense2_launch(const MpnnArgs& a, bool save, hipStream_t st) {
  if (const int rc = dense2_check(a)) return rc;
  const int blocks = (a.B + a.gpb - 1) / a.gpb;
  if (save) mpnn_forward_dense2_kernel<true, 1><<<blocks, 64 * DN_NW, 0, st>>>(a, a);
  else mpnn_forward_dense2_kernel<false, 1><<<blocks, 64 * DN_NW, 0, st>>>(a, a);
  return check_launch("mpnn_forward_dense2");
}
// two networks on the same graphs and features in one launch (a and b differ only in P, q, act, actions)
static int mpnn_forward_dense2_pair_launch(const MpnnArgs& a, const MpnnArgs& b, hipStream_t st) {
  if (const int rc = dense2_check(a)) return rc;
  if (a.gpb != 1) return fail(ECO_ERR_ARG, "paired dense forward: one graph per block only");
  mpnn_forward_dense2_kernel<false, 2><<<a.B, 64 * DN_NW, 0, st>>>(a, b);
  return check_launch("mpnn_forward_dense2_pair");
}


// Two output halves (fragment sets WH0, WH1) of one 64-input transposed Linear sharing the split of x.
__device__ __forceinline__ void mm_fh2(f32x4 (&acc0)[4], f32x4 (&acc1)[4], const float4 (&x)[4], float sf,
                                       const uint16_t* WH0, const uint16_t* WH1, int lane) {
#pragma unroll
  for (int kc2 = 0; kc2 < 2; ++kc2) {
    f16x8 xh, xl;
    split_fh(x[2 * kc2], x[2 * kc2 + 1], sf, xh, xl);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const uint16_t* wl = (hh ? WH1 : WH0) + lane * 8;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        f32x4& acc = hh ? acc1[nt] : acc0[nt];
        const f16x8 w1 = *reinterpret_cast<const f16x8*>(wl + ((0 * 4 + nt) * 2 + kc2) * FH_FRAG);
        const f16x8 w2 = *reinterpret_cast<const f16x8*>(wl + ((1 * 4 + nt) * 2 + kc2) * FH_FRAG);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w2, xh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, xl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, xh, acc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);  // bound the fragments in flight (register pressure at 16 waves)
    }
  }
}

// ============================================================== backward ====
// Autograd of mpnn_forward_dense2_kernel (dqn.py:440-449) on the same fp16x2 operands: the A^T products are the
// forward's scaled-plane aggregation over the gathered gradient G (A symmetric), the Linears transposed fp16x2
// products (PK_FH transposed pieces, the matrix scales of the forward).  Writes the same pre-activation
// gradients and per-graph / per-block partials as mpnn_backward_dense_kernel (the weight-gradient reduction is
// shared).  A layer's two transposed Linears are resident (three rotating 32-KB buffers: Wu^T, Wm^T, and the next
// layer's Wu^T prefetched), three barriers per layer (Wm^T landed | G planes ready, the next layers' weights
// DMA'd | planes read).
// LDS (ECO_D2_LDS): sPL 2 planes (readout scratch first) | sW0, sW1, sW2 | TE | RI | GB
__global__ __launch_bounds__(64 * DN_NW, 1) void mpnn_backward_dense2_kernel(MpnnArgs a) {
  ECO_D2_LDS;
  ECO_TS(16);
  constexpr int NW = DN_NW;
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
  uint32_t* ADJ = reinterpret_cast<uint32_t*>(sPL);
  float* lds = reinterpret_cast<float*>(sPL);  // readout / dw_a scratch
  uint16_t* WB0 = sW0;
  uint16_t* WB1 = sW1;
  uint16_t* WB2 = sW2;
  int* TE = sTE;
  int2* RI = sRI;
  int64_t* GB = sGB;
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

  // ---- staging: Wu^T / Wm^T of layer 2 and Wu^T of layer 1 (LDS-DMA), row info, edge bases ----
  glds_frags<NW>(WB0, WUT(2), 32, w, lane);
  glds_frags<NW>(WB1, WMT(2), 32, w, lane);
  glds_frags<NW>(WB2, WUT(1), 32, w, lane);
  const bool has_tile = w < ntiles;
  const int rw = w * 16 + c16;
  const bool valid = has_tile && rw < rows_valid;
  const int rr = min(rw, rows_pad - 1);
  float nf;
  int md_unused;
  uint32_t adjw[DN_KC];
  d2_stage<NT>(a, blk, rows_pad, rows_valid, rw, valid, s4, RI, GB, sMD, ADJ, nf, md_unused, adjw);
  (void)md_unused;
  const float rnf = 1.f / nf;
  const int g_lo = min(w * 16, rows_pad - 1) / N, g_hi = min(w * 16 + 15, rows_pad - 1) / N;
  const int kc0 = (g_lo * N) >> 5;
  const int kc1 = (min((g_hi + 1) * N, rows_pad) + 31) >> 5;
  const uint16_t* Msk = reinterpret_cast<const uint16_t*>(sv + sv_mask_offset_floats(RT, a.B));
  const uint4 rmask = valid ? *reinterpret_cast<const uint4*>(Msk + ((R0 + rw) * 4 + s4) * SM_TENSORS)
                            : make_uint4(0u, 0u, 0u, 0u);
  ECO_TS(17);

  // ---- readout backward (mpnn.py:143-159), scratch in the plane region ----
  float* DQ = lds;                       // [rows_pad]
  float* DMEAN = DQ + rows_pad;          // [gpb][64]
  float* RED = DMEAN + a.gpb * 64;       // [gpb][NW][64] (split) or [NW][64]
  const bool split = a.gpb < NW && (size_t)(rows_pad + a.gpb * 64 + a.gpb * NW * 64) * 4 <= (size_t)D2_PL_BYTES;
  for (int i = threadIdx.x; i < rows_pad; i += NT) DQ[i] = i < rows_valid ? a.dq[R0 + i] : 0.f;
  lds_barrier();
  if (split) {  // dWr[64:] = sum_v dq_v h3_v, spread over all waves (dq of a train step: one node per graph)
    for (int gl = 0; gl < g_valid; ++gl) {
      const float* h3 = SV(SV_H3) + (R0 + (size_t)gl * N) * 64;
      float dwb = 0.f;
      for (int v = w; v < N; v += NW) {
        const float dv = DQ[gl * N + v];
        if (dv != 0.f) dwb = fmaf(dv, h3[(size_t)v * 64 + lane], dwb);
      }
      RED[(gl * NW + w) * 64 + lane] = dwb;
    }
    lds_barrier();
  }
  for (int gl = w; gl < g_valid; gl += NW) {
    const int e = blk * a.gpb + gl;
    float sacc = 0.f;
    for (int v = lane; v < N; v += 64) sacc += DQ[gl * N + v];
    const float S = wave_sum_f(sacc);
    const float p = PP[(size_t)e * 64 + lane];
    const float dp = P[PK_WR + lane] * S * (p > 0.f ? 1.f : 0.f);
    DP[(size_t)e * 64 + lane] = dp;
    DWRA[(size_t)e * 64 + lane] = relu(p) * S;
    if (lane == 0) DBR[e] = S;
    float dmean = 0.f;
#pragma unroll 16
    for (int k = 0; k < 64; ++k)  // dp_k by readlane (scalar broadcast) instead of a bpermute per k
      dmean = fmaf(P[PK_WP + k * 64 + lane], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dp), k)), dmean);
    DMEAN[gl * 64 + lane] = dmean / (float)N;
    float dwb = 0.f;
    if (split) {
#pragma unroll
      for (int k = 0; k < NW; ++k) dwb += RED[(gl * NW + k) * 64 + lane];  // fixed order
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
  // dh3 (node-operand layout): dq_i * wr[64+f] + dmean_f / N
  float4 dh[4];
  {
    const float dqi = valid ? DQ[rw] : 0.f;
    const int gl = rr / N;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int f = 16 * c + 4 * s4;
      const float4 dm = valid ? f4(DMEAN + gl * 64 + f) : zero4();
      dh[c] = make_float4(fmaf(dqi, P[PK_WR + 64 + f + 0], dm.x), fmaf(dqi, P[PK_WR + 64 + f + 1], dm.y),
                          fmaf(dqi, P[PK_WR + 64 + f + 2], dm.z), fmaf(dqi, P[PK_WR + 64 + f + 3], dm.w));
    }
  }
  glds_wait();     // Wu^T / Wm^T of layer 2 and Wu^T of layer 1 (staged at the start) are read from here on
  lds_barrier();  // readout scratch dead: zero the plane rows [rows_pad, KP) no tile writes
  zero_pad_rows2<NT>(PL, PL1, rows_pad);
  ECO_TS(18);

  // ---- update layers in reverse (mpnn.py:114-120) ----
  // duu, [dh_direct, dm] = Wu^T . duu (resident), dum | wait + [B0] Wm^T landed; [dagg, de] = Wm^T . dum, G planes |
  // [B1] dh = dh_direct + A.G | [B2] planes and this layer's buffers free: DMA of the next layers' weights
  float4 de[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) de[c] = zero4();
  for (int layer = 2; layer >= 0; --layer) {
    const uint16_t* WU = layer == 2 ? WB0 : (layer == 1 ? WB2 : WB1);
    const uint16_t* WM = layer == 2 ? WB1 : (layer == 1 ? WB0 : WB2);
    const size_t ro = (R0 + rr) * 64 + 4 * s4;
    // duu = dh' * [h' > 0]  (in place in dh)
    {
      const uint32_t hmask = mask16(rmask, SM_H0 + layer + 1);
#pragma unroll
      for (int c = 0; c < 4; ++c) dh[c] = masked(f32x4{dh[c].x, dh[c].y, dh[c].z, dh[c].w}, hmask, c);
    }
    // [dh_direct, dm] = Wu^T . duu;  dum = dm * [m > 0]
    f32x4 dhd[4];
    float4 dum[4];
    {
      f32x4 dmm[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dhd[nt] = dmm[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kx = node_exp<4>(dh);
      if (has_tile) mm_fh2(dhd, dmm, dh, exp2i(kx), WU, WU + FH_HALF, lane);
      const int ku = kx + fh_kw(P, 2 + 2 * layer);
      unscale(dhd, ku);
      unscale(dmm, ku);
      const uint32_t mmask = mask16(rmask, SM_M0 + layer);
#pragma unroll
      for (int c = 0; c < 4; ++c) dum[c] = masked(dmm[c], mmask, c);
    }
    if (layer == 1) ECO_TS(24);
    glds_wait();
    lds_barrier();  // B0: Wm^T landed
    if (layer == 1) ECO_TS(25);
    if (valid) {  // stored after the wait: stores count in vmcnt with the weight DMA
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        st4(GR(GR_DUU0 + layer) + ro + 16 * c, dh[c]);
        st4(GR(GR_DUM0 + layer) + ro + 16 * c, dum[c]);
      }
    }
    // [dagg, de] = Wm^T . dum;  G = dagg / norm -> planes
    {
      f32x4 dg[4], dd[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dg[nt] = dd[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kx = node_exp<4>(dum);
      if (has_tile) mm_fh2(dg, dd, dum, exp2i(kx), WM, WM + FH_HALF, lane);
      const int km = kx + fh_kw(P, 1 + 2 * layer);
      unscale(dg, km);
      unscale(dd, km);
      float4 g[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        de[c].x += dd[c][0]; de[c].y += dd[c][1]; de[c].z += dd[c][2]; de[c].w += dd[c][3];
        g[c] = valid ? make_float4(dg[c][0] * rnf, dg[c][1] * rnf, dg[c][2] * rnf, dg[c][3] * rnf) : zero4();
      }
      if (has_tile) tile_planes(PL, PL1, TE, w, rw, s4, g, lane);
    }
    if (layer == 1) ECO_TS(26);
    lds_barrier();  // B1: G planes complete; every wave is past both Linears: this layer's weight buffers free
    // the next layers' weights go out here rather than after B2: the A^T.G aggregation and B2 hide their DMA
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
      for (int kc = 0; kc < DN_KC; ++kc) asm volatile("" : "+v"(adjw[kc]));
      f32x4 ag[4];
#pragma unroll
      for (int ft = 0; ft < 4; ++ft) ag[ft] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (has_tile) agg2<0>(ag, PL, PL1, adjw, sg, kc0, kc1, lane);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float t4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) t4[i] = dhd[c][i] + __builtin_ldexpf(ag[c][i], -sg.c);
        dh[c] = valid ? make_float4(t4[0], t4[1], t4[2], t4[3]) : zero4();
      }
    }
    if (layer == 1) ECO_TS(28);
    lds_barrier();  // B2: planes read
    ECO_TS(21 - layer);
  }

  // ---- h0 = relu(W0.x): du0;  edge embedding (mpnn.py:89-104): due, dEagg = Wf^T . due -> G planes ----
  glds_wait();
  lds_barrier();  // Wf^T landed
  {
    const size_t ro = (R0 + rr) * 64 + 4 * s4;
    float4 due[4];
    const uint32_t h0m = mask16(rmask, SM_H0), em = mask16(rmask, SM_E);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (valid) st4(GR(GR_DU0) + ro + 16 * c, masked(f32x4{dh[c].x, dh[c].y, dh[c].z, dh[c].w}, h0m, c));
      due[c] = masked(f32x4{de[c].x, de[c].y, de[c].z, de[c].w}, em, c);
      if (valid) st4(GR(GR_DUE) + ro + 16 * c, due[c]);
    }
    f32x4 dg[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dg[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kx = node_exp<4>(due);
    if (has_tile) mm_fh(dg, due, exp2i(kx), WB0, lane);
    unscale(dg, kx + fh_kw(P, 0));
    float4 g[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
      g[c] = valid ? make_float4(dg[c][0] * rnf, dg[c][1] * rnf, dg[c][2] * rnf, dg[c][3] * rnf) : zero4();
    if (has_tile) tile_planes(PL, PL1, TE, w, rw, s4, g, lane);
  }
  lds_barrier();
  ECO_TS(22);
  // dz_j = [z_j + w_a > 0] (A+ . G)_j + [z_j - w_a > 0] (A- . G)_j;  dw_a = sum_j of the same with signs
  {
    float dwacc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) dwacc[i] = 0.f;
    float xk0 = 0.f, xk1 = 0.f;  // inputs of Z, loaded ahead of the aggregations
    if (valid) {
      xk0 = a.x[(R0 + rw) * 8 + s4];
      xk1 = a.x[(R0 + rw) * 8 + 4 + s4];
    }
    float wx8[8];
    lin8_load(P + PK_WX, lane, wx8);
    float4 wa4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) wa4[c] = f4(P + PK_WA + 16 * c + 4 * s4);
    const AggScale sg = agg_scale(TE, ntiles, lane);
    f32x4 gp[4], gm[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) gp[nt] = gm[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (has_tile) {
      agg2<1>(gp, PL, PL1, adjw, sg, kc0, kc1, lane);
      agg2<2>(gm, PL, PL1, adjw, sg, kc0, kc1, lane);
    }
    f32x4 zz[4];
    lin8r(zz, wx8, xk0, xk1);  // Z exactly as the forward computed it
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float dz4[4];
      const float wav[4] = {wa4[c].x, wa4[c].y, wa4[c].z, wa4[c].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float z = zz[c][i];
        const float wa = wav[i];
        const float tp = fmaf(1.f, wa, z) > 0.f ? __builtin_ldexpf(gp[c][i], -sg.c) : 0.f;
        const float tm = fmaf(-1.f, wa, z) > 0.f ? __builtin_ldexpf(gm[c][i], -sg.c) : 0.f;
        dz4[i] = valid ? tp + tm : 0.f;
        dwacc[4 * c + i] += valid ? tp - tm : 0.f;
      }
      if (valid) st4(GR(GR_DZ) + (R0 + rw) * 64 + 16 * c + 4 * s4, make_float4(dz4[0], dz4[1], dz4[2], dz4[3]));
    }
    // reduce dw_a over the 16 node lanes sharing s4, then over waves (fixed order)
#pragma unroll
    for (int i = 0; i < 16; ++i) dwacc[i] = row_sum16(dwacc[i]);
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

static int mpnn_backward_dense2_launch(const MpnnArgs& a, hipStream_t st) {
  if (const int rc = dense2_check(a)) return rc;
  const int blocks = (a.B + a.gpb - 1) / a.gpb;
  mpnn_backward_dense2_kernel<<<blocks, 64 * DN_NW, 0, st>>>(a);
  return check_launch("mpnn_backward_dense2");
}

}  // namespace eco
