// Dense-aggregation MPNN forward (src/networks/mpnn.py:40-159) for blocks of <= 224 rows with
// +-1 edge weights (ER/BA EdgeType.DISCRETE / UNIFORM graphs, N <= 224: ER-20 ... ER-200).
//
// The CSR gather of eco_mpnn.hip reads one random 256-B embedding row per edge from LDS; 16 lanes
// of a ds_read_b128 group hit 16 random rows, so at ER-200 density the gather is LDS-bank bound
// and serialises with the Linears.  Here every aggregation is a dense MFMA product instead:
//
//   agg[f][i] = sum_j H[j][f] * A[j][i]      (A symmetric, entries 0/+-1, exact in bf16)
//
// with H split EXACTLY into three bf16 planes H = H1 + H2 + H3 (24 significand bits = fp32), so
// every product is exact and the sums are fp32 MFMA accumulations: f32-exact products, f32 sums
// (the reference's own fp32 bmm differs only in summation order).  The planes are stored
// transposed, HT[p][f][j], so the A-operand fragment (8 consecutive j of one feature) is one
// 16-B read; the B-operand fragment (8 adjacency entries of one node) is built in registers from
// a per-row bitmask.  The 16x16 C layout of D[f][node] is exactly the node-operand layout of the
// f32 Linears (lane: node l&15, features 16c + 4(l>>4) + r), so nothing is transposed.
//
// Edge layer (mpnn.py:89-104): with A in {0, +-1}, sum_j [A_ij != 0] relu(We.[A_ij, x_j]) =
// A+ . relu(Z + w_a) + A- . relu(Z - w_a) (Z = Wx.x per node), two dense products over the same
// plane buffer.  Linears stay on v_mfma_f32_16x16x4_f32 (exact f32) as in eco_mpnn.hip.
//
// One 1024-thread workgroup (16 waves) per block of whole graphs; wave w owns 16-node tile w and
// keeps that tile's h and e in registers across the layers.
// Included once by eco_mpnn.hip (same translation unit: shares the phase-timing buffer).
#pragma once
#include "eco_mpnn.h"
#include "eco_mpnn_dev.h"

namespace eco {

typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int DN_NW = 16;
constexpr int DN_MAX_ROWS = 224;             // rows_pad limit (14 tiles, 7 k-chunks of 32)
constexpr int DN_KC = 7;
constexpr int DN_KPMAX = 224;                // plane rows (nodes j) per feature block
constexpr int DN_PLANE = 4 * DN_KPMAX * 16;  // bf16 elements per plane: [4 feature blocks][j][16 features]
constexpr int DN_ADJW = 2 * DN_KC;           // u32 words per adjacency row while it is built: {nz, neg} per chunk
constexpr int DN_PL_BYTES = 3 * DN_PLANE * 2;
constexpr int DN_WP_BYTES = 2 * BF_HALF * 2;  // a staged 128-input Linear (48 fragments)
constexpr int DN_WX_BYTES = BF_HALF * 2;      // prefetched first half of the update Linear

inline bool dense_eligible(const eco_graph_set* gs, int gpb) {
  const int rows_pad = (gpb * gs->n_spins + 15) & ~15;
  return gs->unit_weights && rows_pad <= DN_MAX_ROWS && gs->n_spins >= 4;
}

inline size_t dense_fwd_lds_bytes(int rows_pad, int gpb) {
  return (size_t)DN_PL_BYTES + DN_WP_BYTES + DN_WX_BYTES + (size_t)rows_pad * 8 + (size_t)gpb * 12 + 16;
}

// Plane image: PL[p][ft][j][16] bf16 (feature block ft = f >> 4, 32-B rows); the 8-B piece of features
// 4k .. 4k+3 of row j sits at piece position k ^ ((j >> 2) & 3), so 16 consecutive rows written by one
// 16-lane group hit 16 distinct bank pairs, and the transposed reads of dense_agg stay conflict-free.
__device__ __forceinline__ int plane_off(int ft, int j, int k) {
  return ft * (DN_KPMAX * 16) + j * 16 + 4 * (k ^ ((j >> 2) & 3));
}
// store features 16ft + 4k .. +3 of node j as three exact bf16 pieces
__device__ __forceinline__ void plane_store4(uint16_t* PL, int ft, int j, int k, float4 v) {
  uint16_t a[4], b[4], c[4];
  split3_bits(v.x, a[0], b[0], c[0]);
  split3_bits(v.y, a[1], b[1], c[1]);
  split3_bits(v.z, a[2], b[2], c[2]);
  split3_bits(v.w, a[3], b[3], c[3]);
  const int o = plane_off(ft, j, k);
  *reinterpret_cast<uint2*>(PL + o) = make_uint2(a[0] | (uint32_t)a[1] << 16, a[2] | (uint32_t)a[3] << 16);
  *reinterpret_cast<uint2*>(PL + DN_PLANE + o) = make_uint2(b[0] | (uint32_t)b[1] << 16, b[2] | (uint32_t)b[3] << 16);
  *reinterpret_cast<uint2*>(PL + 2 * DN_PLANE + o) =
      make_uint2(c[0] | (uint32_t)c[1] << 16, c[2] | (uint32_t)c[3] << 16);
}

// k-slot order of the aggregation MFMAs: lane group q, element jj <-> node 32kc + 16(jj >> 2) + 4q + (jj & 3)
// (the rows the two transposed reads of dense_agg deliver).  Per lane and chunk the 8 adjacency entries
// of those nodes for the lane's node are kept as 16 bits {nz byte, neg byte} (adj_bits16).
__device__ __forceinline__ uint32_t adj_bits16(uint2 w, int q) {
  const uint32_t nz = ((w.x >> (4 * q)) & 0xFu) | (((w.x >> (16 + 4 * q)) & 0xFu) << 4);
  const uint32_t ng = ((w.y >> (4 * q)) & 0xFu) | (((w.y >> (16 + 4 * q)) & 0xFu) << 4);
  return nz | (ng << 8);
}
// B fragment as bf16 0 / +1.0 / -1.0.  MODE 0: A (signed); 1: A+ = [A = +1]; 2: A- = [A = -1].
template <int MODE>
__device__ __forceinline__ bf16x8 adj_frag(uint32_t b16) {
  const uint32_t nz = b16 & 0xFFu, ng = (b16 >> 8) & 0xFFu;
  const uint32_t on = MODE == 0 ? nz : (MODE == 1 ? (nz & ~ng) : (nz & ng));
  bf16x8 f;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    uint32_t v = ((on >> jj) & 1u) ? 0x3F80u : 0u;
    if (MODE == 0) v |= ((ng >> jj) & 1u) << 15;
    f[jj] = (short)v;
  }
  return f;
}

typedef short v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4s tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// acc[ft] += sum over k-chunks [kc0, kc1) and the three planes of H[j][16ft + (l&15)] . A^(MODE)[j][node]:
// acc[ft] = D[16ft + 4q + r][node l&15], the node-operand layout.  A fragments: two ds_read_b64_tr_b16
// per (plane, ft) -- lane 4q'+p of each 16-lane group addresses row j = 32kc + 4q + q' (+16), piece p.
// Call with EXEC all ones (wave-uniform conditions only).
template <int MODE>
__device__ __forceinline__ void dense_agg(f32x4 (&acc)[4], const uint16_t* PL, const uint32_t (&adjb)[4], int kc0,
                                          int kc1, int lane) {
  const int q = lane >> 4;
  const int j_in = 4 * q + ((lane >> 2) & 3);
  const int pc = (lane & 3) ^ q;  // piece position: (j >> 2) & 3 == q for every row read here
#pragma unroll 1
  for (int kc = kc0; kc < kc1; ++kc) {  // not unrolled: bounds the fragment reads in flight (16-wave VGPR budget)
    const uint32_t wd = kc < 2 ? adjb[0] : kc < 4 ? adjb[1] : kc < 6 ? adjb[2] : adjb[3];
    const bf16x8 bf = adj_frag<MODE>((wd >> (16 * (kc & 1))) & 0xFFFFu);
    const uint16_t* base = PL + (32 * kc + j_in) * 16 + 4 * pc;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int ft = 0; ft < 4; ++ft) {
        const uint16_t* a = base + p * DN_PLANE + ft * (DN_KPMAX * 16);
        const v4s lo = tr_read(a), hi = tr_read(a + 16 * 16);
        const bf16x8 af = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[ft] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[ft], 0, 0, 0);
      }
    }
  }
}

__device__ __forceinline__ float4 as_f4(const f32x4& v) { return make_float4(v[0], v[1], v[2], v[3]); }

// 8 activations of the node-operand layout (float4 c = 2kc and 2kc+1 of a 64-feature block) as the
// three exact bf16 pieces of a 16x16x32 B fragment (element j <-> feature of bf16_kprime_feature).
__device__ __forceinline__ void split_frag(const float4& a, const float4& b, bf16x8& f1, bf16x8& f2, bf16x8& f3) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t h1[8], h2[8], h3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h1[j] = __float_as_uint(v[j]) & 0xFFFF0000u;
    const float r1 = v[j] - __uint_as_float(h1[j]);
    h2[j] = __float_as_uint(r1) & 0xFFFF0000u;
    h3[j] = __float_as_uint(r1 - __uint_as_float(h2[j]));
  }
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 w1, w2, w3;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    w1[t] = (h1[2 * t] >> 16) | (h1[2 * t + 1] & 0xFFFF0000u);
    w2[t] = (h2[2 * t] >> 16) | (h2[2 * t + 1] & 0xFFFF0000u);
    w3[t] = (h3[2 * t] >> 16) | (h3[2 * t + 1] & 0xFFFF0000u);
  }
  f1 = __builtin_bit_cast(bf16x8, w1);
  f2 = __builtin_bit_cast(bf16x8, w2);
  f3 = __builtin_bit_cast(bf16x8, w3);
}

// acc[nt] += W[16nt + ..][one 64-input half] . x  on 16x16x32 bf16 MFMAs with both operands split in
// three exact bf16 pieces; the six products above 2^-24 relative are kept (W3.X1, W2.X2, W1.X3, W2.X1,
// W1.X2, W1.X1, smallest first), so each product carries f32 accuracy.  WH: the half's staged
// fragments [p][nt][kc2] (BF_FRAG bf16 each, lane-linear) in LDS.
__device__ __forceinline__ void mm_bf3(f32x4 (&acc)[4], const float4 (&x)[4], const uint16_t* WH, int lane) {
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
    }
  }
}

// mm_bf3 with the fragment loads of one output tile at a time in flight (weights streamed from L2 by the
// CSR-gather kernels, where the register budget, not the load latency, is the constraint)
__device__ __forceinline__ void mm_bf3_lean(f32x4 (&acc)[4], const float4 (&x)[4], const uint16_t* WH, int lane) {
  // opaque to the optimiser: the same fragments are NOT hoisted/CSE'd across the calls of consecutive
  // tiles (which would keep 24 fragments = 96 VGPRs live per Linear half)
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)WH);  // wave-uniform pointer
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)WH >> 32));
  asm volatile("" : "+s"(lo), "+s"(hi));
  const uint16_t* wl = reinterpret_cast<const uint16_t*>(((uint64_t)hi << 32) | lo) + lane * 8;
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

// Two output halves (fragment sets WH0, WH1) of one 64-input transposed Linear, sharing the split of x.
__device__ __forceinline__ void mm_bf3x2(f32x4 (&acc0)[4], f32x4 (&acc1)[4], const float4 (&x)[4],
                                         const uint16_t* WH0, const uint16_t* WH1, int lane) {
#pragma unroll
  for (int kc2 = 0; kc2 < 2; ++kc2) {
    bf16x8 x1, x2, x3;
    split_frag(x[2 * kc2], x[2 * kc2 + 1], x1, x2, x3);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const uint16_t* wl = (hh ? WH1 : WH0) + lane * 8;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        f32x4& acc = hh ? acc1[nt] : acc0[nt];
        const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(wl + ((0 * 4 + nt) * 2 + kc2) * BF_FRAG);
        const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(wl + ((1 * 4 + nt) * 2 + kc2) * BF_FRAG);
        const bf16x8 w3 = *reinterpret_cast<const bf16x8*>(wl + ((2 * 4 + nt) * 2 + kc2) * BF_FRAG);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3, x1, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, x2, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x3, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, x1, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x2, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x1, acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // bound the fragments in flight (register pressure at 16 waves)
      }
    }
  }
}

// bit 4c + i: v[c] component i > 0
__device__ __forceinline__ uint32_t pos_mask(const float4 (&v)[4]) {
  uint32_t m = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    m |= (v[c].x > 0.f ? 1u : 0u) << (4 * c) | (v[c].y > 0.f ? 1u : 0u) << (4 * c + 1) |
         (v[c].z > 0.f ? 1u : 0u) << (4 * c + 2) | (v[c].w > 0.f ? 1u : 0u) << (4 * c + 3);
  return m;
}
__device__ __forceinline__ float4 masked(const f32x4& v, uint32_t m, int c) {
  return make_float4((m >> (4 * c)) & 1u ? v[0] : 0.f, (m >> (4 * c + 1)) & 1u ? v[1] : 0.f,
                     (m >> (4 * c + 2)) & 1u ? v[2] : 0.f, (m >> (4 * c + 3)) & 1u ? v[3] : 0.f);
}

// store the lane's 16-bit ReLU mask of tensor t for block row r (saved-activation mask region)
__device__ __forceinline__ void store_mask(const MpnnArgs& a, size_t RT, size_t grow, int q, int t, uint32_t m) {
  uint16_t* M = reinterpret_cast<uint16_t*>(a.sv + sv_mask_offset_floats(RT, a.B));
  M[(grow * 4 + q) * SM_TENSORS + t] = (uint16_t)m;
}

// 16-bit mask of tensor t from a lane's 8 packed masks
__device__ __forceinline__ uint32_t mask16(const uint4& m, int t) {
  const uint32_t wd = t < 2 ? m.x : t < 4 ? m.y : t < 6 ? m.z : m.w;
  return (wd >> (16 * (t & 1))) & 0xFFFFu;
}

// LDS-DMA copy of n_frag 1-KB weight fragments (global -> LDS, both contiguous, no registers):
// wave w issues fragments w, w + NW, ...  Retire with glds_wait() before the barrier that publishes them.
template <int NW>
__device__ __forceinline__ void glds_frags(uint16_t* dst, const uint16_t* src, int n_frag, int w, int lane) {
  for (int f = w; f < n_frag; f += NW)
    __builtin_amdgcn_global_load_lds((const void*)(src + f * BF_FRAG + lane * 8),
                                     (__attribute__((address_space(3))) void*)(dst + f * BF_FRAG), 16, 0, 0);
}
__device__ __forceinline__ void glds_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Bitmask adjacency operand of one graph per workgroup (eco_graphs_prepare, 104 < N <= 224):
// adjbits[g][v][q][k] = adj_bits16 of chunks 2k (low half) and 2k+1 (high half) for node v, lane quarter q.
__global__ __launch_bounds__(256) void adjbits_kernel(eco_graph_set gs, int first) {
  __shared__ uint32_t bm[DN_MAX_ROWS * DN_ADJW];
  const int g = first + blockIdx.x;
  const int N = gs.n_spins;
  for (int i = threadIdx.x; i < N * DN_ADJW; i += 256) bm[i] = 0u;
  __syncthreads();
  const int32_t* rp = gs.row_ptr + (size_t)g * (N + 1);
  const uint32_t* ed = gs.edges + gs.edge_base[g];
  for (int i = threadIdx.x; i < N * 4; i += 256) {
    const int v = i >> 2;
    for (int e = rp[v] + (i & 3); e < rp[v + 1]; e += 4) {
      const uint32_t ex = ed[e];
      const int j = edge_col(ex);
      atomicOr(&bm[v * DN_ADJW + 2 * (j >> 5)], 1u << (j & 31));
      if (edge_w(ex) < 0) atomicOr(&bm[v * DN_ADJW + 2 * (j >> 5) + 1], 1u << (j & 31));
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < N * 4; i += 256) {
    const int v = i >> 2, q = i & 3;
    const uint2* row = reinterpret_cast<const uint2*>(bm + v * DN_ADJW);
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = adj_bits16(row[2 * k], q) | (2 * k + 1 < DN_KC ? adj_bits16(row[2 * k + 1], q) << 16 : 0u);
    *reinterpret_cast<uint4*>(gs.adjbits + (((size_t)g * N + v) * 4 + q) * 4) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// the lane's adjacency bits of k-chunk kc (adj_bits16: nz byte, neg byte, element jj <-> bit jj) spread for the
// fragment builder: nz of elements 0,2,4,6 -> bits 0..3, neg of them -> 4..7, nz of 1,3,5,7 -> 16..19, neg -> 20..23
__device__ __forceinline__ uint32_t adj_spread(uint32_t b16) {
  uint32_t e = b16 & 0x5555u, o = (b16 >> 1) & 0x5555u;
  e = (e | (e >> 1)) & 0x3333u;
  e = (e | (e >> 2)) & 0x0F0Fu;
  o = (o | (o >> 1)) & 0x3333u;
  o = (o | (o >> 2)) & 0x0F0Fu;
  return ((e | (e >> 4)) & 0xFFu) | (((o | (o >> 4)) & 0xFFu) << 16);
}
// 224 < N <= 512 (eco_mpnn_dl.h): adjbits[g][v][q][DL_AW = 8] -- word m holds chunks 2m (bits 0..15) and 2m + 1
// (bits 16..31) in the PRE-SPREAD form of adj_spread (its bits 0..7 and 16..23 as one 16-bit value), so the
// kernels unpack a chunk with one byte permute.  LDS: [N][2 * 16] {nz, neg} words.
__device__ __forceinline__ uint32_t adj_prespread(uint32_t b16) {
  const uint32_t s = adj_spread(b16);
  return (s & 0xFFu) | ((s >> 8) & 0xFF00u);
}
__global__ __launch_bounds__(256) void adjbits_dl_kernel(eco_graph_set gs, int first) {
  extern __shared__ uint32_t bmd[];
  constexpr int KC = 16, W = 2 * KC;
  const int g = first + blockIdx.x;
  const int N = gs.n_spins;
  for (int i = threadIdx.x; i < N * W; i += 256) bmd[i] = 0u;
  __syncthreads();
  const int32_t* rp = gs.row_ptr + (size_t)g * (N + 1);
  const uint32_t* ed = gs.edges + gs.edge_base[g];
  for (int i = threadIdx.x; i < N * 4; i += 256) {
    const int v = i >> 2;
    for (int e = rp[v] + (i & 3); e < rp[v + 1]; e += 4) {
      const uint32_t ex = ed[e];
      const int j = edge_col(ex);
      atomicOr(&bmd[v * W + 2 * (j >> 5)], 1u << (j & 31));
      if (edge_w(ex) < 0) atomicOr(&bmd[v * W + 2 * (j >> 5) + 1], 1u << (j & 31));
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < N * 4; i += 256) {
    const int v = i >> 2, q = i & 3;
    const uint2* row = reinterpret_cast<const uint2*>(bmd + v * W);
    uint32_t o[8];
#pragma unroll
    for (int m = 0; m < 8; ++m)
      o[m] = adj_prespread(adj_bits16(row[2 * m], q)) | (adj_prespread(adj_bits16(row[2 * m + 1], q)) << 16);
    uint4* dst = reinterpret_cast<uint4*>(gs.adjbits + (((size_t)g * N + v) * 4 + q) * 8);
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
  }
}

int adjbits_build(const eco_graph_set* gs, int first, int count, hipStream_t st) {
  if (gs->n_spins <= DN_MAX_ROWS) {
    adjbits_kernel<<<count, 256, 0, st>>>(*gs, first);
  } else {
    const int lds = gs->n_spins * 32 * 4;
    (void)hipFuncSetAttribute((const void*)adjbits_dl_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    adjbits_dl_kernel<<<count, 256, lds, st>>>(*gs, first);
  }
  return check_launch("graphs_adjbits");
}

// Block bitmask adjacency, built in ADJ (LDS scratch of rows_pad * DN_ADJW words) from the CSR rows;
// unnecessary (returns false) when the block holds one graph with a prepared gs.adjbits.  RI and GB must
// be staged (and a barrier passed).  Uniform over the workgroup (contains barriers).
template <int NT>
__device__ __forceinline__ bool adj_build(const MpnnArgs& a, uint32_t* ADJ, const int2* RI, const int64_t* GB,
                                          int rows_pad, int rows_valid) {
  const int N = a.N;
  if (a.gpb == 1 && a.gs.adjbits != nullptr) return false;
  for (int i = threadIdx.x; i < rows_pad * DN_ADJW; i += NT) ADJ[i] = 0u;
  __syncthreads();
  // 4 threads per row, 8 edge loads in flight per thread
  for (int i = threadIdx.x; i < rows_pad * 4; i += NT) {
    const int row = i >> 2;
    if (row >= rows_valid) continue;
    const RowInfo ri = row_info(RI, row);
    const int base = (row / N) * N;
    const uint32_t* eg = a.gs.edges + GB[row / N];
    for (int e = ri.e0 + (i & 3); e < ri.e1; e += 32) {
      uint32_t ex[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) ex[k] = e + 4 * k < ri.e1 ? eg[e + 4 * k] : 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (e + 4 * k >= ri.e1) break;
        const int j = base + edge_col(ex[k]);
        const int wv = edge_w(ex[k]);
        if (wv != 1 && wv != -1) atomicCAS(a.err, 0, ECO_ERR_GRAPH);  // the caller's unit_weights was wrong
        uint32_t* word = ADJ + row * DN_ADJW + 2 * (j >> 5);
        atomicOr(word, 1u << (j & 31));
        if (wv < 0) atomicOr(word + 1, 1u << (j & 31));
      }
    }
  }
  __syncthreads();
  return true;
}

// The lane's adjacency operand (adj_bits16 of every k-chunk, packed in 4 words) for block row r.
__device__ __forceinline__ void adj_lane(const MpnnArgs& a, const uint32_t* ADJ, bool built, int blk, int r, int rr,
                                         bool valid, int s4, uint32_t (&adjb)[4]) {
  if (!built) {
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (valid) v = *reinterpret_cast<const uint4*>(a.gs.adjbits + (((size_t)a.gids[blk] * a.N + r) * 4 + s4) * 4);
    adjb[0] = v.x; adjb[1] = v.y; adjb[2] = v.z; adjb[3] = v.w;
    return;
  }
  const uint2* arow = reinterpret_cast<const uint2*>(ADJ + rr * DN_ADJW);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t lo = adj_bits16(arow[2 * k], s4);
    const uint32_t hi = 2 * k + 1 < DN_KC ? adj_bits16(arow[2 * k + 1], s4) : 0u;
    adjb[k] = lo | (hi << 16);
  }
}

// The lane's adjacency operand: prepared gs.adjbits, or built here (ADJ free again on return).
template <int NT>
__device__ __forceinline__ void dense_adjacency(const MpnnArgs& a, uint32_t* ADJ, const int2* RI, const int64_t* GB,
                                                int blk, int rows_pad, int rows_valid, int r, int rr, bool valid,
                                                int s4, uint32_t (&adjb)[4]) {
  const bool built = adj_build<NT>(a, ADJ, RI, GB, rows_pad, rows_valid);
  adj_lane(a, ADJ, built, blk, r, rr, valid, s4, adjb);
  if (built) __syncthreads();
}

// d[nt] = W[16 nt + .][0..7] . x of the lane's tile (the 8-input Linears: W0, Wx) on v_mfma_f32_16x16x4_f32,
// in the node-operand layout: A = W (lane: output feature 16 nt + (l & 15), input k = l >> 4 | 4 + (l >> 4)),
// B = x (input k, node l & 15) = this lane's xk0 / xk1.  f32 products; the forward and the backward's
// recomputation of Z share this expression (identical ReLU decisions).  EXEC all ones.
__device__ __forceinline__ void lin8(f32x4 (&d)[4], const float* W, float xk0, float xk1, int lane) {
  const float* wl = W + (lane & 15) * 8 + (lane >> 4);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    d[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wl[nt * 128], xk0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    d[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wl[nt * 128 + 4], xk1, d[nt], 0, 0, 0);
  }
}

#if ECO_AB_DENSE_V1
// The round-2 bf16x3 kernels, superseded by eco_mpnn_dense2.h (fp16x2).  Compiled only into A/B builds
// (-DECO_AB_DENSE_V1=1, tools/); the product library has no path to them.
// LDS: PL 3 bf16 planes [4][DN_KPMAX][16] (also the adjacency bits while they are built, and fp32
//      [rows][LDH] h3 rows for the readout) | WP a staged Linear (48 fragments; readout scratch) |
//      WX the prefetched h-half of the update Linear (24 fragments) | RI [rows_pad] int2 | GB [gpb] i64 | MD [gpb]
template <bool SAVE>
__global__ __launch_bounds__(64 * DN_NW, 1) void mpnn_forward_dense_kernel(MpnnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
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
  const int KP = (rows_pad + 31) & ~31;  // plane rows touched by any k-chunk
  uint16_t* PL = reinterpret_cast<uint16_t*>(lds);
  uint32_t* ADJ = reinterpret_cast<uint32_t*>(lds);  // [rows_pad][DN_ADJW] while the bitmask is built
  uint16_t* WP = PL + 3 * DN_PLANE;
  uint16_t* WX = WP + 2 * BF_HALF;
  int2* RI = reinterpret_cast<int2*>(WX + BF_HALF);
  int64_t* GB = reinterpret_cast<int64_t*>(RI + rows_pad);
  int* MD = reinterpret_cast<int*>(GB + a.gpb);
  const size_t R0 = (size_t)blk * a.gpb * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const uint16_t* PB = reinterpret_cast<const uint16_t*>(P + PK_BF);
  const int s4 = lane >> 4;
  const int c16 = lane & 15;

  // this lane's node (tile w, row w * 16 + c16) and its features k = s4, 4 + s4: the B operand of the
  // 8-input Linears (lin8), loaded before the staging so their latency overlaps it
  const bool has_tile = w < ntiles;
  const int r = w * 16 + c16;
  const bool valid = has_tile && r < rows_valid;
  float xk0 = 0.f, xk1 = 0.f;
  if (valid) {
    xk0 = a.x[(R0 + r) * 8 + s4];
    xk1 = a.x[(R0 + r) * 8 + 4 + s4];
  }
  // ---- staging: Wf fragments (LDS-DMA), row info, per-graph edge base / max degree, zeroed pad rows ----
  glds_frags<NW>(WP, PB + BF_WF, 24, w, lane);
  for (int r2 = threadIdx.x; r2 < rows_pad; r2 += NT) RI[r2] = pack_row_info(a, blk, r2, rows_valid);
  for (int gl = threadIdx.x; gl < g_valid; gl += NT) {
    const int gid = a.gids[blk * a.gpb + gl];
    GB[gl] = a.gs.edge_base[gid];
    MD[gl] = a.gs.max_deg[gid];
  }
  __syncthreads();
  ECO_TS(1);
  // this lane's k-chunk range; its adjacency bits in registers
  const int rr = min(r, rows_pad - 1);
  const RowInfo ri = row_info(RI, rr);
  const float nf = (float)ri.norm;
  const int g_lo = min(w * 16, rows_pad - 1) / N, g_hi = min(w * 16 + 15, rows_pad - 1) / N;
  const int kc0 = (g_lo * N) >> 5;
  const int kc1 = (min((g_hi + 1) * N, rows_pad) + 31) >> 5;
  uint32_t adjb[4];
  dense_adjacency<NT>(a, ADJ, RI, GB, blk, rows_pad, rows_valid, r, rr, valid, s4, adjb);
  // plane rows [rows_pad, KP) are read (as zeros) by the last k-chunk; no tile writes them
  for (int i = threadIdx.x; i < (KP - rows_pad) * 3 * 4 * 4; i += NT) {
    const int k = i & 3, ft = (i >> 2) & 3, p = (i >> 4) % 3, j = rows_pad + (i >> 4) / 3;
    *reinterpret_cast<uint2*>(PL + p * DN_PLANE + plane_off(ft, j, k)) = make_uint2(0u, 0u);
  }
  auto wa_of = [&](int c) { return f4(P + PK_WA + 16 * c + 4 * s4); };  // w_a of features 16c + 4 s4 .. +3

  // ---- phase A: Z = Wx . x (f32 MFMA per tile); U = relu(Z + w_a) planes ----
  if (has_tile) {
    f32x4 z[4];
    lin8(z, P + PK_WX, xk0, xk1, lane);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 wa = wa_of(c);
      plane_store4(PL, c, r, s4, valid ? make_float4(relu(fmaf(1.f, wa.x, z[c][0])), relu(fmaf(1.f, wa.y, z[c][1])),
                                                     relu(fmaf(1.f, wa.z, z[c][2])), relu(fmaf(1.f, wa.w, z[c][3])))
                                       : zero4());
    }
  }
  glds_wait();  // Wf fragments
  __syncthreads();
  ECO_TS(2);

  // ---- phase B: edge embedding (mpnn.py:89-104): A+ . relu(Z + w_a) + A- . relu(Z - w_a) ----
  f32x4 ea[4];
#pragma unroll
  for (int ft = 0; ft < 4; ++ft) ea[ft] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (has_tile) dense_agg<1>(ea, PL, adjb, kc0, kc1, lane);
  __syncthreads();
  if (has_tile) {
    f32x4 z[4];
    lin8(z, P + PK_WX, xk0, xk1, lane);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 wa = wa_of(c);
      plane_store4(PL, c, r, s4, valid ? make_float4(relu(fmaf(-1.f, wa.x, z[c][0])), relu(fmaf(-1.f, wa.y, z[c][1])),
                                                     relu(fmaf(-1.f, wa.z, z[c][2])), relu(fmaf(-1.f, wa.w, z[c][3])))
                                       : zero4());
    }
  }
  __syncthreads();
  float4 ereg[4];
  {
    if (has_tile) dense_agg<2>(ea, PL, adjb, kc0, kc1, lane);
    const int maxdeg_call = a.norm_scope == ECO_NORM_PER_CALL ? *a.call_maxdeg : 0;
    float4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = make_float4(ea[c][0] / nf, ea[c][1] / nf, ea[c][2] / nf, ea[c][3] / nf);
    // feature 63 = norm / norm.max()  (mpnn.py:102)
    const int md = a.norm_scope == ECO_NORM_PER_CALL ? maxdeg_call : (valid ? MD[r / N] : 1);
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
    if (has_tile) mm_bf3(d, acc, WP, lane);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      ereg[nt] = relu4(d[nt]);
      if (SAVE && valid) st4(a.sv + (size_t)SV_E * RT * 64 + (R0 + r) * 64 + 16 * nt + 4 * s4, ereg[nt]);
    }
    if (SAVE && valid) store_mask(a, RT, R0 + r, s4, SM_E, pos_mask(ereg));
  }
  __syncthreads();  // every wave is done with the V planes and with Wf
  ECO_TS(3);

  // ---- phase C: h0 = relu(W0 . x) (mpnn.py:20-23, :55), f32 MFMA per tile, kept in registers + planes ----
  float4 hreg[4];
  {
    f32x4 z[4];
    lin8(z, P + PK_W0, xk0, xk1, lane);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      hreg[c] = valid ? relu4(z[c]) : zero4();
      if (has_tile) plane_store4(PL, c, r, s4, hreg[c]);
      if (SAVE && valid) st4(a.sv + (size_t)SV_H0 * RT * 64 + (R0 + r) * 64 + 16 * c + 4 * s4, hreg[c]);
    }
  }
  if (SAVE && valid) store_mask(a, RT, R0 + r, s4, SM_H0, pos_mask(hreg));
  __syncthreads();
  ECO_TS(4);

  // ---- phase D: 3 x UpdateNodeEmbeddingLayer (mpnn.py:114-120) ----
  // per layer: [planes h_l ready] DMA Wm -> WP and Wu(h-half) -> WX | aggregation MFMAs | [B1] message |
  //            [B2] DMA Wu(m-half) -> WP | Wu(h-half).h | [B3] Wu(m-half).m, h' planes | [next layer]
  for (int layer = 0; layer < 3; ++layer) {
    const uint16_t* Wmb = PB + BF_LAYER + layer * BF_LAYER_STRIDE;
    const uint16_t* Wub = Wmb + 2 * BF_HALF;
    glds_frags<NW>(WP, Wmb, 48, w, lane);
    glds_frags<NW>(WX, Wub, 24, w, lane);
    f32x4 ag[4];
#pragma unroll
    for (int ft = 0; ft < 4; ++ft) ag[ft] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (has_tile) dense_agg<0>(ag, PL, adjb, kc0, kc1, lane);
    float4 agg[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) agg[c] = make_float4(ag[c][0] / nf, ag[c][1] / nf, ag[c][2] / nf, ag[c][3] / nf);
    if (SAVE && valid) {
      float* sa = a.sv + (size_t)(SV_AGG0 + layer) * RT * 64 + (R0 + r) * 64 + 4 * s4;
#pragma unroll
      for (int c = 0; c < 4; ++c) st4(sa + 16 * c, agg[c]);
    }
    glds_wait();
    __syncthreads();  // B1: Wm and Wu(h-half) landed
    // message = relu(Wm . [agg, e])
    f32x4 d[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (has_tile) {
      mm_bf3(d, ereg, WP + BF_HALF, lane);
      mm_bf3(d, agg, WP, lane);
    }
    float4 mrel[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) mrel[c] = relu4(d[c]);
    if (SAVE && valid) {
      float* sm = a.sv + (size_t)(SV_M0 + layer) * RT * 64 + (R0 + r) * 64 + 4 * s4;
#pragma unroll
      for (int c = 0; c < 4; ++c) st4(sm + 16 * c, mrel[c]);
      store_mask(a, RT, R0 + r, s4, SM_M0 + layer, pos_mask(mrel));
    }
    __syncthreads();  // B2: all waves done with Wm and with the planes of h_layer
    glds_frags<NW>(WP, Wub + BF_HALF, 24, w, lane);
    // h' = relu(Wu . [h, m]): the h half while the m half lands
    f32x4 hn[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) hn[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (has_tile) mm_bf3(hn, hreg, WX, lane);
    glds_wait();
    __syncthreads();  // B3
    if (has_tile) mm_bf3(hn, mrel, WP, lane);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      hreg[c] = valid ? relu4(hn[c]) : zero4();
      if (SAVE && valid) st4(a.sv + (size_t)(SV_H0 + layer + 1) * RT * 64 + (R0 + r) * 64 + 16 * c + 4 * s4, hreg[c]);
    }
    if (SAVE && valid) store_mask(a, RT, R0 + r, s4, SM_H1 + layer, pos_mask(hreg));
    if (layer < 2 && has_tile) {
#pragma unroll
      for (int c = 0; c < 4; ++c) plane_store4(PL, c, r, s4, hreg[c]);
    }
    __syncthreads();  // planes of h_{layer+1} complete; WP and WX free
    ECO_TS(5 + layer);
  }

  // ---- phase E: readout + act over h3 rows staged as fp32 [rows][LDH] in the plane buffer ----
  float* Hs = lds;
  if (has_tile) {
#pragma unroll
    for (int c = 0; c < 4; ++c) st4(Hs + r * LDH + 16 * c + 4 * s4, hreg[c]);
  }
  __syncthreads();
  float* Scr = reinterpret_cast<float*>(WP);
  const bool split = a.gpb < NW && readout_scratch_floats(rows_pad, a.gpb, NW, true) * 4 <= DN_WP_BYTES;
  readout_act<SAVE, NW>(a, Hs, LDH, Scr, split, blk, g_valid, rows_valid, R0, RT);
  ECO_TS(8);
}

// ============================================================== backward ====
// Autograd of mpnn_forward_dense_kernel (dqn.py:440-449) for the same blocks: every A^T product is the
// dense aggregation of the forward (A symmetric), every Linear a transposed bf16x3 product (BFT_*
// fragments).  Writes the pre-activation gradients the weight-gradient reduction reads (GR_DUU*, GR_DUM*,
// GR_DUE, GR_DU0, GR_DZ) and the per-graph / per-block partials of the CSR backward; dh and de stay in
// registers (no GR_DE / GR_DH round trips), and the forward's ReLU decisions come from 16-bit masks it
// saved (SM_*) instead of re-reading the f32 activation rows.  NW waves own MAXT 16-node tiles each
// (t = w + ti NW).
// LDS: PL planes of the gathered gradient G (readout scratch first) | WP 48 fragments | WX 24 fragments |
//      RI [rows_pad] int2 | GB [gpb] i64
template <int NW, int MAXT>
__global__ __launch_bounds__(64 * NW, 1) void mpnn_backward_dense_kernel(MpnnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  ECO_TS(16);
  constexpr int NT = 64 * NW;
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int blk = blockIdx.x;
  const int N = a.N;
  const int g_valid = min(a.gpb, a.B - blk * a.gpb);
  const int rows_valid = g_valid * N;
  const int rows_pad = (a.gpb * N + 15) & ~15;
  const int ntiles = rows_pad >> 4;
  uint16_t* PL = reinterpret_cast<uint16_t*>(lds);
  uint32_t* ADJ = reinterpret_cast<uint32_t*>(lds);
  uint16_t* WP = PL + 3 * DN_PLANE;
  uint16_t* WX = WP + 2 * BF_HALF;
  int2* RI = reinterpret_cast<int2*>(WX + BF_HALF);
  int64_t* GB = reinterpret_cast<int64_t*>(RI + rows_pad);
  const size_t R0 = (size_t)blk * a.gpb * N;
  const size_t RT = (size_t)a.B * N;
  const float* P = a.P;
  const uint16_t* PB = reinterpret_cast<const uint16_t*>(P + PK_BF);
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

  // ---- staging: layer-2 transposed weights (LDS-DMA), row info, edge bases ----
  glds_frags<NW>(WP, PB + BFT_LAYER + 2 * BF_LAYER_STRIDE + 2 * BF_HALF, 48, w, lane);  // Wu^T
  glds_frags<NW>(WX, PB + BFT_LAYER + 2 * BF_LAYER_STRIDE, 24, w, lane);                // Wm^T (dagg half)
  for (int r = threadIdx.x; r < rows_pad; r += NT) RI[r] = pack_row_info(a, blk, r, rows_valid);
  for (int gl = threadIdx.x; gl < g_valid; gl += NT) GB[gl] = a.gs.edge_base[a.gids[blk * a.gpb + gl]];
  __syncthreads();
  // per tile: node, validity, norm, k-chunk range, adjacency bits
  bool has_tile[MAXT], valid[MAXT];
  int rw[MAXT], rr[MAXT], kc0[MAXT], kc1[MAXT];
  float nf[MAXT];
  uint32_t adjb[MAXT][4];
  uint4 rmask[MAXT];  // the forward's ReLU masks of this lane's node (SM_* tensors, 16 bits each)
  {
    const bool built = adj_build<NT>(a, ADJ, RI, GB, rows_pad, rows_valid);
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const int t = w + ti * NW;
      has_tile[ti] = t < ntiles;
      rw[ti] = t * 16 + c16;
      valid[ti] = has_tile[ti] && rw[ti] < rows_valid;
      rr[ti] = min(rw[ti], rows_pad - 1);
      nf[ti] = (float)row_info(RI, rr[ti]).norm;
      const int g_lo = min(t * 16, rows_pad - 1) / N, g_hi = min(t * 16 + 15, rows_pad - 1) / N;
      kc0[ti] = (g_lo * N) >> 5;
      kc1[ti] = (min((g_hi + 1) * N, rows_pad) + 31) >> 5;
      adj_lane(a, ADJ, built, blk, rw[ti], rr[ti], valid[ti], s4, adjb[ti]);
      const uint16_t* M = reinterpret_cast<const uint16_t*>(sv + sv_mask_offset_floats(RT, a.B));
      rmask[ti] = valid[ti] ? *reinterpret_cast<const uint4*>(M + ((R0 + rw[ti]) * 4 + s4) * SM_TENSORS)
                            : make_uint4(0u, 0u, 0u, 0u);
    }
    if (built) __syncthreads();
  }
  ECO_TS(17);

  // ---- readout backward (mpnn.py:143-159), scratch in the plane region ----
  float* DQ = lds;                       // [rows_pad]
  float* DMEAN = DQ + rows_pad;          // [gpb][64]
  float* RED = DMEAN + a.gpb * 64;       // [gpb][NW][64] (split) or [NW][64]
  const bool split = a.gpb < NW && (size_t)(rows_pad + a.gpb * 64 + a.gpb * NW * 64) * 4 <= (size_t)DN_PL_BYTES;
  for (int i = threadIdx.x; i < rows_pad; i += NT) DQ[i] = i < rows_valid ? a.dq[R0 + i] : 0.f;
  __syncthreads();
  if (split) {  // dWr[64:] = sum_v dq_v h3_v, spread over all waves
    for (int gl = 0; gl < g_valid; ++gl) {
      const float* h3 = SV(SV_H3) + (R0 + (size_t)gl * N) * 64;
      float dwb = 0.f;
      for (int v = w; v < N; v += NW) {
        const float dv = DQ[gl * N + v];
        if (dv != 0.f) dwb = fmaf(dv, h3[(size_t)v * 64 + lane], dwb);
      }
      RED[(gl * NW + w) * 64 + lane] = dwb;
    }
    __syncthreads();
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
    for (int k = 0; k < 64; ++k) dmean = fmaf(P[PK_WP + k * 64 + lane], __shfl(dp, k, 64), dmean);
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
  __syncthreads();
  // dh3 (node-operand layout): dq_i * wr[64+f] + dmean_f / N
  float4 dh[MAXT][4];
#pragma unroll
  for (int ti = 0; ti < MAXT; ++ti) {
    const float dqi = valid[ti] ? DQ[rw[ti]] : 0.f;
    const int gl = rr[ti] / N;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int f = 16 * c + 4 * s4;
      const float4 dm = valid[ti] ? f4(DMEAN + gl * 64 + f) : zero4();
      dh[ti][c] = make_float4(fmaf(dqi, P[PK_WR + 64 + f + 0], dm.x), fmaf(dqi, P[PK_WR + 64 + f + 1], dm.y),
                              fmaf(dqi, P[PK_WR + 64 + f + 2], dm.z), fmaf(dqi, P[PK_WR + 64 + f + 3], dm.w));
    }
  }
  __syncthreads();  // readout scratch dead: zero the plane rows [rows_pad, KP) no tile writes (0 * garbage = NaN)
  {
    const int KP = (rows_pad + 31) & ~31;
    const int pad = KP - rows_pad;  // 0 or 16 rows
    for (int i = threadIdx.x; i < 3 * 4 * pad * 8; i += NT) {  // 8 dwords per 32-B row
      const int pf = i / (pad * 8), rem = i - pf * (pad * 8);
      reinterpret_cast<uint32_t*>(PL + (pf >> 2) * DN_PLANE + (pf & 3) * (DN_KPMAX * 16) + rows_pad * 16)[rem] = 0u;
    }
  }
  ECO_TS(18);

  // ---- update layers in reverse (mpnn.py:114-120) ----
  // [B0: Wu^T in WP, Wm^T(dagg half) in WX; planes free] dh_direct, dm | [B1] DMA Wm^T(de half) -> WP;
  // dagg -> G planes | [B2] de; DMA next Wm^T(dagg half) -> WX; dh = dh_direct + A.G | [B3] DMA next Wu^T -> WP
  float4 de[MAXT][4];
#pragma unroll
  for (int ti = 0; ti < MAXT; ++ti)
#pragma unroll
    for (int c = 0; c < 4; ++c) de[ti][c] = zero4();
  for (int layer = 2; layer >= 0; --layer) {
    const uint16_t* WmT = PB + BFT_LAYER + layer * BF_LAYER_STRIDE;
    // duu = dh' * [h' > 0]  (in place in dh), m > 0 masks
    uint32_t mmask[MAXT];
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      const size_t ro = (R0 + rr[ti]) * 64 + 4 * s4;
      mmask[ti] = mask16(rmask[ti], SM_M0 + layer);
      const uint32_t hmask = mask16(rmask[ti], SM_H0 + layer + 1);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        dh[ti][c] = masked(f32x4{dh[ti][c].x, dh[ti][c].y, dh[ti][c].z, dh[ti][c].w}, hmask, c);
        if (valid[ti]) st4(GR(GR_DUU0 + layer) + ro + 16 * c, dh[ti][c]);
      }
    }
    if (layer == 1) ECO_TS(24);
    glds_wait();
    __syncthreads();  // B0
    if (layer == 1) ECO_TS(25);
    // [dh_direct, dm] = Wu^T . duu;  dum = dm * [m > 0]
    f32x4 dhd[MAXT][4];
    float4 dum[MAXT][4];
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      f32x4 dmm[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        dhd[ti][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dmm[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (has_tile[ti]) mm_bf3x2(dhd[ti], dmm, dh[ti], WP, WP + BF_HALF, lane);
      const size_t ro = (R0 + rr[ti]) * 64 + 4 * s4;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        dum[ti][c] = masked(dmm[c], mmask[ti], c);
        if (valid[ti]) st4(GR(GR_DUM0 + layer) + ro + 16 * c, dum[ti][c]);
      }
    }
    if (layer == 1) ECO_TS(26);
    __syncthreads();  // B1: WP free
    if (layer == 1) ECO_TS(27);
    glds_frags<NW>(WP, WmT + BF_HALF, 24, w, lane);  // Wm^T, de half
    // dagg = Wm^T(agg half) . dum;  G = dagg / norm (d agg / d(A.h) = 1/norm) -> planes
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      if (!has_tile[ti]) continue;  // wave-uniform
      f32x4 dg[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dg[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      mm_bf3(dg, dum[ti], WX, lane);
      const float n_ = nf[ti];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        plane_store4(PL, c, rw[ti], s4,
                     valid[ti] ? make_float4(dg[c][0] / n_, dg[c][1] / n_, dg[c][2] / n_, dg[c][3] / n_) : zero4());
    }
    if (layer == 1) ECO_TS(28);
    glds_wait();
    __syncthreads();  // B2: G planes complete, Wm^T de half landed, WX free
    if (layer == 1) ECO_TS(29);
    if (layer > 0) glds_frags<NW>(WX, PB + BFT_LAYER + (layer - 1) * BF_LAYER_STRIDE, 24, w, lane);
    else glds_frags<NW>(WX, PB + BFT_WF, 24, w, lane);  // Wf^T for the edge layer
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      f32x4 dd[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dd[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (has_tile[ti]) mm_bf3(dd, dum[ti], WP, lane);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        de[ti][c].x += dd[c][0]; de[ti][c].y += dd[c][1]; de[ti][c].z += dd[c][2]; de[ti][c].w += dd[c][3];
      }
      // dh_layer = dh_direct + A^T . G  (A symmetric: the forward aggregation)
      if (has_tile[ti]) dense_agg<0>(dhd[ti], PL, adjb[ti], kc0[ti], kc1[ti], lane);
#pragma unroll
      for (int c = 0; c < 4; ++c) dh[ti][c] = valid[ti] ? as_f4(dhd[ti][c]) : zero4();
    }
    if (layer == 1) ECO_TS(30);
    __syncthreads();  // B3: WP and the planes free
    if (layer > 0) glds_frags<NW>(WP, PB + BFT_LAYER + (layer - 1) * BF_LAYER_STRIDE + 2 * BF_HALF, 48, w, lane);
    ECO_TS(21 - layer);
  }

  // ---- h0 = relu(W0.x): du0;  edge embedding (mpnn.py:89-104): due, dEagg = Wf^T . due -> G planes ----
  glds_wait();
  __syncthreads();  // Wf^T landed
#pragma unroll
  for (int ti = 0; ti < MAXT; ++ti) {
    const size_t ro = (R0 + rr[ti]) * 64 + 4 * s4;
    float4 due[4];
    const uint32_t h0m = mask16(rmask[ti], SM_H0), em = mask16(rmask[ti], SM_E);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (valid[ti])
        st4(GR(GR_DU0) + ro + 16 * c, masked(f32x4{dh[ti][c].x, dh[ti][c].y, dh[ti][c].z, dh[ti][c].w}, h0m, c));
      due[c] = masked(f32x4{de[ti][c].x, de[ti][c].y, de[ti][c].z, de[ti][c].w}, em, c);
      if (valid[ti]) st4(GR(GR_DUE) + ro + 16 * c, due[c]);
    }
    if (has_tile[ti]) {
      f32x4 dg[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dg[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      mm_bf3(dg, due, WX, lane);
      const float n_ = nf[ti];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        plane_store4(PL, c, rw[ti], s4,
                     valid[ti] ? make_float4(dg[c][0] / n_, dg[c][1] / n_, dg[c][2] / n_, dg[c][3] / n_) : zero4());
    }
  }
  __syncthreads();
  ECO_TS(22);
  // dz_j = [z_j + w_a > 0] (A+ . G)_j + [z_j - w_a > 0] (A- . G)_j;  dw_a = sum_j of the same with signs
  {
    float dwacc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) dwacc[i] = 0.f;
#pragma unroll
    for (int ti = 0; ti < MAXT; ++ti) {
      f32x4 gp[4], gm[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        gp[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        gm[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (has_tile[ti]) {
        dense_agg<1>(gp, PL, adjb[ti], kc0[ti], kc1[ti], lane);
        dense_agg<2>(gm, PL, adjb[ti], kc0[ti], kc1[ti], lane);
      }
      float xk0 = 0.f, xk1 = 0.f;
      if (valid[ti]) {
        xk0 = a.x[(R0 + rw[ti]) * 8 + s4];
        xk1 = a.x[(R0 + rw[ti]) * 8 + 4 + s4];
      }
      f32x4 zz[4];
      lin8(zz, P + PK_WX, xk0, xk1, lane);  // Z exactly as the forward computed it
#ifdef ECO_DBG_VALU_Z
      {
        float4 x0 = zero4(), x1 = zero4();
        if (valid[ti]) { x0 = f4(a.x + (R0 + rw[ti]) * 8); x1 = f4(a.x + (R0 + rw[ti]) * 8 + 4); }
        for (int c = 0; c < 4; ++c) for (int i = 0; i < 4; ++i) {
          const int f = 16 * c + 4 * s4 + i;
          const float4 w0 = f4(P + PK_WX + f * 8), w1 = f4(P + PK_WX + f * 8 + 4);
          zz[c][i] = w0.x * x0.x + w0.y * x0.y + w0.z * x0.z + w0.w * x0.w + w1.x * x1.x + w1.y * x1.y + w1.z * x1.z + w1.w * x1.w;
        }
      }
#endif
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float dz4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int f = 16 * c + 4 * s4 + i;
          const float z = zz[c][i];
          const float wa = P[PK_WA + f];
          const float tp = fmaf(1.f, wa, z) > 0.f ? gp[c][i] : 0.f;
          const float tm = fmaf(-1.f, wa, z) > 0.f ? gm[c][i] : 0.f;
          dz4[i] = valid[ti] ? tp + tm : 0.f;
          dwacc[4 * c + i] += valid[ti] ? tp - tm : 0.f;
        }
        if (valid[ti])
          st4(GR(GR_DZ) + (R0 + rw[ti]) * 64 + 16 * c + 4 * s4, make_float4(dz4[0], dz4[1], dz4[2], dz4[3]));
      }
    }
    // reduce dw_a over the 16 node lanes sharing s4, then over waves (fixed order)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float v = dwacc[i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      dwacc[i] = v;
    }
    __syncthreads();  // every wave is done reading the G planes: the region becomes the dwa scratch
    float* REDW = lds;  // [NW][64]
    if (c16 == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        st4(REDW + w * 64 + 16 * c + 4 * s4,
            make_float4(dwacc[4 * c], dwacc[4 * c + 1], dwacc[4 * c + 2], dwacc[4 * c + 3]));
    }
    __syncthreads();
    if (w == 0) {
      float sacc = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) sacc += REDW[k * 64 + lane];
      DWA[(size_t)blk * 64 + lane] = sacc;
    }
  }
  ECO_TS(23);
}

static int mpnn_backward_dense_launch(const MpnnArgs& a, hipStream_t st) {
  const int rows_pad = (a.gpb * a.N + 15) & ~15;
  const size_t lds = dense_fwd_lds_bytes(rows_pad, a.gpb);
  if (lds > 160 * 1024) return fail(ECO_ERR_ARG, "dense MPNN block exceeds the LDS budget");
  const int blocks = (a.B + a.gpb - 1) / a.gpb;
  // 16 waves x 1 tile (latency hiding; 2 VGPRs spill) is faster than 8 x 2 (no spills): 0.70 vs 0.82 ms
  // at M=2048 ER-200.
  if (true) {
    (void)hipFuncSetAttribute((const void*)mpnn_backward_dense_kernel<16, 1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    mpnn_backward_dense_kernel<16, 1><<<blocks, 1024, lds, st>>>(a);
  } else {
    (void)hipFuncSetAttribute((const void*)mpnn_backward_dense_kernel<8, 2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    mpnn_backward_dense_kernel<8, 2><<<blocks, 512, lds, st>>>(a);
  }
  return check_launch("mpnn_backward_dense");
}

static int mpnn_forward_dense_launch(const MpnnArgs& a, bool save, hipStream_t st) {
  const int rows_pad = (a.gpb * a.N + 15) & ~15;
  const size_t lds = dense_fwd_lds_bytes(rows_pad, a.gpb);
  if (lds > 160 * 1024) return fail(ECO_ERR_ARG, "dense MPNN block exceeds the LDS budget");
  const int blocks = (a.B + a.gpb - 1) / a.gpb;
  if (save) {
    (void)hipFuncSetAttribute((const void*)mpnn_forward_dense_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    mpnn_forward_dense_kernel<true><<<blocks, 64 * DN_NW, lds, st>>>(a);
  } else {
    (void)hipFuncSetAttribute((const void*)mpnn_forward_dense_kernel<false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    mpnn_forward_dense_kernel<false><<<blocks, 64 * DN_NW, lds, st>>>(a);
  }
  return check_launch("mpnn_forward_dense");
}

#endif  // ECO_AB_DENSE_V1

}  // namespace eco
