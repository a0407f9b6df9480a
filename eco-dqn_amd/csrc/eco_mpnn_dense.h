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


}  // namespace eco
