// Shared layout constants of the MPNN kernels (forward/backward, eco_train.hip).
#pragma once
#include "eco_common.h"
#include <cstdlib>

namespace eco {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int MPNN_MAX_SPINS = 512;  // block of one graph must fit LDS (rows_pad * 272 B + scratch)
constexpr int MPNN_MAX_SPINS_LARGE = ECO_MAX_SPINS;  // global-memory embeddings (inference only) above 512
constexpr int LDH = 72;              // LDS row stride (floats) of 64-wide tiles: = 8 (mod 64) makes the MFMA
                                     // operand reads (16 rows x 4 quads per ds_read_b128 lane group) conflict-free
constexpr int LDW = 136;             // LDS row stride of staged [64][128] weights (same property)

// ---- packed parameter image (floats) ----
constexpr int PK_W0 = 0;                     // [64][8]  node_init_embedding (cols >= n_obs zero)
constexpr int PK_WX = 512;                   // [64][8]  edge_embedding_NN.weight[:, 1:] (row 63 zero)
constexpr int PK_WA = 1024;                  // [64]     edge_embedding_NN.weight[:, 0]  ([63] = 0)
constexpr int PK_WF = 1088;                  // [64][64] edge_feature_NN
constexpr int PK_LAYER = 5184;               // + l*16384: message [64][128], +8192: update [64][128]
constexpr int PK_WP = PK_LAYER + 3 * 16384;  // [64][64] layer_pooled
constexpr int PK_WR = PK_WP + 4096;          // [128] layers_readout.0.weight
constexpr int PK_BR = PK_WR + 128;           // [1]   layers_readout.0.bias
constexpr int PK_WFT = PK_BR + 64;           // [64][64]  Wf^T          (backward)
constexpr int PK_LAYERT = PK_WFT + 4096;     // + l*16384: Wm^T [128][64], +8192: Wu^T [128][64]
constexpr int PK_FP32_END = PK_LAYERT + 3 * 16384;
// bf16 pieces (exact 3-way split W = W1 + W2 + W3) of the dense-path Linears as ready-made 16x16x32
// A-operand fragments, a uint16 array starting at float PK_BF.  Per Linear: fragments
// [half][piece p][nt][kc2] of 64 lanes x 8 bf16 (1 KB; lane l holds W_p[16nt + (l&15)][feature of
// k' = 64 half + 32 kc2 + 8 (l>>4) + j], bf16_kprime_feature), so LDS-DMA copies them verbatim and every
// operand read is one conflict-free ds_read_b128.  half = 64-input block (Wf: 1, Wm/Wu: 2).
constexpr int PK_BF = (PK_FP32_END + 3) & ~3;
constexpr int BF_FRAG = 512;                         // bf16 per fragment
constexpr int BF_HALF = 3 * 4 * 2 * BF_FRAG;         // one 64-input half of a Linear (24 fragments)
constexpr int BF_WF = 0;                             // edge_feature_NN: 1 half
constexpr int BF_LAYER = BF_HALF;                    // + l * BF_LAYER_STRIDE: message (2 halves), then update
constexpr int BF_LAYER_STRIDE = 4 * BF_HALF;
constexpr int BF_FWD_END = BF_LAYER + 3 * BF_LAYER_STRIDE;
// transposed Linears of the dense backward (y = W^T x: 64 inputs = forward outputs, forward inputs as
// outputs in halves of 64): fragments [out half][p][nt][kc2], lane l: row 64 half + 16nt + (l&15) of W^T
constexpr int BFT_WF = BF_FWD_END;                   // Wf^T: 1 half
constexpr int BFT_LAYER = BFT_WF + BF_HALF;          // + l * BF_LAYER_STRIDE: Wm^T (2 halves), then Wu^T
constexpr int BF_TOTAL = BFT_LAYER + 3 * BF_LAYER_STRIDE;  // bf16 elements
// node-feature columns 8..15 (n_obs_in > 8, MAIN_OBSERVABLES): W0 [64][8] and Wx [64][8] (row 63 zero)
constexpr int PK_W0H = (PK_BF + BF_TOTAL / 2 + 3) & ~3;
constexpr int PK_WXH = PK_W0H + 512;
// fp16x2 pieces of the dense-path Linears (eco_mpnn_dense2.h): every Linear scaled by a power of two 2^kw
// (kw per matrix, from its max |w|, into [2^14, 2^15)) and split W s = W1 + W2 with W1 = fp16(W s) and
// W2 = fp16(W s - W1) (round to nearest): 22 significand bits, representation error <= 2^-22 |w| (or
// 2^-39 max|W| for entries 2^17 below the matrix maximum).  Same fragment geometry as the bf16 pieces
// ([half][piece p][nt][kc2], 64 lanes x 8 fp16, bf16_kprime_feature order), two pieces per half.
// PK_FHS: the exponents kw as int32 bits, in the order Wf, (Wm, Wu) x 3 layers.
constexpr int PK_FHS = PK_WXH + 512;
constexpr int FH_NMAT = 7;
constexpr int PK_FH = PK_FHS + 8;
constexpr int FH_FRAG = 512;                         // fp16 per fragment (1 KB)
constexpr int FH_HALF = 2 * 4 * 2 * FH_FRAG;         // one 64-input half (16 fragments, 16 KB)
constexpr int FH_WF = 0;
constexpr int FH_LAYER = FH_HALF;                    // + l * FH_LAYER_STRIDE: message (2 halves), update (2)
constexpr int FH_LAYER_STRIDE = 4 * FH_HALF;
constexpr int FH_FWD_END = FH_LAYER + 3 * FH_LAYER_STRIDE;
constexpr int FHT_WF = FH_FWD_END;                   // transposed (backward), as BFT_*
constexpr int FHT_LAYER = FHT_WF + FH_HALF;
constexpr int FH_TOTAL = FHT_LAYER + 3 * FH_LAYER_STRIDE;  // fp16 elements
constexpr int PK_TOTAL = PK_FH + FH_TOTAL / 2;

// k' -> input feature of the bf16 Linear operands: within each 64-feature block, k' = 32kc + 8q + j
// (kc = 0,1; q = lane >> 4; j = 0..7) holds feature 16(2kc + (j >> 2)) + 4q + (j & 3), i.e. the two
// float4 registers c = 2kc, 2kc+1 of the f32 node-operand layout, so no lane exchange is needed.
__host__ __device__ inline int bf16_kprime_feature(int kp) {
  const int b = kp >> 6, r = kp & 63;
  const int kc = r >> 5, q = (r >> 3) & 3, j = r & 7;
  return 64 * b + 16 * (2 * kc + (j >> 2)) + 4 * q + (j & 3);
}

// Exact split v = p1 + p2 + p3 into bf16 bit patterns (truncation: each remainder is exact in f32,
// the last one has <= 8 significant bits and is exact in bf16).
__host__ __device__ inline void split3_bits(float v, uint16_t& p1, uint16_t& p2, uint16_t& p3) {
  union { float f; uint32_t u; } a, b, c, d;
  a.f = v;
  b.u = a.u & 0xFFFF0000u;
  c.f = v - b.f;
  d.u = c.u & 0xFFFF0000u;
  const float r2 = c.f - d.f;
  union { float f; uint32_t u; } e;
  e.f = r2;
  p1 = (uint16_t)(b.u >> 16);
  p2 = (uint16_t)(d.u >> 16);
  p3 = (uint16_t)(e.u >> 16);
}

// ---- flat (state_dict order) parameter offsets, src/networks/mpnn.py ----
struct FlatOffsets {
  int W0, We, Wf, L, Wp, Wr, Br, total;
};
__host__ __device__ inline FlatOffsets flat_offsets(int nobs) {
  FlatOffsets o;
  o.W0 = 0;
  o.We = 64 * nobs;
  o.Wf = o.We + 63 * (1 + nobs);
  o.L = o.Wf + 4096;
  o.Wp = o.L + 6 * 8192;
  o.Wr = o.Wp + 4096;
  o.Br = o.Wr + 128;
  o.total = o.Br + 1;
  return o;
}

// ---- saved activations of the training forward: [tensor][R][64] then per graph ----
enum { SV_H0 = 0, SV_H1, SV_H2, SV_H3, SV_E, SV_EAGG, SV_M0, SV_M1, SV_M2, SV_AGG0, SV_AGG1, SV_AGG2,
       SV_NODE_TENSORS };  // then MEAN [B][64], P [B][64], then the ReLU masks (dense path)
// ReLU sign masks of the dense forward, read by the dense backward instead of the f32 rows:
// uint16 [R][4 lane quarters][8 tensors], bit 4c + i = feature 16c + 4q + i > 0
enum { SM_H0 = 0, SM_H1, SM_H2, SM_H3, SM_E, SM_M0, SM_M1, SM_M2, SM_TENSORS };
__host__ __device__ inline size_t sv_mask_offset_floats(size_t RT, size_t B) {
  return (size_t)SV_NODE_TENSORS * RT * 64 + 2 * B * 64;
}

// ---- backward gradient workspace: [tensor][R][64] then per graph / per block ----
enum { GR_DUU0 = 0, GR_DUU1, GR_DUU2, GR_DUM0, GR_DUM1, GR_DUM2, GR_DUE, GR_DU0, GR_DZ, GR_DE, GR_DH,
       GR_NODE_TENSORS };  // then DP [B][64], DWRA [B][64], DWRB [B][64], DBR [B(pad 64)], DWA [nblocks][64]

// whole graphs per workgroup block: up to 208 rows (13 tiles) share the LDS-resident embeddings
// Graphs per workgroup block for B graphs of N vertices (every MPNN launch and workspace size of a call
// uses the same value).  Up to 208 rows per block; within that, the count whose launch is estimated
// fastest: rounds of blocks over the CUs x (16-row tiles per SIMD + 1 for the block's staging and
// readout) -- e.g. ER-20 x4096: 8 graphs (10 tiles, 512 blocks) beats 10 (13 tiles, 410 blocks) by 16 %.
// Forward workspace header (the first 256 B): int 0 = the call's max degree (norm scope per call); bytes
// [WS_KEY_OFFSET, +16) = the key of the shared-graph tables cached after it (eco_mpnn_shared.h).  Every other
// path that writes the workspace past the header zeroes the key (ws_invalidate_key), so cached tables it
// overwrote are rebuilt.
constexpr int WS_KEY_OFFSET = 64;
__device__ __forceinline__ void ws_invalidate_key(const int* call_maxdeg) {
  if (blockIdx.x == 0 && threadIdx.x == 0)
    *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(const_cast<int*>(call_maxdeg)) + WS_KEY_OFFSET) = 0ull;
}

inline int device_cu_count() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                               hipSuccess || n < 1)
      n = 256;
    return n;
  }();
  return cus;
}
inline int graphs_per_block(int N, int B) {
  const int cus = device_cu_count();
  const int gmax = N >= 208 ? 1 : 208 / N;
  int best = gmax;
  double best_cost = 1e300;
  for (int g = gmax; g >= 1 && 2 * g >= gmax; --g) {
    const int tiles = (g * N + 15) / 16;
    const long long blocks = ((long long)B + g - 1) / g;
    const double cost = (double)((blocks + cus - 1) / cus) * ((tiles + 3) / 4 + 1);
    if (cost < best_cost) { best_cost = cost; best = g; }
  }
  return best;
}

// dense-path bitmask adjacency of graphs [first, first + count) into gs->adjbits (eco_mpnn_dense.h)
int adjbits_build(const eco_graph_set* gs, int first, int count, hipStream_t st);
inline bool adjbits_applies(int n_spins) { return n_spins > 104 && n_spins <= 512; }
// u32 words of gs->adjbits per node: 4 lane quarters x (4 words up to 224 vertices, 8 above)
inline int adjbits_words_per_node(int n_spins) { return n_spins <= 224 ? 16 : 32; }

// kernel-path policy (eco_set_kernel_paths, include/eco_hip.h): ECO_PATH_* bits, process-wide
int kernel_paths();

size_t mpnn_grad_ws_bytes(int32_t n_spins, int32_t batch);
int mpnn_backward_launch(const float* packed, int32_t n_obs_in, const eco_graph_set* gs, const int32_t* graph_ids,
                         int32_t batch, const float* obs_x, const void* saved, const float* dq, void* gradws,
                         hipStream_t st);

}  // namespace eco
