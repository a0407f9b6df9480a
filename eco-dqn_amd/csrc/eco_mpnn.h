// Shared layout constants of the MPNN kernels (forward/backward, eco_train.hip).
#pragma once
#include "eco_common.h"

namespace eco {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int MPNN_MAX_SPINS = 512;  // block of one graph must fit LDS (rows_pad * 272 B + scratch)
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
constexpr int PK_TOTAL = PK_LAYERT + 3 * 16384;

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
       SV_NODE_TENSORS };  // then MEAN [B][64], P [B][64]

// ---- backward gradient workspace: [tensor][R][64] then per graph / per block ----
enum { GR_DUU0 = 0, GR_DUU1, GR_DUU2, GR_DUM0, GR_DUM1, GR_DUM2, GR_DUE, GR_DU0, GR_DZ, GR_DE, GR_DH,
       GR_NODE_TENSORS };  // then DP [B][64], DWRA [B][64], DWRB [B][64], DBR [B(pad 64)], DWA [nblocks][64]

// whole graphs per workgroup block: up to 208 rows (13 tiles) share the LDS-resident embeddings
inline int graphs_per_block(int N) { return N >= 208 ? 1 : 208 / N; }

size_t mpnn_grad_ws_bytes(int32_t n_spins, int32_t batch);
int mpnn_backward_launch(const float* packed, int32_t n_obs_in, const eco_graph_set* gs, const int32_t* graph_ids,
                         int32_t batch, const float* obs_x, const void* saved, const float* dq, void* gradws,
                         hipStream_t st);

}  // namespace eco
