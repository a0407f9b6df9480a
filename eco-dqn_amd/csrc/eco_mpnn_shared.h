// MPNN forward for many episodes on ONE shared large graph (N > 512: GSet G22 best-cut search,
// configs[4]; src/networks/mpnn.py:40-159 batched as in experiments/utils.py:154-187).
//
// The per-episode large kernel (mpnn_forward_large_kernel) gathers a 256-B embedding row per edge per
// episode from that episode's private rows: 4 x nnz x 256 B per episode, ~41 GB per 1024-episode call,
// served by HBM.  Here every buffer is NODE-major, [node][episode][64] fp32, so the rows of one node for a
// slice of consecutive episodes are one contiguous block, and one neighbour's contribution to a wave tile
// is one such block per tile node.  The aggregation A.[H_1 ... H_B] then reads each neighbour block once per
// slice of 4 episodes, and the slices are dealt so that all workgroups of one group (one per XCD: block b
// works for group b % 8) sweep the nodes of the same slice together: the slice's H (N x 1 KB = 2 MB at
// G22) is what the gathers of that XCD re-read, from its 4-MB L2.  A wave tile is 4 nodes of similar
// degree (visited by decreasing degree) x the slice's 4 episodes = the 16 rows of the MFMA node operand;
// the tiles' CSR rows are pre-interleaved into one padded edge table per call, so the 4 nodes walk their
// rows in lockstep without per-lane bounds.  (16-episode slices of one node: 8 MB per slice, 28 % L2 hits,
// ~8 GB fetched per layer at 6 TB/s.)
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

#ifndef SH_EPS_X
#define SH_EPS_X 4
#endif
#ifndef SH_NW_X
#define SH_NW_X 16
#endif
#ifndef SH_GRP_X
#define SH_GRP_X 4
#endif
constexpr int SH_GRP = SH_GRP_X;       // edges per node gathered per group (row loads in flight per lane: 4 x SH_GRP)
constexpr int SH_EPS = SH_EPS_X;       // episodes per slice
constexpr int SH_NPT = 16 / SH_EPS;    // nodes per wave tile: 16 MFMA rows = SH_NPT nodes x SH_EPS episodes
constexpr int SH_NW = SH_NW_X;         // waves per workgroup (one workgroup per CU: <= 128 VGPRs at 16)
constexpr int SH_GROUPS = 8;           // episode-slice groups: one per XCD (block b -> group b % 8)
constexpr int SH_PART = SH_EPS * 64;   // floats of one slice's column-sum partial
constexpr int SH_CTR = 64;             // int32 stride of the work counters: one 256-B line each (counters
                                       // sharing a line serialise at one memory channel: ~88 dequeues/us)

struct SharedBufs {
  float* U;       // [S][N + 1][4][SH_EPS][16] (slice, node, feature chunk, episode, 16 features): SLICE-major, so
                  // the rows a slice's gathers touch are one contiguous 2 MB block (a node-major [node][4][Epad][16]
                  // put them 64 KB apart -- one L2 set -- and the L2 hit rate was 31 %); row N of every slice is the zero
                  // row the padded edge-table slots point at
  float* V;       // (graphs with negative weights only)
  float* HA;
  float* HB;
  float* EB;      // as U
  float* part;    // [S][ntiles][SH_EPS][64] column-sum partials of h3, one per wave tile
  float* ql;      // [Epad][N] Wr[64:] . h3
  int32_t* perm;  // [N] nodes by decreasing degree
  int32_t* tinfo; // [ntiles][SH_NPT] {node} , [ntiles][SH_NPT] {norm}, [ntiles] {max row length}
  uint32_t* et;   // [ntiles][MD][SH_NPT] interleaved edge words (edge q of tile node k at q * SH_NPT + k)
  int32_t* ctr;   // [4 launches][SH_GROUPS][SH_CTR] work counters, 256-B aligned (zeroed per forward)
  int Epad, S, nlb, ntiles, MD;
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

// MD: row slots per tile in the edge table = N + SH_GRP (the largest possible degree of a simple graph,
// rounded up to whole groups): the table is sized without a device -> host read of max_deg.
inline size_t shared_ws_bytes(int N, int B) {
  const size_t S = ((size_t)B + SH_EPS - 1) / SH_EPS, Epad = S * SH_EPS;
  const size_t nlb = shared_grid() / SH_GROUPS, nt = ((size_t)N + SH_NPT - 1) / SH_NPT;
  (void)nlb;
  return (5 * ((size_t)N + 1) * Epad * 64 + S * nt * SH_PART + Epad * (size_t)N + N +
          nt * (2 * SH_NPT + 1) + nt * ((size_t)N + SH_GRP) * SH_NPT + (4 * SH_GROUPS + 1) * SH_CTR) * sizeof(float);
}

inline SharedBufs shared_carve(float* base, int N, int B) {
  SharedBufs sb;
  sb.S = (B + SH_EPS - 1) / SH_EPS;
  sb.Epad = sb.S * SH_EPS;
  sb.nlb = shared_grid() / SH_GROUPS;
  sb.ntiles = (N + SH_NPT - 1) / SH_NPT;
  sb.MD = N + SH_GRP;
  const size_t T1 = ((size_t)N + 1) * sb.Epad * 64;
  sb.U = base;
  sb.V = sb.U + T1;
  sb.HA = sb.V + T1;
  sb.HB = sb.HA + T1;
  sb.EB = sb.HB + T1;
  sb.part = sb.EB + T1;
  sb.ql = sb.part + (size_t)sb.S * sb.ntiles * SH_PART;
  sb.perm = reinterpret_cast<int32_t*>(sb.ql + (size_t)sb.Epad * N);
  sb.tinfo = sb.perm + N;
  sb.et = reinterpret_cast<uint32_t*>(sb.tinfo + (size_t)sb.ntiles * (2 * SH_NPT + 1));
  sb.ctr = reinterpret_cast<int32_t*>(((uintptr_t)(sb.et + (size_t)sb.ntiles * sb.MD * SH_NPT) + 255) & ~(uintptr_t)255);
  return sb;
}

// this wave's XCD (0..7): speed only -- the work-counter protocol is correct for any placement
__device__ __forceinline__ int xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return (int)(x & 7u);
}

// streaming (non-temporal) row access: the layer's own e rows and its output rows are touched once, and
// should not push the gathered slice of H out of the L2
__device__ __forceinline__ float4 f4_nt(const float* p) {
  typedef float v4 __attribute__((ext_vector_type(4)));
  const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p));
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st4_nt(float* p, float4 x) {
  typedef float v4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(v4{x.x, x.y, x.z, x.w}, reinterpret_cast<v4*>(p));
}

// output rows of a layer launch (e, h'): read by the NEXT launch only.  SH_SC1_STORE: sc1 stores, which drop
// the line from this XCD's L2 instead of keeping it beside the slice being gathered.
__device__ __forceinline__ void st4_out(float* base, size_t off, float4 x) {  // base: wave-uniform
#ifdef SH_SC1_STORE
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(u4{__float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z),
                                            __float_as_uint(x.w)}, r, (int)(off * 4), 0, 16);
#else
  st4_nt(base + off, x);
#endif
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

// perm[rank] = node, nodes ranked by decreasing degree (index on ties): one thread per node, the degrees
// staged in LDS in chunks of 2048 (each thread compares against every node: from LDS, not N global loads);
// one wave per workgroup, so N / 64 CUs share the work
__global__ __launch_bounds__(64) void shared_perm_kernel(MpnnArgs a, SharedBufs sb) {
  __shared__ int DG[2048];
  const int N = a.N;
  const int i = blockIdx.x * 64 + threadIdx.x;
  const int32_t* rp = a.gs.row_ptr + (size_t)a.gids[0] * (N + 1);
  const int di = i < N ? rp[i + 1] - rp[i] : 0;
  int r = 0;
  for (int j0 = 0; j0 < N; j0 += 2048) {
    const int nj = min(2048, N - j0);
    __syncthreads();
    for (int j = threadIdx.x; j < nj; j += 64) DG[j] = rp[j0 + j + 1] - rp[j0 + j];
    __syncthreads();
    for (int j = 0; j < nj; ++j) {
      const int dj = DG[j];
      r += (dj > di) || (dj == di && j0 + j < i);
    }
  }
  if (i < N) sb.perm[r] = i;
}

// tile tables: thread (tile t, slot k) -> node, norm, its edge words interleaved with the tile's other
// nodes (padding slots: column N = the zero row, weight 0), and the tile's longest row
__global__ __launch_bounds__(256) void shared_tiles_kernel(MpnnArgs a, SharedBufs sb) {
  const int N = a.N;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int t = i / SH_NPT, k = i % SH_NPT;
  if (t >= sb.ntiles) return;
  const int gid = a.gids[0];
  const int32_t* rp = a.gs.row_ptr + (size_t)gid * (N + 1);
  const uint32_t* eg = a.gs.edges + a.gs.edge_base[gid];
  const int slot = t * SH_NPT + k;
  const bool valid = slot < N;
  const int n = valid ? sb.perm[slot] : 0;
  const int len = valid ? rp[n + 1] - rp[n] : 0;
  sb.tinfo[t * SH_NPT + k] = valid ? n : 0;
  sb.tinfo[(size_t)sb.ntiles * SH_NPT + t * SH_NPT + k] = valid ? max(a.gs.deg[(size_t)gid * N + n], 1) : 1;
  int ml = len;
  for (int o = 1; o < SH_NPT; o <<= 1) ml = max(ml, __shfl_xor(ml, o, 64));  // the tile's 4 slots are lanes 4t'..
  uint32_t* et = sb.et + (size_t)t * sb.MD * SH_NPT;
  const int ml4 = (ml + SH_GRP - 1) / SH_GRP * SH_GRP;
  for (int q = 0; q < ml4; ++q) et[q * SH_NPT + k] = q < len ? eg[rp[n] + q] : (uint32_t)N;  // pad: col N, w 0
  if (k == 0) sb.tinfo[(size_t)sb.ntiles * 2 * SH_NPT + t] = ml4;
}

// U (, V) and h0: one wave per tile of SH_NPT consecutive nodes x the SH_EPS episodes of one slice (the
// layer kernels' 16-row tile, in node order), the 8-input Linears on f32 MFMA (lin8, as the dense kernels),
// results stored straight from the MFMA layout: one float4 per lane and feature chunk, SH_NPT whole 256-B
// runs per store instruction (full cache lines, no LDS image, no write amplification).  Rows of padding
// episodes and the sentinel node N are zero; nodes past N are not stored.  V only for graphs with negative
// weights.
constexpr int SHP_WAVES = 4;
__global__ __launch_bounds__(64 * SHP_WAVES) void shared_prep_kernel(MpnnArgs a, SharedBufs sb) {
  const int lane = threadIdx.x & 63;
  const int c16 = lane & 15, s4 = lane >> 4;
  const int kn = c16 / SH_EPS, eps = c16 % SH_EPS;
  const int N = a.N;
  const int ntn = (N + 1 + SH_NPT - 1) / SH_NPT;  // node tiles incl. the sentinel row
  const int tile = blockIdx.x * SHP_WAVES + (threadIdx.x >> 6);
  if (tile >= ntn * sb.S) return;  // wave-uniform
  const int s = tile / ntn, n = (tile - s * ntn) * SH_NPT + kn;
  const int e = s * SH_EPS + eps;
  const bool valid = e < a.B && n < N;
  float xk0 = 0.f, xk1 = 0.f;
  if (valid) {
    xk0 = a.x[((size_t)e * N + n) * 8 + s4];
    xk1 = a.x[((size_t)e * N + n) * 8 + 4 + s4];
  }
  const bool neg = a.gs.meta[(size_t)a.gids[0] * 4 + 2] < 0.0;
  const size_t ld = (size_t)SH_EPS * 64, cs = (size_t)SH_EPS * 16;
  const size_t ro = (size_t)s * ((size_t)N + 1) * ld + (size_t)n * ld + (size_t)eps * 16 + 4 * s4;
  const bool st = n <= N;
  f32x4 z[4];
  lin8(z, a.P + PK_WX, xk0, xk1, lane);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float4 wa = f4(a.P + PK_WA + 16 * c + 4 * s4);
    if (st)
      st4_nt(sb.U + ro + c * cs, valid ? make_float4(relu(fmaf(1.f, wa.x, z[c][0])), relu(fmaf(1.f, wa.y, z[c][1])),
                                                     relu(fmaf(1.f, wa.z, z[c][2])), relu(fmaf(1.f, wa.w, z[c][3])))
                                       : zero4());
    if (neg && st)
      st4_nt(sb.V + ro + c * cs, valid ? make_float4(relu(fmaf(-1.f, wa.x, z[c][0])), relu(fmaf(-1.f, wa.y, z[c][1])),
                                                     relu(fmaf(-1.f, wa.z, z[c][2])), relu(fmaf(-1.f, wa.w, z[c][3])))
                                       : zero4());
  }
  lin8(z, a.P + PK_W0, xk0, xk1, lane);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (st) st4_nt(sb.HA + ro + c * cs, valid ? relu4(z[c]) : zero4());
    if (n == N) st4_nt(sb.HB + ro + c * cs, zero4());  // the other ping-pong buffer's sentinel row
  }
}

// PHASE 0: edge embedding -> EB; 1: update layer Hc -> Hn; 2: last update layer -> q_local + column sums.
// Wave tile: the SH_NPT nodes of tile t (similar degrees) x the slice's SH_EPS episodes; lane row c16 =
// node kn x episode eps.  The tile's edge table is walked in groups of 4 edges per node, the next group's
// edge words loaded while the current group's row blocks are in flight; padding slots read the zero row.
template <int PHASE>
__global__ __launch_bounds__(64 * SH_NW, 1) void shared_layer_kernel(MpnnArgs a, SharedBufs sb, int layer,
                                                                     const float* Hc, float* Hn) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  uint16_t* WL = reinterpret_cast<uint16_t*>(lds);  // Wf (24 fragments) or Wm, Wu (96 fragments)
  const int lane = threadIdx.x & 63;
  const int w = uniform_i(threadIdx.x >> 6);
  const int c16 = lane & 15, s4 = lane >> 4;
  const int kn = c16 / SH_EPS, eps = c16 % SH_EPS;
  const uint16_t* PB = reinterpret_cast<const uint16_t*>(a.P + PK_BF);
  if (PHASE == 0) glds_frags<SH_NW>(WL, PB + BF_WF, 24, w, lane);
  else glds_frags<SH_NW>(WL, PB + BF_LAYER + layer * BF_LAYER_STRIDE, 96, w, lane);
  const int N = a.N;
  const int gid = a.gids[0];
#ifdef SH_GROUP_BY_BLOCK
  const int home = blockIdx.x % SH_GROUPS;  // round-robin placement assumed
#else
  const int home = xcc_id();  // this CU's XCD: its waves share one counter (and one L2) whatever the placement
#endif
  const float* P = a.P;
  const float md = PHASE == 0 ? (float)(a.norm_scope == ECO_NORM_PER_CALL ? *a.call_maxdeg : a.gs.max_deg[gid]) : 1.f;
  // [slice][node][chunk c][episode][16]: chunk c of the 4 slice episodes of a node is one 256-B run, so each
  // gather instruction (fixed c, 16 rows = 4 nodes x 4 episodes) reads 4 whole 256-B runs
  const size_t ld = (size_t)SH_EPS * 64;  // floats per node block of a slice
  const size_t cs = (size_t)SH_EPS * 16;  // floats per feature chunk of a node block
  const size_t ss = ((size_t)N + 1) * ld;  // floats per slice
  const float* Ub = PHASE == 0 ? sb.U : Hc;
  glds_wait();
  __syncthreads();
  // Work items (slice-major, tile-minor) are taken from the group's counter one tile at a time, so the
  // waves of one XCD stay within about one slice of each other whatever their speeds (a static split
  // drifted apart over many slices and the L2 held none of them); the next item is claimed while the
  // current one is computed.
  // Every group's counter is drained by whoever gets there: the home group's first, then the others' (only
  // their tails are left when the placement is balanced), so each tile is computed exactly once whatever
  // the workgroup -> XCD placement.
  for (int gi = 0; gi < SH_GROUPS; ++gi) {
  const int grp = (home + gi) % SH_GROUPS;
  const int n_slices = (sb.S - grp + SH_GROUPS - 1) / SH_GROUPS;  // slices grp, grp + 8, ...
  int32_t* ctr = sb.ctr + ((PHASE == 0 ? 0 : layer + 1) * SH_GROUPS + grp) * SH_CTR;
  int item = 0;
  if (lane == 0) item = atomicAdd(ctr, 1);
  item = __shfl(item, 0, 64);
  while (true) {
    const int sl = item / sb.ntiles;
    if (sl >= n_slices) break;
    int next = 0;
    if (lane == 0) next = atomicAdd(ctr, 1);
    const int s = grp + SH_GROUPS * sl, t = item - sl * sb.ntiles;
    const int ep = s * SH_EPS + eps;
    const bool evalid = ep < a.B;
    const size_t co = (size_t)s * ss + (size_t)eps * 16 + 4 * s4;  // slice base + this lane's offset in chunk 0
    {
      const int slot = t * SH_NPT + kn;
      const bool nvalid = slot < N;
      const int n = sb.tinfo[t * SH_NPT + kn];
      const float nf = (float)sb.tinfo[sb.ntiles * SH_NPT + t * SH_NPT + kn];
      const int ml = uniform_i(sb.tinfo[sb.ntiles * 2 * SH_NPT + t]);
      const uint32_t* et = sb.et + (size_t)t * sb.MD * SH_NPT + kn;
      float4 acc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = zero4();
      uint32_t ex[SH_GRP], nx[SH_GRP];
#ifdef SH_PROBE_NOGATHER
      const int mlg = 0;
      acc[0] = f4(Ub + (size_t)n * ld + co);  // probe: no gather
#else
      const int mlg = ml;
#endif
      if (mlg > 0) {
#pragma unroll
        for (int k = 0; k < SH_GRP; ++k) ex[k] = et[k * SH_NPT];
      }
      for (int q = 0; q < mlg; q += SH_GRP) {
        if (q + SH_GRP < mlg) {
#pragma unroll
          for (int k = 0; k < SH_GRP; ++k) nx[k] = et[(q + SH_GRP + k) * SH_NPT];  // next group's edge words
        }
        float4 r[SH_GRP][4];
#pragma unroll
        for (int k = 0; k < SH_GRP; ++k) {
          const int wv = edge_w(ex[k]);
          const float* src = (PHASE == 0 && wv < 0 ? sb.V : Ub) + (size_t)edge_col(ex[k]) * ld + co;
#pragma unroll
          for (int c = 0; c < 4; ++c) r[k][c] = f4(src + c * cs);
        }
#pragma unroll
        for (int k = 0; k < SH_GRP; ++k) {
          const float fw = PHASE == 0 ? 1.f : (float)edge_w(ex[k]);  // padding: zero row
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            acc[c].x = fmaf(fw, r[k][c].x, acc[c].x); acc[c].y = fmaf(fw, r[k][c].y, acc[c].y);
            acc[c].z = fmaf(fw, r[k][c].z, acc[c].z); acc[c].w = fmaf(fw, r[k][c].w, acc[c].w);
          }
        }
#pragma unroll
        for (int k = 0; k < SH_GRP; ++k) ex[k] = nx[k];
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c].x = acc[c].x / nf; acc[c].y = acc[c].y / nf; acc[c].z = acc[c].z / nf; acc[c].w = acc[c].w / nf;
      }
      const bool rvalid = nvalid && evalid;
      const size_t ro = (size_t)n * ld + co;  // this lane's row (node n, episode ep)
      if (PHASE == 0) {
        if (s4 == 3) acc[3].w = nf / md;  // feature 63 = norm / norm.max() (mpnn.py:102)
        f32x4 d[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        mm_bf3_seq(d, acc, WL, lane);
        if (nvalid) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) st4_out(sb.EB, ro + nt * cs, rvalid ? relu4(d[nt]) : zero4());
        }
      } else {
#ifdef SH_PROBE_NOLIN
        if (PHASE == 1) {  // probe: gather only
          if (nvalid) {
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) st4_nt(Hn + ro + nt * cs, rvalid ? acc[nt] : zero4());
          }
          item = __shfl(next, 0, 64);
          continue;
        }
#endif
        f32x4 d[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) d[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        mm_bf3_seq(d, acc, WL, lane);               // message = relu(Wm . [agg, e])
        {
          float4 ev[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) ev[c] = f4_nt(sb.EB + ro + c * cs);
          mm_bf3_seq(d, ev, WL + BF_HALF, lane);
        }
        float4 mr[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) mr[c] = relu4(d[c]);
        f32x4 hn[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) hn[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        {
          float4 hc[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) hc[c] = f4(Hc + ro + c * cs);
          mm_bf3_seq(hn, hc, WL + 2 * BF_HALF, lane);  // h' = relu(Wu . [h, m])
        }
        mm_bf3_seq(hn, mr, WL + 3 * BF_HALF, lane);
        if (PHASE == 1) {
          if (nvalid) {
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) st4_out(Hn, ro + nt * cs, rvalid ? relu4(hn[nt]) : zero4());
          }
        } else {
          float qp = 0.f;
          float* pt = sb.part + ((size_t)s * sb.ntiles + t) * SH_PART + eps * 64 + 4 * s4;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const float4 h3 = rvalid ? relu4(hn[nt]) : zero4();
            const int f = 16 * nt + 4 * s4;
            qp = fmaf(h3.x, P[PK_WR + 64 + f], qp);
            qp = fmaf(h3.y, P[PK_WR + 65 + f], qp);
            qp = fmaf(h3.z, P[PK_WR + 66 + f], qp);
            qp = fmaf(h3.w, P[PK_WR + 67 + f], qp);
            // the tile's column sums over its SH_NPT nodes (fixed butterfly order), one partial per tile
            float4 csum = h3;
#pragma unroll
            for (int o = SH_EPS; o < 16; o <<= 1) {
              csum.x += __shfl_xor(csum.x, o, 64); csum.y += __shfl_xor(csum.y, o, 64);
              csum.z += __shfl_xor(csum.z, o, 64); csum.w += __shfl_xor(csum.w, o, 64);
            }
            if (kn == 0) st4_nt(pt + 16 * nt, csum);
          }
          qp += __shfl_xor(qp, 16, 64);
          qp += __shfl_xor(qp, 32, 64);
          if (s4 == 0 && rvalid) sb.ql[(size_t)ep * N + n] = qp;
        }
      }
    }
    item = __shfl(next, 0, 64);
  }
  }
}

// ReadoutLayer (mpnn.py:143-159) + epsilon-greedy act, one wave per episode: column sums from the
// partials (fixed order), p = Wp . mean, q = relu(p) . Wr[:64] + q_local + b, then the act of readout_act.
__global__ __launch_bounds__(256) void shared_readout_kernel(MpnnArgs a, SharedBufs sb) {
  __shared__ float red[4][64];
  const int e = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int N = a.N;
  const float* P = a.P;
  const int s = e / SH_EPS, er = e % SH_EPS;
  {  // the slice's per-tile column sums: wave w takes tiles w, w + 4, ...; the four combined in order
    const float* pp = sb.part + (size_t)s * sb.ntiles * SH_PART + er * 64 + lane;
    float c0 = 0.f;
#pragma unroll 8
    for (int k = w; k < sb.ntiles; k += 4) c0 += pp[(size_t)k * SH_PART];
    red[w][lane] = c0;
  }
  __syncthreads();
  if (w != 0) return;
  const float cs = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
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
  shared_perm_kernel<<<(a.N + 63) / 64, 64, 0, st>>>(a, sb);
  shared_tiles_kernel<<<(sb.ntiles * SH_NPT + 255) / 256, 256, 0, st>>>(a, sb);
  {
    const int ntn = (a.N + 1 + SH_NPT - 1) / SH_NPT;
    shared_prep_kernel<<<(ntn * sb.S + SHP_WAVES - 1) / SHP_WAVES, 64 * SHP_WAVES, 0, st>>>(a, sb);
  }
  if (hipMemsetAsync(sb.ctr, 0, 4 * SH_GROUPS * SH_CTR * sizeof(int32_t), st) != hipSuccess)
    return fail(ECO_ERR_HIP, "memset failed");
  const int grid = shared_grid();
  const size_t lds_edge = 24 * BF_FRAG * 2, lds_layer = 96 * BF_FRAG * 2,
               lds_last = lds_layer;
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
  shared_readout_kernel<<<a.B, 256, 0, st>>>(a, sb);
  return check_launch("mpnn_forward_shared");
}

}  // namespace eco
