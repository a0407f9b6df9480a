// DQN training hot path on gfx950 (src/agents/dqn/dqn.py:403-451, dqn/utils.py:28-83):
// device replay ring, double-DQN TD target + MSE gradient, MPNN weight gradients
// (split-K reductions over every node of the minibatch on bf16x3-split v_mfma_f32_32x32x16_bf16,
// per-wave partial slabs reduced in a fixed order -> bitwise reproducible), Adam.
#include <cmath>

#include "eco_mpnn.h"
#include "eco_env_dev.h"

namespace eco {

// ------------------------------------------------------------ weight grads ----
// dW[o][i] = sum_r dY[r][o] * X[r][i]  with X = [X1 (K1 cols) | X2 (K2 cols)]
struct WJob {
  const float* dY;   // [R][64]
  const float* X1;
  const float* X2;
  int ld1, K1, ld2, K2;
  int R;
  int nO;            // rows of dW (64, or 63 for the edge-embedding Wx)
  int out_off;       // flat offset of dW[0][0]
  int out_ld;        // row stride in the flat buffer
  int out_col0;      // first column in the flat buffer
};
constexpr int MAX_JOBS = 10;
#ifndef WGRAD_NT
#define WGRAD_NT 0  // A/B: nontemporal (streaming) loads of the dY / X rows
#endif
constexpr int WGRAD_WG_X = 3;  // workgroups per CU over all jobs (46 KB LDS each: 3 resident per CU)
constexpr int WG_PER_JOB = 128;
constexpr int SLABS_PER_JOB = WG_PER_JOB;  // one [64][128] partial per workgroup
constexpr int SLAB = 64 * 128;
constexpr int WROWS = 32;                  // rows per LDS tile

struct WJobs {
  WJob j[MAX_JOBS];
  int n;
  int nwgj[MAX_JOBS];     // wgrad_bf3_kernel / reduce: workgroups (= slabs) of job j, <= WG_PER_JOB
  int first[MAX_JOBS + 1];  // wgrad_bf3_kernel: first flat block of job j (1-D grid of first[n] blocks)
};


// Same reduction on 32x32x16 bf16 MFMAs: dY and X are split EXACTLY into three bf16 pieces while a
// 32-row tile is staged (split3_bits), and the six products above 2^-24 relative are accumulated in
// f32 (as mm_bf3 does for the forward Linears), so the sums keep f32 accuracy at ~2.7x the f32-MFMA
// rate.  Staging transposes through registers: thread t loads column (t & 63) of 8 consecutive rows
// (each wave-level load is one contiguous 256-B row segment), splits, and writes the three 8-row
// pieces as 16-B LDS stores into [p][column][row] planes, which are exactly the MFMA fragments
// (lane l: column l & 31, rows 8 (l >> 5) .. +7 of a 16-row k-step).
constexpr int WB_LD = 40;  // bf16 per plane column (32 rows + 8 pad: 80-B stride, conflict-light 16-B reads)
typedef short bf16x8w __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4w __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split8_store(uint16_t* base, int plane_stride, const float (&v)[8]) {
  u32x4w p1, p2, p3;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    uint16_t a0, b0, c0, a1, b1, c1;
    split3_bits(v[2 * t], a0, b0, c0);
    split3_bits(v[2 * t + 1], a1, b1, c1);
    p1[t] = a0 | (uint32_t)a1 << 16;
    p2[t] = b0 | (uint32_t)b1 << 16;
    p3[t] = c0 | (uint32_t)c1 << 16;
  }
  *reinterpret_cast<u32x4w*>(base) = p1;
  *reinterpret_cast<u32x4w*>(base + plane_stride) = p2;
  *reinterpret_cast<u32x4w*>(base + 2 * plane_stride) = p3;
}

// WIDE: X of up to 128 columns (two 64-column groups per thread); narrow jobs (K <= 64: Wf, W0, Wx, Wp) stage one
// group of 8 rows x 1 column per thread and issue half the X loads.
template <bool WIDE>
__device__ __forceinline__ void wgrad_bf3_job(const WJobs& jobs, float* slabs, int jb, uint16_t* sY, uint16_t* sX) {
  constexpr int PY = 64 * WB_LD, PX = 128 * WB_LD;  // plane strides (bf16)
  constexpr int XU = WIDE ? 2 : 1;                  // X row groups per thread
  const int wg = (int)blockIdx.x - jobs.first[jb], nwg = jobs.nwgj[jb];
  const WJob& J = jobs.j[jb];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int jj = lane & 31, h = lane >> 5;
  const int K = J.K1 + J.K2;
  const int ntile = 2 * ((K + 31) / 32);
  const int chunk = ((J.R + nwg - 1) / nwg + WROWS - 1) / WROWS * WROWS;
  const int r0 = wg * chunk;
  const int r1 = min(J.R, r0 + chunk);
  // staging roles: dY column yc of rows 8 yg .. +7; X columns xc (+ 0 / 1 x 128 units) of rows 8 xg .. +7
  const int yc = threadIdx.x & 63, yg = threadIdx.x >> 6;
  // X: WIDE: column t & 127 of row groups (t >> 7) + 2u, u < 2; narrow: column t & 63 of row group t >> 6
  const int xc = WIDE ? threadIdx.x & 127 : threadIdx.x & 63, xg0 = WIDE ? threadIdx.x >> 7 : threadIdx.x >> 6;
  constexpr int XG = WIDE ? 2 : 4;  // row-group step between a thread's X units
  typedef const __attribute__((address_space(1))) float gfloat;
  // loads are unconditional (rows clamped to r1 - 1, dead columns read column 0) and masked after:
  // predicated loads compiled to one branch + vmcnt(0) wait per row, serialising the whole tile
  const bool xlive = xc < K;
  gfloat* ysrc = (gfloat*)(J.dY + yc);
  const float* xsrc = !xlive ? J.X1 : (xc < J.K1 ? J.X1 + xc : J.X2 + (xc - J.K1));
  int xld = xlive && xc >= J.K1 ? J.ld2 : J.ld1;
  uint32_t xmask = xlive ? 0xFFFFFFFFu : 0u;
  // keep the per-lane source and mask opaque (otherwise the select is sunk into every load as a branch)
  asm volatile("" : "+v"(xsrc), "+v"(xld), "+v"(xmask));
  gfloat* xg = (gfloat*)xsrc;
  const int rlast = r1 - 1;
  f32x16 acc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[q][k] = 0.f;
  // two register buffers: tiles i+1 and i+2 are in flight while tile i is split and multiplied
  // (one tile in flight held the reduction at ~4 TB/s: too few bytes outstanding per CU)
  struct Regs {
    float y[8], x[XU][8];
  };
  // raw loads only; the row / column masks are applied when the tile is stored (masking at load
  // time makes the compiler wait for every load before the multiply it should overlap)
  auto load_tile = [&](Regs& R, int rb) {
#if WGRAD_NT
#pragma unroll
    for (int k = 0; k < 8; ++k) R.y[k] = __builtin_nontemporal_load(&ysrc[(size_t)min(rb + 8 * yg + k, rlast) * 64]);
#pragma unroll
    for (int u = 0; u < XU; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k)
        R.x[u][k] = __builtin_nontemporal_load(&xg[(size_t)min(rb + 8 * (xg0 + XG * u) + k, rlast) * (size_t)xld]);
#else
#pragma unroll
    for (int k = 0; k < 8; ++k) R.y[k] = ysrc[(size_t)min(rb + 8 * yg + k, rlast) * 64];
#pragma unroll
    for (int u = 0; u < XU; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k)
        R.x[u][k] = xg[(size_t)min(rb + 8 * (xg0 + XG * u) + k, rlast) * (size_t)xld];
#endif
  };
  auto store_tile = [&](Regs& R, int rb) {
    asm volatile("" : "+s"(rb));  // keeps the masking (and this tile's wait) at the store
#pragma unroll
    for (int k = 0; k < 8; ++k) R.y[k] = rb + 8 * yg + k < r1 ? R.y[k] : 0.f;
    split8_store(sY + yc * WB_LD + 8 * yg, PY, R.y);
#pragma unroll
    for (int u = 0; u < XU; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        R.x[u][k] = rb + 8 * (xg0 + XG * u) + k < r1 ? __uint_as_float(__float_as_uint(R.x[u][k]) & xmask) : 0.f;
      split8_store(sX + xc * WB_LD + 8 * (xg0 + XG * u), PX, R.x[u]);
    }
  };
  // this wave's output tiles: t = w + 4q -> o-tile w & 1, i-tiles (w >> 1) and (w >> 1) + 2
  const int ot = w & 1;
  const bool live0 = w < ntile, live1 = w + 4 < ntile;
  const uint16_t* ya = sY + (32 * ot + jj) * WB_LD + 8 * h;
  const uint16_t* xb0 = sX + (32 * (w >> 1) + jj) * WB_LD + 8 * h;
  const uint16_t* xb1 = xb0 + 64 * WB_LD;
  auto compute = [&]() {
  if (live0) {
#pragma unroll
    for (int s = 0; s < WROWS / 16; ++s) {
      const bf16x8w a1 = *reinterpret_cast<const bf16x8w*>(ya + 16 * s);
      const bf16x8w a2 = *reinterpret_cast<const bf16x8w*>(ya + PY + 16 * s);
      const bf16x8w a3 = *reinterpret_cast<const bf16x8w*>(ya + 2 * PY + 16 * s);
      const bf16x8w b1 = *reinterpret_cast<const bf16x8w*>(xb0 + 16 * s);
      const bf16x8w b2 = *reinterpret_cast<const bf16x8w*>(xb0 + PX + 16 * s);
      const bf16x8w b3 = *reinterpret_cast<const bf16x8w*>(xb0 + 2 * PX + 16 * s);
      if (live1) {
        const bf16x8w c1 = *reinterpret_cast<const bf16x8w*>(xb1 + 16 * s);
        const bf16x8w c2 = *reinterpret_cast<const bf16x8w*>(xb1 + PX + 16 * s);
        const bf16x8w c3 = *reinterpret_cast<const bf16x8w*>(xb1 + 2 * PX + 16 * s);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, b1, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, c1, acc[1], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b2, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, c2, acc[1], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b3, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, c3, acc[1], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b1, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, c1, acc[1], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b2, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, c2, acc[1], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, c1, acc[1], 0, 0, 0);
      } else {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, b1, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b2, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b3, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b1, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b2, acc[0], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[0], 0, 0, 0);
      }
    }
  }
  };
  // loads are issued unconditionally (rows past r1 clamp to r1 - 1 and are masked at the store): a
  // conditional load makes the compiler drain every tile in flight at the join (vmcnt(0))
  if (r0 < r1) {
    Regs RA, RB;
    load_tile(RA, r0);
    load_tile(RB, r0 + WROWS);
    for (int rb = r0; rb < r1; rb += 2 * WROWS) {
      store_tile(RA, rb);
      __syncthreads();
      load_tile(RA, rb + 2 * WROWS);
      compute();
      __syncthreads();
      if (rb + WROWS >= r1) break;
      store_tile(RB, rb + WROWS);
      __syncthreads();
      load_tile(RB, rb + 3 * WROWS);
      compute();
      __syncthreads();
    }
  }
  float* slab = slabs + ((size_t)jb * SLABS_PER_JOB + wg) * SLAB;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int t = w + 4 * q;
    if (t < ntile) {
      const int it = t >> 1;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int o = 32 * ot + (k & 3) + 8 * (k >> 2) + 4 * h;  // 32x32 C/D layout
        slab[o * 128 + 32 * it + jj] = acc[q][k];
      }
    }
  }
}

__global__ __launch_bounds__(256) void wgrad_bf3_kernel(WJobs jobs, float* slabs) {
  __shared__ __attribute__((aligned(16))) uint16_t sY[3 * 64 * WB_LD];
  __shared__ __attribute__((aligned(16))) uint16_t sX[3 * 128 * WB_LD];
  int jb = 0;
  while (jb + 1 < jobs.n && (int)blockIdx.x >= jobs.first[jb + 1]) ++jb;
  if (jobs.j[jb].K1 + jobs.j[jb].K2 > 64) wgrad_bf3_job<true>(jobs, slabs, jb, sY, sX);
  else wgrad_bf3_job<false>(jobs, slabs, jb, sY, sX);
}


// fixed-order sum of the slabs of every job into the flat gradient
__global__ void wgrad_reduce_kernel(WJobs jobs, const float* slabs, float* grad) {
  const WJob& J = jobs.j[blockIdx.y];
  const int K = J.K1 + J.K2;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int o = idx / 128, i = idx % 128;
  if (o >= J.nO || i >= K) return;
  const float* s = slabs + (size_t)blockIdx.y * SLABS_PER_JOB * SLAB + o * 128 + i;
  float acc = 0.f;
  const int nk = jobs.nwgj[blockIdx.y];
  int k = 0;
  for (; k + 8 <= nk; k += 8) {  // eight slab loads in flight, summed in slab order (same result as one by one)
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = s[(size_t)(k + u) * SLAB];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; k < nk; ++k) acc += s[(size_t)k * SLAB];
  grad[J.out_off + o * J.out_ld + J.out_col0 + i] = acc;
}

// the readout / edge-weight column sums of one backward in ONE launch: one workgroup per output column, blocks
// dealt to the four jobs in order; a fixed-order sum per column (256 strided partials, then a tree)
struct ColJob {
  const float* X;
  int R, ld, C;
  float* out;
  int out_stride;
};
struct ColJobs {
  ColJob j[4];
  int first[5];
};
__global__ void colsum_jobs_kernel(ColJobs jobs) {
  int jb = 0;
  while (jb < 3 && (int)blockIdx.x >= jobs.first[jb + 1]) ++jb;
  const ColJob& J = jobs.j[jb];
  __shared__ float red[256];
  const int c = (int)blockIdx.x - jobs.first[jb];
  float acc = 0.f;
  for (int r = threadIdx.x; r < J.R; r += 256) acc += J.X[(size_t)r * J.ld + c];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s2 = 128; s2 > 0; s2 >>= 1) {
    if ((int)threadIdx.x < s2) red[threadIdx.x] += red[threadIdx.x + s2];
    __syncthreads();
  }
  if (threadIdx.x == 0) J.out[(size_t)c * J.out_stride] = red[0];
}

// ---------------------------------------------------------------------- TD ----
// dqn.py:403-440 for a reversible env: q_t = target(s')[argmax online(s')] (double DQN),
// td = r + (1 - done) * gamma * q_t, loss = mean((q(s,a) - td)^2), dq = dloss/dq.
// One thread per element of dq[B][N]: the element of the taken action gets the TD gradient (and its row's
// squared error), every other element zero -- the zero-fill of loss.backward()'s dQ and the TD step in one pass.
__global__ void td_kernel(const float* q_s, const float* q_tn, const int32_t* a_star, const int32_t* actions,
                          const float* rewards, const float* dones, int B, int N, float gamma, int clip,
                          float* dq, float* sqerr) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)B * N) return;
  const int b = (int)(i / N), j = (int)(i - (size_t)b * N);
  int a = actions[b];
  if ((unsigned)a >= (unsigned)N) a = 0;
  if (j != a) {
    dq[i] = 0.f;
    return;
  }
  int as = a_star[b];
  if ((unsigned)as >= (unsigned)N) as = 0;  // never index outside the row (all-masked argmax is 0)
  float qt = q_tn[(size_t)b * N + as];
  if (clip && qt < 0.f) qt = 0.f;  // clip_Q_targets (dqn.py:431-432)
  const float td = rewards[b] + (1.f - dones[b]) * gamma * qt;
  const float q = q_s[i];
  const float diff = q - td;
  dq[i] = 2.f * diff / (float)B;  // mse_loss(reduction='mean') backward
  sqerr[b] = diff * diff;
}

__global__ void mean_kernel(const float* v, int n, float* out) {
  __shared__ float red[256];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) acc += v[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0] / (float)n;
}

// -------------------------------------------------------------------- Adam ----
// torch.optim.Adam (amsgrad=False): m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2;
// p -= step_size * m / (sqrt(v)/sqrt(bc2) + eps)      (dqn.py:212, :443-449)
__global__ void adam_kernel(float* p, const float* g, float* m, float* v, int n, float b1, float b2, float step_size,
                            float bc2_sqrt, float eps, float wd, float gscale) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float gi = gscale == 1.f ? g[i] : g[i] * gscale;
  if (wd != 0.f) gi = fmaf(wd, p[i], gi);
  const float mi = m[i] + (1.f - b1) * (gi - m[i]);
  const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = p[i] - step_size * (mi / denom);
}

// ------------------------------------------------------------------ replay ----
// ReplayBuffer (dqn/utils.py:28-83) as a device ring of compact transitions:
// node features of s and s' ([N][x_stride] fp32), graph id, action, reward, done.
__device__ __forceinline__ int xstride(const eco_replay& rb) { return rb.x_stride == 16 ? 16 : 8; }

__global__ void replay_push_kernel(eco_replay rb, int pos, int B, const float* xs, const float* xn,
                                   const int32_t* gids, const int32_t* actions, const double* rewards,
                                   const uint8_t* dones) {
  const int b = blockIdx.y;
  if (b >= B) return;
  const int slot = (int)(((long long)pos + b) % rb.capacity);
  const int per = rb.n_spins * xstride(rb) / 4;  // float4s per state
  const float4* s4 = reinterpret_cast<const float4*>(xs + (size_t)b * rb.n_spins * xstride(rb));
  const float4* n4 = reinterpret_cast<const float4*>(xn + (size_t)b * rb.n_spins * xstride(rb));
  float4* ds = reinterpret_cast<float4*>(rb.xs + (size_t)slot * rb.n_spins * xstride(rb));
  float4* dn = reinterpret_cast<float4*>(rb.xn + (size_t)slot * rb.n_spins * xstride(rb));
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < per; i += gridDim.x * blockDim.x) {
    ds[i] = s4[i];
    dn[i] = n4[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    rb.gid[slot] = gids[b];
    rb.act[slot] = actions[b];
    rb.rew[slot] = (float)rewards[b];  // torch.as_tensor([reward], dtype=torch.float) (dqn.py:299)
    rb.done[slot] = dones[b] ? 1.f : 0.f;
  }
}

// Feistel bijection on [0, 2^bits) with cycle walking into [0, n): distinct indices,
// i.e. sampling WITHOUT replacement like random.sample (dqn/utils.py:53).
__device__ __forceinline__ uint32_t feistel(uint32_t x, int half, uint64_t key) {
  const uint32_t mask = (1u << half) - 1u;
  uint32_t L = x >> half, R = x & mask;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t F = (uint32_t)(rng3(key, (uint64_t)r, (uint64_t)R) & mask);
    const uint32_t nL = R;
    R = L ^ F;
    L = nL;
  }
  return (L << half) | R;
}

__global__ void replay_sample_kernel(eco_replay rb, int size, int M, uint64_t key, float* xs, float* xn,
                                     int32_t* gid, int32_t* act, float* rew, float* done) {
  const int m = blockIdx.y;
  if (m >= M) return;
  int bits = 2;
  while ((1 << bits) < size) ++bits;
  if (bits & 1) ++bits;
  const int half = bits / 2;
  uint32_t x = (uint32_t)m;
  do { x = feistel(x, half, key); } while (x >= (uint32_t)size);
  const int slot = (int)x;
  const int per = rb.n_spins * xstride(rb) / 4;
  const float4* s4 = reinterpret_cast<const float4*>(rb.xs + (size_t)slot * rb.n_spins * xstride(rb));
  const float4* n4 = reinterpret_cast<const float4*>(rb.xn + (size_t)slot * rb.n_spins * xstride(rb));
  float4* ds = reinterpret_cast<float4*>(xs + (size_t)m * rb.n_spins * xstride(rb));
  float4* dn = reinterpret_cast<float4*>(xn + (size_t)m * rb.n_spins * xstride(rb));
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < per; i += gridDim.x * blockDim.x) {
    ds[i] = s4[i];
    dn[i] = n4[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    gid[m] = rb.gid[slot];
    act[m] = rb.act[slot];
    rew[m] = rb.rew[slot];
    done[m] = rb.done[slot];
  }
}

// ------------------------------------------------------------ compact replay ----
// ReplayBuffer of MaxCut (OptimisationTarget.CUT) transitions as the env's integer state instead of fp32
// feature rows.  A transition stores ONE state: s, per vertex one u32 {spin sign bit 31 | time-since-flip
// count bits 16..30 | local field h = (J s)_v as int16 bits 0..15}; s' is a deterministic function of s, the
// action and the graph (env_step_kernel: flip spin a, reset its count, count +1 elsewhere, h_j -= 2 w_aj s_a
// over the CSR row of a), rebuilt on sample.  Per state the scalars {|score - best| / mlr, termination
// immanency, step t, Hamming distance to the best spins} are stored for s and s' (the Hamming distance needs
// the best spins, which are not kept).  4N + 80 B per transition (880 B at N=200) against 64N of the feature
// ring.  The sample kernel rebuilds the fp32 feature rows with the env's own obs_value (the same float64
// operations, so the features equal, bit for bit, the rows the env wrote).
// Ring of P = capacity + batch slots; transition k (k-th push, counted over the buffer's life) lives in slot
// k % P.  push(k0) writes the s' of episode e straight into slot (k0 + batch + e) % P as the s of that
// episode's next transition (a reset overwrites it through snapshot), so s is never copied; the `batch`
// slots ahead of the newest transition are never sampled (size <= capacity = P - batch).
// Layout: rows [P][N] u32 | ctx_s [P][4] f64 | ctx_n [P][4] f64 | gid | act | rew | done [P].
// act bit 30 marks a transition whose step left the state unchanged (an auto-masked finished episode).
constexpr uint32_t CR_NOFLIP = 0x40000000u;

struct CompactRing {
  uint32_t* rows;
  double *ctx_s, *ctx_n;
  int32_t *gid, *act;
  float *rew, *done;
};

static CompactRing compact_carve(void* base, int N, long long P, size_t* bytes = nullptr) {
  CompactRing r;
  char* b = (char*)base;
  size_t o = 0;
  auto t = [&](size_t n) { void* p = b + o; o = align_up(o + n, 256); return p; };
  r.rows = (uint32_t*)t((size_t)P * N * 4);
  r.ctx_s = (double*)t((size_t)P * 32);
  r.ctx_n = (double*)t((size_t)P * 32);
  r.gid = (int32_t*)t((size_t)P * 4);
  r.act = (int32_t*)t((size_t)P * 4);
  r.rew = (float*)t((size_t)P * 4);
  r.done = (float*)t((size_t)P * 4);
  if (bytes) *bytes = o;
  return r;
}

static size_t compact_bytes(int N, long long P) {
  size_t o = 0;
  compact_carve(nullptr, N, P, &o);
  return o;
}

// pack episode e's current state (spins, local field, time-since-flip counts, scalars) into rows / ctx (and
// ctx2 when given: the same scalars as the s' of the transition just taken)
__device__ __forceinline__ void compact_pack(const eco_env_config& cfg, const EnvLayout& L, const uint8_t* state, int e,
                                             uint32_t* rows, double* ctx, double* ctx2, int32_t* err) {
  const int N = L.N;
  const int8_t* sp = (const int8_t*)(state + L.off_spins) + (size_t)e * N;
  const int32_t* hf = (const int32_t*)(state + L.off_field) + (size_t)e * N;
  const int16_t* ts = (const int16_t*)(state + L.off_tsf) + (size_t)e * N;
  for (int v = threadIdx.x; v < N; v += blockDim.x) {
    const int h = hf[v];
    if (h < -32768 || h > 32767) atomicCAS(err, 0, ECO_ERR_GRAPH);  // compact rows need |J s| < 2^15
    rows[v] = (sp[v] < 0 ? 0x80000000u : 0u) | ((uint32_t)(ts[v] & 0x7FFF) << 16) | ((uint32_t)h & 0xFFFFu);
  }
  if (threadIdx.x < 4) {
    const EpScal* sc = (const EpScal*)(state + L.off_scal) + e;
    const int t = sc->t;
    double dist = 0.0, term = 0.0;  // a reset state's rows are 0 (_reset_state never sets them)
    if (t > 0) {
      const double dsc = sc->score - sc->best_score;
      dist = (dsc < 0.0 ? -dsc : dsc) / sc->mlr;                          // spinsystem.py:516-519
      const double x = (double)(t - cfg.max_steps) / (double)cfg.horizon_length + 1.0;
      term = x > 0.0 ? x : 0.0;                                           // :509-511
    }
    const double v = threadIdx.x == 0 ? dist : threadIdx.x == 1 ? term : threadIdx.x == 2 ? (double)t
                                                                                          : (double)sc->hamming;
    ctx[threadIdx.x] = v;
    if (ctx2) ctx2[threadIdx.x] = v;
  }
}

__device__ __forceinline__ long long cr_slot(long long k, long long P) { return k % P; }

__global__ __launch_bounds__(256) void replay_compact_snapshot_kernel(eco_env_config cfg, EnvLayout L, const uint8_t* state,
                                                                      CompactRing r, long long P, long long pushed,
                                                                      const uint8_t* mask, int32_t* err) {
  const int e = blockIdx.x;
  if (mask && !mask[e]) return;
  const long long slot = cr_slot(pushed + e, P);
  compact_pack(cfg, L, state, e, r.rows + slot * L.N, r.ctx_s + slot * 4, nullptr, err);
}

__global__ __launch_bounds__(256) void replay_compact_push_kernel(eco_env_config cfg, EnvLayout L, const uint8_t* state,
                                                                  CompactRing r, long long P, long long pushed, int B,
                                                                  const int32_t* actions, const double* rewards,
                                                                  const uint8_t* dones, int32_t* err) {
  const int e = blockIdx.x;
  const int N = L.N;
  const long long slot = cr_slot(pushed + e, P), next = cr_slot(pushed + B + e, P);
  if (threadIdx.x == 0) {
    const int a = actions[e];
    // did the step flip spin a (s' != s)?  An auto-masked finished episode returns its state unchanged.
    const bool flipped = a >= 0 && a < N &&
                         ((r.rows[slot * N + a] >> 31) != (uint32_t)(((const int8_t*)(state + L.off_spins))[(size_t)e * N + a] < 0));
    r.gid[slot] = ((const EpScal*)(state + L.off_scal) + e)->graph;
    r.act[slot] = (int32_t)((uint32_t)a | (flipped ? 0u : CR_NOFLIP));
    r.rew[slot] = (float)rewards[e];  // torch.as_tensor([reward], dtype=torch.float) (dqn.py:299)
    r.done[slot] = dones[e] ? 1.f : 0.f;
  }
  compact_pack(cfg, L, state, e, r.rows + next * N, r.ctx_s + next * 4, r.ctx_n + slot * 4, err);
}

// feature rows of one compact state, written exactly as write_obs does (same obs_value, same casts)
__device__ __forceinline__ void compact_expand(const eco_env_config& cfg, const uint32_t* rows, const double* ctx,
                                               double mlr, const double* tab, int N, float* out, int* red) {
  int cnt = 0;
  for (int v = threadIdx.x; v < N; v += blockDim.x) {
    const uint32_t w = rows[v];
    const int sv = (w >> 31) ? -1 : 1;
    const int h = (int)(int16_t)(w & 0xFFFFu);
    cnt += (sv * h > 0);
  }
  cnt = wave_sum_i(cnt);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  int total = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) total += red[k];
  ObsCtx c;
  c.mlr = mlr; c.dist_best = ctx[0]; c.term = ctx[1]; c.hamming = ctx[3];
  const int t = (int)ctx[2];
  c.ep_time = tab[t];
  c.nqi = (double)total / (double)N;
  c.basis = cfg.spin_basis;
  for (int v = threadIdx.x; v < N; v += blockDim.x) {
    const uint32_t w = rows[v];
    const int sv = (w >> 31) ? -1 : 1;
    const int tsfk = (int)((w >> 16) & 0x7FFFu);
    const int h = (int)(int16_t)(w & 0xFFFFu);
    float xf[ECO_MAX_OBS];
#pragma unroll
    for (int i = 0; i < ECO_MAX_OBS; ++i) xf[i] = i < cfg.n_obs ? (float)obs_value(cfg.obs_ids[i], c, sv, h, tsfk, tab) : 0.f;
    store_obs_row(out, (size_t)v, cfg.n_obs, xf);
  }
}

// grid (2, M): blockIdx.x = 0 rebuilds s, 1 rebuilds s' of the m-th sampled transition.  The Feistel index x
// names the slot the fp32 feature ring would read (replay_sample_kernel: slot x of a ring of `capacity`
// written at k % capacity); here it is resolved to the transition k == x (mod capacity) among the newest
// `size` and read from slot k % P.
__global__ __launch_bounds__(256) void replay_compact_sample_kernel(eco_env_config cfg, CompactRing r, long long P,
                                                                    int capacity, int size, long long pushed, int M,
                                                                    uint64_t key, const double* tab, eco_graph_set gs,
                                                                    float* xs, float* xn, int32_t* gid, int32_t* act,
                                                                    float* rew, float* done) {
  extern __shared__ uint32_t cr_lds[];
  __shared__ int red[4];
  const int m = blockIdx.y;
  if (m >= M) return;
  int bits = 2;
  while ((1 << bits) < size) ++bits;
  if (bits & 1) ++bits;
  const int half = bits / 2;
  uint32_t x = (uint32_t)m;
  do { x = feistel(x, half, key); } while (x >= (uint32_t)size);
  const long long base = pushed - size;  // oldest transition still held
  const long long k = base + (((long long)x - base % capacity) % capacity + capacity) % capacity;
  const long long slot = cr_slot(k, P);
  const int N = cfg.n_spins;
  const int W = ECO_OBS_X_STRIDE(cfg.n_obs);
  const int g = r.gid[slot];
  const double mlr = gs.meta[(size_t)g * 4];
  const uint32_t* rows = r.rows + slot * N;
  const uint32_t av = (uint32_t)r.act[slot];
  const int a = (int)(av & ~CR_NOFLIP);
  if (blockIdx.x == 0) {
    compact_expand(cfg, rows, r.ctx_s + slot * 4, mlr, tab, N, xs + (size_t)m * N * W, red);
    if (threadIdx.x == 0) { gid[m] = g; act[m] = a; rew[m] = r.rew[slot]; done[m] = r.done[slot]; }
    return;
  }
  // s' = env step of s by a (env_step_kernel, spinsystem.py:397, :492-497): flip a, counts, local field
  const bool flip = !(av & CR_NOFLIP);
  const int sa_old = (rows[a] >> 31) ? -1 : 1;
  for (int v = threadIdx.x; v < N; v += blockDim.x) {
    uint32_t w = rows[v];
    if (flip) {
      const uint32_t tsfk = v == a ? 0u : (((w >> 16) & 0x7FFFu) + 1u) & 0x7FFFu;
      w = ((v == a ? ~w : w) & 0x80000000u) | (tsfk << 16) | (w & 0xFFFFu);
    }
    cr_lds[v] = w;
  }
  __syncthreads();
  if (flip) {
    const int32_t* rp = gs.row_ptr + (size_t)g * (N + 1);
    const uint32_t* ed = gs.edges + gs.edge_base[g];
    for (int q = rp[a] + threadIdx.x; q < rp[a + 1]; q += blockDim.x) {
      const uint32_t ex = ed[q];
      const int j = edge_col(ex);
      const uint32_t w = cr_lds[j];
      const int h = (int)(int16_t)(w & 0xFFFFu) - 2 * edge_w(ex) * sa_old;
      cr_lds[j] = (w & 0xFFFF0000u) | ((uint32_t)h & 0xFFFFu);
    }
    __syncthreads();
  }
  compact_expand(cfg, cr_lds, r.ctx_n + slot * 4, mlr, tab, N, xn + (size_t)m * N * W, red);
}

static size_t slab_bytes() { return (size_t)MAX_JOBS * SLABS_PER_JOB * SLAB * sizeof(float); }

}  // namespace eco

using namespace eco;

extern "C" size_t eco_mpnn_backward_workspace_bytes(int32_t n_spins, int32_t batch) {
  const size_t g = mpnn_grad_ws_bytes(n_spins, batch);
  if (!g) return 0;
  return align_up(g, 256) + slab_bytes();
}

extern "C" int eco_mpnn_backward(const float* packed, int32_t n_obs_in, const eco_graph_set* gs,
                                 const int32_t* graph_ids, int32_t batch, const float* obs_x, const void* saved,
                                 const float* dq, float* grad, void* workspace, eco_stream_t stream) {
  if (!grad || !workspace) return fail(ECO_ERR_ARG, "null grad/workspace");
  hipStream_t st = (hipStream_t)stream;
  int rc = mpnn_backward_launch(packed, n_obs_in, gs, graph_ids, batch, obs_x, saved, dq, workspace, st);
  if (rc) return rc;
  const int N = gs->n_spins;
  const size_t RT = (size_t)batch * N;
  if (RT > (size_t)INT32_MAX / 64) return fail(ECO_ERR_ARG, "batch * n_spins too large");
  const float* sv = (const float*)saved;
  const float* gr = (const float*)workspace;
  auto SV = [&](int t) { return sv + (size_t)t * RT * 64; };
  auto GR = [&](int t) { return gr + (size_t)t * RT * 64; };
  const float* MEAN = sv + (size_t)SV_NODE_TENSORS * RT * 64;
  const float* DP = gr + (size_t)GR_NODE_TENSORS * RT * 64;
  const float* DWRA = DP + (size_t)batch * 64;
  const float* DWRB = DWRA + (size_t)batch * 64;
  const float* DBR = DWRB + (size_t)batch * 64;
  const float* DWA = DBR + (((size_t)batch + 63) & ~63ull);
  const int gpb = graphs_per_block(N, batch);
  const int nblk = (batch + gpb - 1) / gpb;
  float* slabs = (float*)((char*)workspace + align_up(mpnn_grad_ws_bytes(N, batch), 256));
  const FlatOffsets fo = flat_offsets(n_obs_in);
  WJobs J{};
  int n = 0;
  const int R = (int)RT;
  for (int l = 0; l < 3; ++l) {
    J.j[n++] = WJob{GR(GR_DUM0 + l), SV(SV_AGG0 + l), SV(SV_E), 64, 64, 64, 64, R, 64, fo.L + l * 16384, 128, 0};
    J.j[n++] = WJob{GR(GR_DUU0 + l), SV(SV_H0 + l), SV(SV_M0 + l), 64, 64, 64, 64, R, 64, fo.L + l * 16384 + 8192,
                    128, 0};
  }
  J.j[n++] = WJob{GR(GR_DUE), SV(SV_EAGG), nullptr, 64, 64, 0, 0, R, 64, fo.Wf, 64, 0};
  const int xw = ECO_OBS_X_STRIDE(n_obs_in);
  J.j[n++] = WJob{GR(GR_DU0), obs_x, nullptr, xw, n_obs_in, 0, 0, R, 64, fo.W0, n_obs_in, 0};
  J.j[n++] = WJob{GR(GR_DZ), obs_x, nullptr, xw, n_obs_in, 0, 0, R, 63, fo.We, 1 + n_obs_in, 1};
  J.j[n++] = WJob{DP, MEAN, nullptr, 64, 64, 0, 0, batch, 64, fo.Wp, 64, 0};
  J.n = n;
  {
    // one resident wave of workgroups over the 256 CUs (46 KB LDS: 3 per CU for bf16x3; 27 KB and 168 VGPRs:
    // 3 per CU for fp16x2).  Measured splits (M = 2048 ER-200): in proportion to the bytes each job reads,
    // 1.28 vs 1.05 ms per gradient step of backward + weight gradients against an even split; more workgroups
    // for the K = 128 jobs at the others' expense (96 / 112 each) slower again (9.25 / 12.1 vs 8.66 ms
    // per vector step): the K <= 64 jobs cost as much per row.  The fp16x2 variant (round 3)
    // measured 0.62 vs 0.52 ms per launch: its per-fragment scales and splits sit after the barrier, on the
    // critical path.
    const int total = WGRAD_WG_X * 256;
    double rows = 0.0;
    for (int j = 0; j < n; ++j) rows += J.j[j].R;
    J.first[0] = 0;
    for (int j = 0; j < n; ++j) {
      // in proportion to the job's rows (a row costs about the same in every job); the per-graph readout job
      // (R = batch) gets one
      const int g = (int)(total * (double)J.j[j].R / rows);
      J.nwgj[j] = std::max(1, std::min(WG_PER_JOB, g));
      J.first[j + 1] = J.first[j] + J.nwgj[j];
    }
    wgrad_bf3_kernel<<<J.first[n], 256, 0, st>>>(J, slabs);
  }
  wgrad_reduce_kernel<<<dim3(64 * 128 / 256, n), 256, 0, st>>>(J, slabs, grad);
  ColJobs CJ{};
  CJ.j[0] = ColJob{DWRA, batch, 64, 64, grad + fo.Wr, 1};
  CJ.j[1] = ColJob{DWRB, batch, 64, 64, grad + fo.Wr + 64, 1};
  CJ.j[2] = ColJob{DBR, batch, 1, 1, grad + fo.Br, 1};
  CJ.j[3] = ColJob{DWA, nblk, 64, 63, grad + fo.We, 1 + n_obs_in};
  CJ.first[0] = 0;
  for (int k = 0; k < 4; ++k) CJ.first[k + 1] = CJ.first[k] + CJ.j[k].C;
  colsum_jobs_kernel<<<CJ.first[4], 256, 0, st>>>(CJ);
  return check_launch("mpnn_backward_wgrad");
}

extern "C" int eco_dqn_td(const float* q_s, const float* q_target_next, const int32_t* a_star,
                          const int32_t* actions, const float* rewards, const float* dones, int32_t batch,
                          int32_t n_spins, float gamma, int32_t clip_q_targets, float* dq, float* sqerr,
                          float* loss, eco_stream_t stream) {
  if (!q_s || !q_target_next || !a_star || !actions || !rewards || !dones || !dq || !sqerr || !loss)
    return fail(ECO_ERR_ARG, "null argument");
  if (batch < 1 || n_spins < 1) return fail(ECO_ERR_ARG, "bad batch/n_spins");
  hipStream_t st = (hipStream_t)stream;
  const size_t n = (size_t)batch * n_spins;
  td_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(q_s, q_target_next, a_star, actions, rewards, dones, batch,
                                                         n_spins, gamma, clip_q_targets, dq, sqerr);
  mean_kernel<<<1, 256, 0, st>>>(sqerr, batch, loss);
  return check_launch("dqn_td");
}

extern "C" int eco_adam(float* params, const float* grad, float* exp_avg, float* exp_avg_sq, int32_t n, double lr,
                        double beta1, double beta2, double eps, double weight_decay, double grad_scale, int64_t step,
                        eco_stream_t stream) {
  if (!params || !grad || !exp_avg || !exp_avg_sq || n < 1 || step < 1) return fail(ECO_ERR_ARG, "bad adam args");
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  adam_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(params, grad, exp_avg, exp_avg_sq, n, (float)beta1,
                                                               (float)beta2, (float)(lr / bc1),
                                                               (float)std::sqrt(bc2), (float)eps,
                                                               (float)weight_decay, (float)grad_scale);
  return check_launch("adam");
}

extern "C" int eco_replay_push(const eco_replay* rb, int32_t pos, int32_t batch, const float* xs, const float* xn,
                               const int32_t* graph_ids, const int32_t* actions, const double* rewards,
                               const uint8_t* dones, eco_stream_t stream) {
  if (!rb || !xs || !xn || !graph_ids || !actions || !rewards || !dones) return fail(ECO_ERR_ARG, "null argument");
  if (rb->x_stride != 0 && rb->x_stride != 8 && rb->x_stride != 16) return fail(ECO_ERR_ARG, "x_stride must be 8 or 16");
  if (batch < 1 || rb->capacity < 1 || pos < 0) return fail(ECO_ERR_ARG, "bad batch/capacity/pos");
  if (batch > rb->capacity) return fail(ECO_ERR_ARG, "replay push: batch larger than the ring (slots would collide)");
  replay_push_kernel<<<dim3(1, batch), 256, 0, (hipStream_t)stream>>>(*rb, pos, batch, xs, xn, graph_ids, actions,
                                                                      rewards, dones);
  return check_launch("replay_push");
}

extern "C" int eco_replay_sample(const eco_replay* rb, int32_t size, int32_t m, uint64_t seed, uint64_t counter,
                                 float* xs, float* xn, int32_t* graph_ids, int32_t* actions, float* rewards,
                                 float* dones, eco_stream_t stream) {
  if (!rb || !xs || !xn || !graph_ids || !actions || !rewards || !dones) return fail(ECO_ERR_ARG, "null argument");
  if (rb->x_stride != 0 && rb->x_stride != 8 && rb->x_stride != 16) return fail(ECO_ERR_ARG, "x_stride must be 8 or 16");
  if (size < m || m < 1 || size > rb->capacity)
    return fail(ECO_ERR_ARG, "replay sample: need m <= size <= capacity (random.sample without replacement)");
  replay_sample_kernel<<<dim3(1, m), 256, 0, (hipStream_t)stream>>>(*rb, size, m, rng3(seed, counter, 0x5A5A),
                                                                    xs, xn, graph_ids, actions, rewards, dones);
  return check_launch("replay_sample");
}

static int compact_check(const eco_env_config* cfg, int32_t batch, int32_t capacity) {
  if (!cfg) return fail(ECO_ERR_ARG, "null config");
  if (cfg->optimisation_target != ECO_TARGET_CUT) return fail(ECO_ERR_TARGET, "compact replay: OptimisationTarget.CUT only");
  if (cfg->max_steps > 32767) return fail(ECO_ERR_ARG, "compact replay: max_steps must be < 32768");
  if (cfg->n_spins < 1 || cfg->n_spins > ECO_COMPACT_MAX_SPINS) return fail(ECO_ERR_ARG, "compact replay: n_spins out of range");
  if (batch < 1 || capacity < 1) return fail(ECO_ERR_ARG, "bad batch/capacity");
  return ECO_OK;
}

extern "C" size_t eco_replay_compact_bytes(int32_t n_spins, int32_t capacity, int32_t batch) {
  if (n_spins < 1 || n_spins > ECO_COMPACT_MAX_SPINS || capacity < 1 || batch < 1) return 0;
  return compact_bytes(n_spins, (long long)capacity + batch);
}

extern "C" int eco_replay_compact_snapshot(const eco_env_config* cfg, const void* env_state, int32_t batch, void* ring,
                                           int32_t capacity, int64_t pushed, const uint8_t* mask, eco_stream_t stream) {
  int rc = compact_check(cfg, batch, capacity);
  if (rc) return rc;
  if (!env_state || !ring || pushed < 0) return fail(ECO_ERR_ARG, "null state/ring or negative push count");
  const EnvLayout L = env_layout(cfg->n_spins, cfg->max_steps, batch);
  const long long P = (long long)capacity + batch;
  replay_compact_snapshot_kernel<<<batch, 256, 0, (hipStream_t)stream>>>(
      *cfg, L, (const uint8_t*)env_state, compact_carve(ring, cfg->n_spins, P), P, pushed, mask, err_word());
  return check_launch("replay_compact_snapshot");
}

extern "C" int eco_replay_compact_push(const eco_env_config* cfg, const void* env_state, int32_t batch, void* ring,
                                       int32_t capacity, int64_t pushed, const int32_t* actions, const double* rewards,
                                       const uint8_t* dones, eco_stream_t stream) {
  int rc = compact_check(cfg, batch, capacity);
  if (rc) return rc;
  if (!env_state || !ring || !actions || !rewards || !dones) return fail(ECO_ERR_ARG, "null argument");
  if (pushed < 0 || batch > capacity) return fail(ECO_ERR_ARG, "replay push: negative push count or batch larger than the ring");
  const EnvLayout L = env_layout(cfg->n_spins, cfg->max_steps, batch);
  const long long P = (long long)capacity + batch;
  replay_compact_push_kernel<<<batch, 256, 0, (hipStream_t)stream>>>(
      *cfg, L, (const uint8_t*)env_state, compact_carve(ring, cfg->n_spins, P), P, pushed, batch, actions, rewards,
      dones, err_word());
  return check_launch("replay_compact_push");
}

extern "C" int eco_replay_compact_sample(const eco_env_config* cfg, const void* env_state, const eco_graph_set* gs,
                                         int32_t env_batch, const void* ring, int32_t capacity, int32_t size,
                                         int64_t pushed, int32_t m, uint64_t seed, uint64_t counter, float* xs,
                                         float* xn, int32_t* graph_ids, int32_t* actions, float* rewards, float* dones,
                                         eco_stream_t stream) {
  int rc = compact_check(cfg, env_batch, capacity);
  if (rc) return rc;
  if (!env_state || !gs || !ring || !xs || !xn || !graph_ids || !actions || !rewards || !dones)
    return fail(ECO_ERR_ARG, "null argument");
  if (size < m || m < 1 || size > capacity || pushed < size)
    return fail(ECO_ERR_ARG, "replay sample: need m <= size <= min(capacity, pushed) (random.sample without replacement)");
  if (gs->n_spins != cfg->n_spins) return fail(ECO_ERR_ARG, "replay sample: graph set / env size mismatch");
  const EnvLayout L = env_layout(cfg->n_spins, cfg->max_steps, env_batch);
  const double* tab = (const double*)((const uint8_t*)env_state + L.off_tab + 256);
  const long long P = (long long)capacity + env_batch;
  // threads per transition: 4096 workgroups of a few nodes' work each are latency chains (ring slot -> graph ->
  // rows -> count -> features); smaller workgroups keep more of them resident
  // (ER-200 x M = 2048: 30.6 / 24.2 / 21.0 us per call at 256 / 128 / 64 threads, profiles/r03/ab/sample_threads_*)
  const int nt = cfg->n_spins <= 256 ? 64 : 128;
  replay_compact_sample_kernel<<<dim3(2, m), nt, (size_t)cfg->n_spins * 4, (hipStream_t)stream>>>(
      *cfg, compact_carve(const_cast<void*>(ring), cfg->n_spins, P), P, capacity, size, pushed, m,
      rng3(seed, counter, 0x5A5A), tab, *gs, xs, xn, graph_ids, actions, rewards, dones);
  return check_launch("replay_compact_sample");
}
