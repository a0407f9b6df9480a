// Device-side pieces shared by the batched env kernels: the MaxCut kernels (eco_env.hip) and the
// generic-scorer kernels (eco_env_problems.hip).
#pragma once
#include "eco_common.h"

namespace eco {

struct EnvArgs {
  eco_env_config cfg;
  eco_graph_set gs;
  EnvLayout L;
  uint8_t* state;
  int B;
  const int32_t* graph_ids;
  const int8_t* spins_in;
  const uint8_t* mask;
  uint64_t seed;
  const int32_t* actions;
  double* rewards;
  uint8_t* dones;
  float* obs_x;
  double* obs_f64;
  int32_t* err;  // device error word (first error wins)
};

__device__ __forceinline__ EpScal* scal_ptr(const EnvArgs& a) { return (EpScal*)(a.state + a.L.off_scal); }
__device__ __forceinline__ const double* tab_ptr(const EnvArgs& a) { return (const double*)(a.state + a.L.off_tab + 256); }

// one node's fp32 feature row: ECO_OBS_X_STRIDE(nobs) floats (8, or 16 beyond 8 observables)
__device__ __forceinline__ void store_obs_row(float* obs_x, size_t row, int nobs, const float (&xf)[ECO_MAX_OBS]) {
  if (nobs <= 8) {
    float4* dst = (float4*)(obs_x + row * 8);
    dst[0] = make_float4(xf[0], xf[1], xf[2], xf[3]);
    dst[1] = make_float4(xf[4], xf[5], xf[6], xf[7]);
  } else {
    float4* dst = (float4*)(obs_x + row * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = make_float4(xf[4 * i], xf[4 * i + 1], xf[4 * i + 2], xf[4 * i + 3]);
  }
}

// One observable row value, float64, exactly as spinsystem.py:303-328 / :486-535.
struct ObsCtx {
  double mlr, dist_best, hamming, nqi, term, ep_time;
  int basis;
};
// g is passed as the field h; the reference's g = s * (J@s) is a float64 product, so
// s = -1 with h = +0.0 gives -0.0 (kept: observations are compared bitwise).
__device__ __forceinline__ double obs_value(int id, const ObsCtx& c, int s, int h, int tsfk, const double* tab) {
  switch (id) {
    case ECO_OBS_SPIN_STATE: return c.basis == ECO_BASIS_BINARY ? (double)(1 - s) / 2.0 : (double)s;
    case ECO_OBS_IMMEDIATE_QUALITY_CHANGE: return ((double)s * (double)h) / c.mlr;
    case ECO_OBS_TIME_SINCE_FLIP: return tab[tsfk];
    case ECO_OBS_EPISODE_TIME: return c.ep_time;
    case ECO_OBS_TERMINATION_IMMANENCY: return c.term;
    case ECO_OBS_NUMBER_OF_QUALITY_IMPROVEMENTS: return c.nqi;
    case ECO_OBS_DISTANCE_FROM_BEST_SOLUTION: return c.dist_best;
    case ECO_OBS_DISTANCE_FROM_BEST_STATE: return c.hamming;
    case ECO_OBS_VALIDITY_BIT: return 1.0;  // MaxCut: every spin vector is valid
    default: return 0.0;  // GLOBAL_VALIDITY_DIFFERENCE: (0 - 0) / 1 (the mask observables are rejected)
  }
}

// LDS written by a wave and read back by the same wave only: a wave-scope fence suffices
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Pre-flip spin and field of vertex `act` (lane act & 63, slot act >> 6) from the wave's registers.
template <int VPT>
__device__ __forceinline__ void read_vertex(const int (&s)[VPT], const int (&f)[VPT], int act, int& sa, int& fa) {
  const int kk = act >> 6, la = act & 63;
  sa = 0;
  fa = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k)
    if (k == kk) { sa = __builtin_amdgcn_readlane(s[k], la); fa = __builtin_amdgcn_readlane(f[k], la); }
}

// f_j += coef(J_ja) for every neighbour j of `act`: the lanes load the CSR row in parallel and scatter the
// deltas through the wave's LDS slice dl[N] (a row has distinct columns, so the stores never collide) --
// one round of loads instead of deg(a) dependent ones.
struct NoIssue {
  __device__ void operator()() const {}
};
// after_loads: issued right after the row's edge loads (the step's next loads, e.g. the visited-set probe)
template <int VPT, class Coef, class After = NoIssue>
__device__ __forceinline__ void row_update(int32_t* dl, const uint32_t* ed, int q0, int q1, int N, int lane,
                                           int (&f)[VPT], Coef coef, After after_loads = After()) {
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) dl[v] = 0;
  }
  wave_lds_sync();
  if (q1 - q0 <= 64) {  // one load per lane (every ER-200 / BA-500 row): the caller's next loads go out behind it
    const uint32_t x = q0 + lane < q1 ? ed[q0 + lane] : 0u;
    after_loads();
    if (q0 + lane < q1) dl[edge_col(x)] = coef(edge_w(x));
  } else {
    after_loads();
    for (int q = q0 + lane; q < q1; q += 64) {
      const uint32_t x = ed[q];
      dl[edge_col(x)] = coef(edge_w(x));
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) f[k] += dl[v];
  }
}

// HistoryBuffer.update (src/envs/utils.py:438-464): is the flipped-vertex set after flipping `act` new?
// The set is identified by the spin configuration (words = ballot(s > 0) per 64 vertices); a Zobrist
// hash of the set indexes an open-addressing table of the episode's visited configurations.  The
// initial (empty) set is never inserted, as in the reference.
template <int VPT>
__device__ __forceinline__ bool history_update(const EnvArgs& a, int e, int lane, EpScal* sc, int act,
                                               const uint64_t (&words)[VPT]) {
  const EnvLayout& L = a.L;
  const int T = a.cfg.max_steps;
  const uint64_t hash = sc->hash ^ zobrist(act);
  const int cap = L.cap;
  const int W = L.words;
  uint32_t* vidx = (uint32_t*)(a.state + L.off_vidx) + (size_t)e * cap;
  uint64_t* vh = (uint64_t*)(a.state + L.off_vhash) + (size_t)e * cap;
  uint64_t* vst = (uint64_t*)(a.state + L.off_vstates) + (size_t)e * (T + 1) * W;
  bool isnew = true;
  int slot = (int)(hash & (uint64_t)(cap - 1));
  for (;;) {
    const uint32_t id = vidx[slot];
    const uint64_t hs = vh[slot];  // issued together with the index load
    if (id == 0u) break;
    if (hs == hash) {
      bool same = true;
#pragma unroll
      for (int k = 0; k < VPT; ++k) same = same && (k >= W || vst[(size_t)(id - 1) * W + k] == words[k]);
      if (same) { isnew = false; break; }
    }
    slot = (slot + 1) & (cap - 1);
  }
  if (lane == 0) {
    sc->hash = hash;
    if (isnew) {
      const int n = sc->visit_count;
#pragma unroll
      for (int k = 0; k < VPT; ++k)
        if (k < W) vst[(size_t)n * W + k] = words[k];  // VPT = next power of two >= W
      vh[slot] = hash;
      vidx[slot] = (uint32_t)(n + 1);
      sc->visit_count = n + 1;
    }
  }
  return isnew;
}

// The same update with the first probe slot loaded ahead by the caller (history_probe, issued right after the
// step's CSR-row loads so its latency runs under the field update and the ballots; vmcnt is in order, so issuing
// it before loads the step needs sooner would delay those instead).
struct HistProbe {
  uint64_t hash;
  int slot;
  uint32_t id;
  uint64_t hs;
};
__device__ __forceinline__ void history_probe(const EnvArgs& a, int e, uint64_t prev_hash, int act, HistProbe& p) {
  const EnvLayout& L = a.L;
  const int cap = L.cap;
  p.hash = prev_hash ^ zobrist(act);
  p.slot = (int)(p.hash & (uint64_t)(cap - 1));
  p.id = ((const uint32_t*)(a.state + L.off_vidx) + (size_t)e * cap)[p.slot];
  p.hs = ((const uint64_t*)(a.state + L.off_vhash) + (size_t)e * cap)[p.slot];
}
template <int VPT>
__device__ __forceinline__ bool history_update_from(const EnvArgs& a, int e, int lane, EpScal* sc, const HistProbe& p,
                                                    const uint64_t (&words)[VPT]) {
  const EnvLayout& L = a.L;
  const int T = a.cfg.max_steps;
  const int cap = L.cap;
  const int W = L.words;
  uint32_t* vidx = (uint32_t*)(a.state + L.off_vidx) + (size_t)e * cap;
  uint64_t* vh = (uint64_t*)(a.state + L.off_vhash) + (size_t)e * cap;
  uint64_t* vst = (uint64_t*)(a.state + L.off_vstates) + (size_t)e * (T + 1) * W;
  bool isnew = true;
  int slot = p.slot;
  uint32_t id = p.id;
  uint64_t hs = p.hs;
  for (;;) {
    if (id == 0u) break;
    if (hs == p.hash) {
      bool same = true;
#pragma unroll
      for (int k = 0; k < VPT; ++k) same = same && (k >= W || vst[(size_t)(id - 1) * W + k] == words[k]);
      if (same) { isnew = false; break; }
    }
    slot = (slot + 1) & (cap - 1);
    id = vidx[slot];
    hs = vh[slot];
  }
  if (lane == 0) {
    sc->hash = p.hash;
    if (isnew) {
      const int n = sc->visit_count;
#pragma unroll
      for (int k = 0; k < VPT; ++k)
        if (k < W) vst[(size_t)n * W + k] = words[k];
      vh[slot] = p.hash;
      vidx[slot] = (uint32_t)(n + 1);
      sc->visit_count = n + 1;
    }
  }
  return isnew;
}

// vertices per lane for N spins (one 64-lane wave per episode)
// dynamic LDS of the step kernels: int32 row deltas [4 waves][N], then MinDomSet codes [4][N]
inline size_t env_step_lds(int N) { return (size_t)4 * N * 4 + (size_t)4 * N; }

#define ECO_DISPATCH_VPT(N, CALL)                                   \
  do {                                                              \
    if ((N) <= 64) { constexpr int V = 1; CALL; }                   \
    else if ((N) <= 128) { constexpr int V = 2; CALL; }             \
    else if ((N) <= 256) { constexpr int V = 4; CALL; }             \
    else if ((N) <= 512) { constexpr int V = 8; CALL; }             \
    else if ((N) <= 1024) { constexpr int V = 16; CALL; }           \
    else { constexpr int V = 32; CALL; }                            \
  } while (0)

// generic-scorer launches (eco_env_problems.hip): 4 episodes per 256-thread block, lds = env_step_lds(N)
int env_reset_problem_launch(const EnvArgs& a, int blocks, size_t lds, hipStream_t st);
int env_step_problem_launch(const EnvArgs& a, int blocks, size_t lds, hipStream_t st);
int env_greedy_problem_launch(const EnvArgs& a, int32_t* actions, int blocks, size_t lds, hipStream_t st);

}  // namespace eco
