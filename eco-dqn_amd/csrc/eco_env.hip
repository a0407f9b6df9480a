// Batched MaxCut SpinSystem on gfx950: graph preparation, reset, step, read-out.
//
// One 64-lane wave owns one episode; lane l owns vertices l, l+64, ... (VPT per
// lane), so every per-vertex reduction of the reference step (count of positive
// gains, all(g<=0), Hamming distance to best, the visited-state bitset) is a
// ballot/popcount and the episode scalars live in SGPRs.  The local field
// h = J.s is kept resident and updated by ONE CSR row per flip
// (h_j -= 2 w_aj s_a), so a step touches deg(a) edges instead of the reference's
// four dense J@s matvecs and two dense calculate_cut quadratic forms
// (spinsystem.py:393-416, 516-519).  All scores are exact integers in f64, and the
// f64 observation values are produced by the same IEEE operations as the
// reference, so rewards/observations match it bit for bit.
#include "eco_common.h"
#include "eco_mpnn.h"
#include "eco_env_dev.h"

namespace eco {

// ------------------------------------------------------------------ graphs ----
// score_solver.py:347-375 (normalisers) and mpnn.py:34-38 (degree norm).
// The graph's edge words are streamed ONCE, coalesced (thread t of the graph reads edges t, t + 64 WPG,
// ...), and each lane follows its edge's row through the row pointers staged in LDS (rows are contiguous, so a
// lane's row index only moves forward); per-vertex row sums and nonzero counts are LDS integer atomics (exact,
// order-free).  Walking one row per lane instead (each lane its own vertex's row) moved 3.58 GB for 8,192
// ER-200 graphs (18x their CSR): every load instruction touched 64 different lines.
constexpr int GP_WAVES = 4;
// WPG waves per graph: 1 for N <= 512 (four graphs per workgroup, wave-level sync only), all four for larger
// graphs (one graph per workgroup: a lone wave took 353 us over the 40 k edge words of a G22-like graph)
template <int WPG>
__global__ __launch_bounds__(64 * GP_WAVES) void graphs_prepare_kernel(eco_graph_set gs, int first, int count) {
  extern __shared__ int gp_lds[];  // per graph: rp [N + 1], rowsum [N], deg [N]
  constexpr int GPB = GP_WAVES / WPG;
  constexpr int NTG = 64 * WPG;  // threads per graph
  const int lane = threadIdx.x & 63;
  const int gl = (int)threadIdx.x / NTG;  // graph of the workgroup
  const int tg = (int)threadIdx.x % NTG;  // thread within the graph
  const int g = first + blockIdx.x * GPB + gl;
  const bool live = g < first + count;  // WPG == 1: wave-uniform; WPG > 1: one graph per workgroup
  if (WPG == 1 && !live) return;
  const int N = gs.n_spins;
  int* rpl = gp_lds + gl * (3 * N + 1);
  int* rsum = rpl + N + 1;
  int* dcnt = rsum + N;
  auto sync = [&]() {
    if (WPG == 1) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS operations done
      __builtin_amdgcn_wave_barrier();
    } else {
      __syncthreads();
    }
  };
  const int32_t* rp = gs.row_ptr + (size_t)g * (N + 1);
  const uint32_t* ed = gs.edges + gs.edge_base[live ? g : first];
  if (live) {
    for (int v = tg; v <= N; v += NTG) rpl[v] = rp[v];
    for (int v = tg; v < N; v += NTG) rsum[v] = dcnt[v] = 0;
  }
  sync();
  long long pos = 0, neg = 0;
  if (live) {
    const int e0 = rpl[0], e1 = rpl[N];
    int row = 0;
    for (int e = e0 + tg; e < e1; e += NTG) {
      while (rpl[row + 1] <= e) ++row;  // the row holding edge e (empty rows skipped)
      const int w = edge_w(ed[e]);
      if (w > 0) pos += w; else neg += w;
      if (w != 0) {
        atomicAdd(&rsum[row], w);
        atomicAdd(&dcnt[row], 1);
      }
    }
  }
  sync();
  long long sum = 0;
  int mdeg = 1;
  int best = INT_MIN;
  int has = 0;
  if (live) {
    for (int v = tg; v < N; v += NTG) {
      const int rs = rsum[v], d = dcnt[v];
      sum += rs;
      gs.deg[(size_t)g * N + v] = d;
      mdeg = max(mdeg, max(d, 1));
      // g(s=-1)_v = (-1) * (J.(-1))_v = row sum; mlr = max over NONZERO entries
      if (rs != 0) { has = 1; best = max(best, rs); }
    }
  }
  pos = wave_sum_ll(pos);
  neg = wave_sum_ll(neg);
  sum = wave_sum_ll(sum);
  mdeg = wave_max_i(mdeg);
  best = wave_max_i(best);
  has = wave_max_i(has);
  if (WPG > 1) {  // combine the graph's waves (fixed order: integer results, exact anyway)
    __shared__ long long rpos[GP_WAVES], rneg[GP_WAVES], rsm[GP_WAVES];
    __shared__ int rmd[GP_WAVES], rbest[GP_WAVES], rhas[GP_WAVES];
    const int wv = threadIdx.x >> 6;
    if (lane == 0) { rpos[wv] = pos; rneg[wv] = neg; rsm[wv] = sum; rmd[wv] = mdeg; rbest[wv] = best; rhas[wv] = has; }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int k = 1; k < WPG; ++k) {
      pos += rpos[k]; neg += rneg[k]; sum += rsm[k];
      mdeg = max(mdeg, rmd[k]); best = max(best, rbest[k]); has = max(has, rhas[k]);
    }
    if (!live) return;
  }
  if (lane == 0) {
    gs.max_deg[g] = mdeg;
    gs.valid[g] = has;
    double* m = gs.meta + (size_t)g * 4;
    m[0] = has ? (double)best : 1.0;
    const double q = (double)pos / 2.0;  // np.sum(J*(J>0))/2
    m[1] = q > 1.0 ? q : 1.0;            // max(1, .)
    const double lb = (double)neg / 2.0;
    m[2] = lb < 0.0 ? lb : 0.0;          // min(0, .)
    m[3] = (double)sum;
  }
}

// ------------------------------------------------------------- env kernels ----
// time table: tab[k] = running f64 sum of k additions of 1/T (spinsystem.py:493, :506)
__global__ void build_time_table_kernel(uint8_t* state, size_t off_tab, int T) {
  int* hdr = (int*)(state + off_tab);
  if (*hdr == T) return;
  double* tab = (double*)(state + off_tab + 256);
  double v = 0.0;
  const double inc = 1.0 / (double)T;
  tab[0] = 0.0;
  for (int k = 1; k <= T; ++k) { v += inc; tab[k] = v; }
  *hdr = T;
}

template <int VPT>
__device__ __forceinline__ void write_obs(const EnvArgs& a, int e, int lane, const int (&s)[VPT], const int (&h)[VPT],
                                          const int (&tsf)[VPT], const ObsCtx& c) {
  const int N = a.cfg.n_spins;
  const int nobs = a.cfg.n_obs;
  const double* tab = tab_ptr(a);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v >= N) continue;
    float xf[ECO_MAX_OBS];
#pragma unroll
    for (int i = 0; i < ECO_MAX_OBS; ++i) {
      double val = 0.0;
      if (i < nobs) {
        val = obs_value(a.cfg.obs_ids[i], c, s[k], h[k], tsf[k], tab);
        if (a.obs_f64) a.obs_f64[((size_t)e * nobs + i) * N + v] = val;
      }
      xf[i] = (float)val;
    }
    if (a.obs_x) store_obs_row(a.obs_x, (size_t)e * N + v, nobs, xf);
  }
}

// write_obs for DEFAULT_OBSERVABLES (spinsystem.py:486-535 with the ECO training observables, the hot path) and no
// float64 rows: the fp32 feature rows directly.  Per vertex only three values vary -- the spin (basis-mapped), the
// immediate quality change g / mlr and the time since flip -- and the other four are wave-uniform, converted
// once.  g / mlr is the correctly rounded f32 quotient of the two integers (exact in f32: |g|, |mlr| < 2^18),
// which equals the reference's float64 quotient rounded to f32: the exact quotient of integers below 2^18 is
// never within 2^-53 of an f32 rounding midpoint without being one (its distance from any K / 2^j is at least
// 2^-42 relative), so rounding through float64 cannot change the f32 result.  -0.0 is kept (the product is a
// float product: s = -1, h = 0 gives -0.0, as the reference's float64 product does).  tests/test_env_gpu.py
// checks these rows bitwise against the general path.
__device__ __forceinline__ bool obs_default_layout(const eco_env_config& c) {
  return c.n_obs == 7 && c.obs_ids[0] == ECO_OBS_SPIN_STATE && c.obs_ids[1] == ECO_OBS_IMMEDIATE_QUALITY_CHANGE &&
         c.obs_ids[2] == ECO_OBS_TIME_SINCE_FLIP && c.obs_ids[3] == ECO_OBS_DISTANCE_FROM_BEST_SOLUTION &&
         c.obs_ids[4] == ECO_OBS_DISTANCE_FROM_BEST_STATE && c.obs_ids[5] == ECO_OBS_NUMBER_OF_QUALITY_IMPROVEMENTS &&
         c.obs_ids[6] == ECO_OBS_TERMINATION_IMMANENCY;
}
template <int VPT>
__device__ __forceinline__ void write_obs_default(const EnvArgs& a, int e, int lane, const int (&s)[VPT],
                                                  const int (&h)[VPT], const int (&tsf)[VPT], const ObsCtx& c) {
  const int N = a.cfg.n_spins;
  const double* tab = tab_ptr(a);
  const float mlrf = (float)c.mlr;
  const float u3 = (float)c.dist_best, u4 = (float)c.hamming, u5 = (float)c.nqi, u6 = (float)c.term;
  const bool binary = c.basis == ECO_BASIS_BINARY;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v >= N) continue;
    const float sf = (float)s[k];
    const float x0 = binary ? (float)((1 - s[k]) / 2) : sf;  // (1 - s) / 2 is exact: 0 or 1
    const float x1 = __fdiv_rn(sf * (float)h[k], mlrf);
    const float x2 = (float)tab[tsf[k]];
    float4* dst = (float4*)(a.obs_x + ((size_t)e * N + v) * 8);
    dst[0] = make_float4(x0, x1, x2, u3);
    dst[1] = make_float4(u4, u5, u6, 0.f);
  }
}

// SpinSystemBase.reset (spinsystem.py:183-259) + _reset_state (:283-330)
template <int VPT>
__global__ __launch_bounds__(256) void env_reset_kernel(EnvArgs a) {
  extern __shared__ int8_t s_lds[];  // [4 waves][N] spins staged for the J.s matvec
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int e = uniform_i(blockIdx.x * 4 + wv);
  if (e >= a.B) return;
  if (a.mask && !a.mask[e]) return;
  const int N = a.cfg.n_spins;
  const EnvLayout& L = a.L;
  int8_t* my_s = s_lds + wv * N;
  const int gid = uniform_i(a.graph_ids[e]);
  if (gid < 0 || gid >= a.gs.n_graphs || !a.gs.valid[gid]) {
    if (lane == 0) atomicCAS(a.err, 0, ECO_ERR_GRAPH);
    return;
  }
  const double* meta = a.gs.meta + (size_t)gid * 4;
  const double mlr = meta[0], qn = meta[1], lb = meta[2];
  const long long sumJ = (long long)meta[3];
  int s[VPT], h[VPT], g[VPT], tsf[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    int sv = 0;
    if (v < N) {
      if (a.spins_in) {
        sv = a.spins_in[(size_t)e * N + v];
        if (sv != 1 && sv != -1) { atomicCAS(a.err, 0, ECO_ERR_BASIS); sv = -1; }
      } else if (a.cfg.reversible_spins) {
        sv = (int)(rng3(a.seed, (uint64_t)e, (uint64_t)v) >> 63) * 2 - 1;  // 2*randint(2)-1
      } else {
        sv = -1;  // irreversible: all -1 (spinsystem.py:295-297)
      }
      my_s[v] = (int8_t)sv;
    }
    s[k] = sv;
    tsf[k] = 0;
  }
  // each wave reads back only its own LDS slice: a wave-scope fence suffices
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int32_t* rp = a.gs.row_ptr + (size_t)gid * (N + 1);
  const uint32_t* ed = a.gs.edges + a.gs.edge_base[gid];
  long long sg = 0;
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    int hv = 0;
    if (v < N) {
      for (int q = rp[v]; q < rp[v + 1]; ++q) {
        const uint32_t x = ed[q];
        hv += edge_w(x) * (int)my_s[edge_col(x)];
      }
    }
    h[k] = hv;
    g[k] = s[k] * hv;  // calculate_cut_changes: s * (J @ s)
    sg += g[k];
    cnt += (g[k] > 0);
  }
  sg = wave_sum_ll(sg);
  cnt = wave_sum_i(cnt);
  // calculate_cut = 1/4 sum J (1 - s s^T) = (sum J - s.Js)/4, exact integer for integer weights
  const double cut = (double)((sumJ - sg) / 4);
  const double lbabs = lb < 0.0 ? -lb : lb;
  const double score = cut + lbabs;        // MaximizationProblem.get_score (score_solver.py:182-188)
  const double nscore = score / qn;        // get_normalized_score (:190-194)
  int8_t* gsp = (int8_t*)(a.state + L.off_spins) + (size_t)e * N;
  int32_t* gh = (int32_t*)(a.state + L.off_field) + (size_t)e * N;
  int16_t* gt = (int16_t*)(a.state + L.off_tsf) + (size_t)e * N;
  int8_t* gb = (int8_t*)(a.state + L.off_best) + (size_t)e * N;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) { gsp[v] = (int8_t)s[k]; gh[v] = h[k]; gt[v] = 0; gb[v] = (int8_t)s[k]; }
  }
  uint32_t* vidx = (uint32_t*)(a.state + L.off_vidx) + (size_t)e * L.cap;
  for (int i = lane; i < L.cap; i += 64) vidx[i] = 0u;
  if (lane == 0) {
    EpScal* sc = scal_ptr(a) + e;
    sc->score = score; sc->nscore = nscore;
    sc->best_score = score; sc->best_nscore = nscore; sc->best_solution = cut;
    sc->mlr = mlr; sc->qn = qn; sc->lbabs = lbabs;
    sc->hash = 0ull; sc->t = 0; sc->hamming = 0; sc->graph = gid; sc->done = 0; sc->early = 0;
    sc->visit_count = 0;
    sc->inorm = 1.0; sc->lb = lb; sc->inv = 0; sc->best_inv = 0;
  }
  int n1 = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) n1 += __popcll(__ballot(s[k] > 0));
  if (lane == 0) { (scal_ptr(a) + e)->n1 = n1; (scal_ptr(a) + e)->best_n1 = n1; }
  ObsCtx c;
  c.mlr = mlr; c.dist_best = 0.0; c.hamming = 0.0; c.nqi = (double)cnt / (double)N;
  c.term = 0.0; c.ep_time = 0.0; c.basis = a.cfg.spin_basis;
  write_obs<VPT>(a, e, lane, s, h, tsf, c);
}

// Optional per-phase stamps of env_step_kernel (timing build only: make timing; tools/r04/env_timing.py):
// [episode][8] wall_clock64 values, first ECO_ENV_TS_EPS episodes.
#ifdef ECO_PHASE_TIMING
constexpr int ECO_ENV_TS_EPS = 16384;
__device__ unsigned long long eco_env_ts[ECO_ENV_TS_EPS * 8];
#define ECO_ENV_TS(k)                                                                                      \
  do {                                                                                                    \
    if (lane == 0 && e < ECO_ENV_TS_EPS) eco_env_ts[e * 8 + (k)] = wall_clock64();                        \
  } while (0)
#else
#define ECO_ENV_TS(k) \
  do {                \
  } while (0)
#endif

// SpinSystemBase.step (spinsystem.py:355-559), ExtraAction.NONE, memory_length None.
// FASTOBS: DEFAULT_OBSERVABLES, fp32 rows only (write_obs_default).
template <int VPT, bool FASTOBS>
__device__ __forceinline__ void env_step_body(const EnvArgs& a) {
  extern __shared__ int32_t d_lds[];  // [4 waves][N] row deltas
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int e = uniform_i(blockIdx.x * 4 + wv);
  if (e >= a.B) return;
  ECO_ENV_TS(0);
  const int N = a.cfg.n_spins;
  const int T = a.cfg.max_steps;
  const EnvLayout& L = a.L;
  EpScal* sc = scal_ptr(a) + e;
  const int act = uniform_i(a.actions[e]);  // loaded alongside the done flag
  if (sc->done) {  // auto-masked
    if (lane == 0) { a.rewards[e] = 0.0; a.dones[e] = 1; }
    return;
  }
  if (act < 0 || act >= N) {
    if (lane == 0) { atomicCAS(a.err, 0, ECO_ERR_ARG); a.rewards[e] = 0.0; a.dones[e] = 0; }
    return;
  }
  const int t = sc->t + 1;  // :362
  int8_t* gsp = (int8_t*)(a.state + L.off_spins) + (size_t)e * N;
  int32_t* gh = (int32_t*)(a.state + L.off_field) + (size_t)e * N;
  int16_t* gt = (int16_t*)(a.state + L.off_tsf) + (size_t)e * N;
  int8_t* gb = (int8_t*)(a.state + L.off_best) + (size_t)e * N;
  const int gid = sc->graph;
  const int32_t* rp = a.gs.row_ptr + (size_t)gid * (N + 1);
  const uint32_t* ed = a.gs.edges + a.gs.edge_base[gid];
  const int q0 = rp[act], q1 = rp[act + 1];
  int s[VPT], h[VPT], tsf[VPT], bs[VPT], g[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) { s[k] = gsp[v]; h[k] = gh[v]; tsf[k] = gt[v]; bs[k] = gb[v]; }
    else { s[k] = 0; h[k] = 0; tsf[k] = 0; bs[k] = 0; }
  }
  int sa_old, ha;
  read_vertex<VPT>(s, h, act, sa_old, ha);
  ECO_ENV_TS(1);
  const double qn = sc->qn, mlr = sc->mlr;
  const double delta = (double)sa_old * (double)ha;  // f64 product: keeps -0.0 like the reference
  const double delta_n = delta / qn;     // get_normalized_score_mask(state)[action] (:394)
  const double score = sc->score + delta;           // :399
  const double nscore = sc->nscore + delta_n;       // :400 (accumulated)
  // incremental local field: h_j -= 2 w_aj s_a(old) over the CSR row of `act`
  const bool track = a.cfg.has_basin_reward || a.cfg.has_stag_punishment;
  HistProbe hp;
  row_update<VPT>(d_lds + wv * N, ed, q0, q1, N, lane, h, [&](int w) { return -2 * w * sa_old; },
                  [&] { if (track) history_probe(a, e, sc->hash, act, hp); });
  ECO_ENV_TS(2);
  // flip + time-since-flip counters (:397, :492-497)
  int cnt = 0;
  uint64_t words[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v == act) { s[k] = -s[k]; tsf[k] = 0; }
    else if (v < N) { tsf[k] = tsf[k] + 1; }
    g[k] = s[k] * h[k];  // immediate quality / score changes (:414, :416)
    cnt += __popcll(__ballot(g[k] > 0));
    words[k] = __ballot(s[k] > 0);
  }
  const int negs = [&] { int c = 0;
#pragma unroll
    for (int k = 0; k < VPT; ++k) c += __popcll(__ballot(s[k] < 0)); return c; }();
  // HistoryBuffer.update (utils.py:444-464): is the flipped set (== spin configuration) new?
  const bool isnew = track ? history_update_from<VPT>(a, e, lane, sc, hp, words) : true;
  ECO_ENV_TS(3);
  // reward (:418-457)
  double best_score = sc->best_score, best_nscore = sc->best_nscore;
  double rew = 0.0;
  int early = sc->early + 1;
  const bool improved = score > best_score;
  if (improved) {
    early = 0;
    if (a.cfg.reward_signal == ECO_REWARD_BLS)
      rew = a.cfg.norm_rewards ? nscore - best_nscore : score - best_score;
  }
  if (a.cfg.reward_signal == ECO_REWARD_DENSE) rew = a.cfg.norm_rewards ? delta_n : delta;
  if (a.cfg.has_stag_punishment && !isnew) rew -= a.cfg.stag_punishment;
  if (a.cfg.has_basin_reward && cnt == 0 && isnew) rew += a.cfg.basin_reward;
  // best tracking (:459-477)
  double best_solution = sc->best_solution;
  if (improved) {
    best_score = score;
    best_nscore = nscore;
    best_solution = score - sc->lbabs;  // calculate_cut(best_spins), exact for integer weights
#pragma unroll
    for (int k = 0; k < VPT; ++k) bs[k] = s[k];
  }
  int ham = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) ham += __popcll(__ballot(bs[k] != s[k]));
  // termination (:541-556)
  bool done = (t == T);
  if (a.cfg.stopping == ECO_STOP_EARLY && early == 15) done = true;
  if (a.cfg.stopping == ECO_STOP_QUARTER && t == T / 4) done = true;
  if (!a.cfg.reversible_spins && negs == 0) done = true;
  // write back
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) {
      gsp[v] = (int8_t)s[k];
      gh[v] = h[k];
      gt[v] = (int16_t)tsf[k];
      if (improved) gb[v] = (int8_t)bs[k];
    }
  }
  if (lane == 0) {
    sc->score = score; sc->nscore = nscore;
    sc->best_score = best_score; sc->best_nscore = best_nscore; sc->best_solution = best_solution;
    sc->t = t; sc->hamming = ham; sc->done = done ? 1 : 0; sc->early = early;
    a.rewards[e] = rew;
    a.dones[e] = done ? 1 : 0;
  }
  ECO_ENV_TS(4);
  ObsCtx c;
  c.mlr = mlr;
  const double dsc = score - best_score;
  c.dist_best = (dsc < 0.0 ? -dsc : dsc) / mlr;                       // :516-519
  c.hamming = (double)ham;                                            // :526-527
  c.nqi = (double)cnt / (double)N;                                    // :513-514
  const double x = (double)(t - T) / (double)a.cfg.horizon_length + 1.0;
  c.term = x > 0.0 ? x : 0.0;                                         // :509-511
  c.ep_time = tab_ptr(a)[t];                                          // :506
  c.basis = a.cfg.spin_basis;
  if (FASTOBS) write_obs_default<VPT>(a, e, lane, s, h, tsf, c);
  else write_obs<VPT>(a, e, lane, s, h, tsf, c);
  ECO_ENV_TS(5);
}
template <int VPT, bool FASTOBS>
__global__ __launch_bounds__(256) void env_step_kernel(EnvArgs a) {
  env_step_body<VPT, FASTOBS>(a);
}
// The training / bench configuration up to N = 256 at 8 waves per SIMD (<= 64 VGPRs, no spills): all 8192
// ER-200 episodes of a step are resident at once (one wave each) instead of 6144 plus a second round of 2048
// (tools/r04/env_timing.py); above 4 vertices per lane that budget spills, so larger N runs env_step_kernel
template <int VPT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void env_step_fast_kernel(EnvArgs a) {
  env_step_body<VPT, true>(a);
}

// Greedy solver action (src/agents/solver.py:100-131): the vertex with the largest immediate
// cut change g = s * (J s) (first index on ties); an episode whose best change is negative is
// finished (the solver stops, :124-127) and is marked done so later steps leave it unchanged.
// Irreversible envs consider only still-flippable vertices (s == -1, :117-121).
template <int VPT>
__global__ __launch_bounds__(256) void env_greedy_kernel(EnvArgs a, int32_t* actions) {
  const int lane = threadIdx.x & 63;
  const int e = uniform_i(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (e >= a.B) return;
  const int N = a.cfg.n_spins;
  EpScal* sc = scal_ptr(a) + e;
  if (sc->done) {
    if (lane == 0) actions[e] = 0;
    return;
  }
  const int8_t* gsp = (const int8_t*)(a.state + a.L.off_spins) + (size_t)e * N;
  const int32_t* gh = (const int32_t*)(a.state + a.L.off_field) + (size_t)e * N;
  int best = INT_MIN, bi = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) {
      const int s = gsp[v];
      if (a.cfg.reversible_spins || s < 0) {
        const int g = s * gh[v];
        if (g > best || (g == best && v < bi)) { best = g; bi = v; }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int ob = __shfl_xor(best, o, 64), oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) {
    if (best < 0 || bi == 0x7fffffff) {  // no improving (or no allowed) flip: solver stops
      sc->done = 1;
      actions[e] = 0;
    } else {
      actions[e] = bi;
    }
  }
}

// read-out of episode scalars / spins
__global__ void env_read_kernel(EnvArgs a, double* scalars, int8_t* spins, int8_t* best) {
  const int e = blockIdx.x;
  if (e >= a.B) return;
  const int N = a.cfg.n_spins;
  const EpScal* sc = scal_ptr(a) + e;
  if (threadIdx.x == 0 && scalars) {
    double* o = scalars + (size_t)e * ECO_ENV_SCALARS;
    o[0] = sc->t; o[1] = sc->score; o[2] = sc->nscore; o[3] = sc->best_score;
    o[4] = sc->best_nscore; o[5] = sc->best_solution; o[6] = sc->hamming; o[7] = sc->done;
    o[8] = sc->mlr; o[9] = sc->qn; o[10] = sc->inorm > 0.0 ? sc->inorm : 1.0; o[11] = sc->lb;
    o[12] = sc->n1; o[13] = sc->inv; o[14] = sc->graph; o[15] = 0.0;
  }
  const int8_t* gsp = (const int8_t*)(a.state + a.L.off_spins) + (size_t)e * N;
  const int8_t* gb = (const int8_t*)(a.state + a.L.off_best) + (size_t)e * N;
  for (int v = threadIdx.x; v < N; v += blockDim.x) {
    if (spins) spins[(size_t)e * N + v] = gsp[v];
    if (best) best[(size_t)e * N + v] = gb[v];
  }
}

// ------------------------------------------------------------------ host ----
static int validate_cfg(const eco_env_config* c) {
  if (!c) return fail(ECO_ERR_ARG, "null env config");
  if (c->n_spins < 1 || c->n_spins > ECO_MAX_SPINS)
    return fail(ECO_ERR_ARG, "n_spins out of range [1, " + std::to_string(ECO_MAX_SPINS) + "]");
  if (c->max_steps < 1 || c->max_steps > 32767) return fail(ECO_ERR_ARG, "max_steps out of range [1, 32767]");
  if (c->n_obs < 1 || c->n_obs > 13) return fail(ECO_ERR_ARG, "n_obs out of range [1, 13]");
  if (c->obs_ids[0] != ECO_OBS_SPIN_STATE)
    return fail(ECO_ERR_OBSERVABLE, "First observable must be Observation.SPIN_STATE.");
  const int t = c->optimisation_target;
  if (t < ECO_TARGET_CUT || t > ECO_TARGET_MIN_DOM_SET || t == ECO_TARGET_ENERGY)
    return fail(ECO_ERR_TARGET, "Invalid optimization target: " + std::to_string(t) + " and biased False");
  for (int i = 0; i < c->n_obs; ++i) {
    const int id = c->obs_ids[i];
    if (id < 1 || id > 13) return fail(ECO_ERR_ARG, "unknown observable id");
    if ((t == ECO_TARGET_CUT || t == ECO_TARGET_MIN_CUT) &&
        (id == ECO_OBS_IMMEDIATE_VALIDITY_DIFFERENCE || id == ECO_OBS_IMMEDIATE_VALIDITY_CHANGE ||
         id == ECO_OBS_NUMBER_OF_VALIDITY_IMPROVEMENTS))
      return fail(ECO_ERR_OBSERVABLE, "validity-mask observables are undefined for cut targets (the "
                                      "reference's scorer returns a list: TypeError)");
  }
  if (c->spin_basis != ECO_BASIS_SIGNED && c->spin_basis != ECO_BASIS_BINARY)
    return fail(ECO_ERR_BASIS, "Unrecognised SpinBasis");
  if (c->horizon_length < 1) return fail(ECO_ERR_ARG, "horizon_length must be >= 1");
  return ECO_OK;
}

static int validate_gs(const eco_graph_set* gs, int N) {
  if (!gs || !gs->row_ptr || !gs->edge_base || !gs->edges || !gs->deg || !gs->max_deg || !gs->meta || !gs->valid)
    return fail(ECO_ERR_ARG, "incomplete graph set");
  if (gs->n_spins != N) return fail(ECO_ERR_ARG, "graph set n_spins does not match the env");
  if (gs->n_graphs < 1) return fail(ECO_ERR_ARG, "empty graph set");
  return ECO_OK;
}

int32_t* err_word() {
  static int32_t* w = nullptr;  // one device word per process (read back after each call)
  if (!w) {
    if (hipMalloc(&w, sizeof(int32_t)) != hipSuccess) return nullptr;
    (void)hipMemset(w, 0, sizeof(int32_t));
  }
  return w;
}

static int check_err_word(int32_t* w, hipStream_t st) {
  int32_t h = 0;
  if (hipMemcpyAsync(&h, w, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(ECO_ERR_HIP, "error-word readback failed");
  if (h != 0) {
    (void)hipMemsetAsync(w, 0, sizeof(int32_t), st);
    (void)hipStreamSynchronize(st);
    switch (h) {
      case ECO_ERR_GRAPH: return fail(h, "graph has no nonzero local reward (empty graph) or bad graph id");
      case ECO_ERR_BASIS: return fail(h, "SpinSystem is configured for signed spins ([-1,1]).");
      case ECO_ERR_ARG: return fail(h, "action out of range [0, n_spins)");
      default: return fail(h, "device error");
    }
  }
  return ECO_OK;
}

static inline bool generic_target(const eco_env_config* c) { return c->optimisation_target != ECO_TARGET_CUT; }

}  // namespace eco

using namespace eco;

int eco::graphs_prepare_range(eco_graph_set* gs, int first, int count, hipStream_t st) {
  if (!gs || !gs->row_ptr || !gs->edge_base || !gs->edges || !gs->deg || !gs->max_deg || !gs->meta || !gs->valid)
    return fail(ECO_ERR_ARG, "incomplete graph set");
  if (gs->n_graphs < 1 || gs->n_spins < 1) return fail(ECO_ERR_ARG, "empty graph set");
  if (first < 0 || count < 1 || first + count > gs->n_graphs) return fail(ECO_ERR_ARG, "graph range out of set");
  if (gs->n_spins <= 512) {
    const size_t lds = (size_t)GP_WAVES * (3 * gs->n_spins + 1) * sizeof(int);
    (void)hipFuncSetAttribute((const void*)graphs_prepare_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    graphs_prepare_kernel<1><<<(count + GP_WAVES - 1) / GP_WAVES, 64 * GP_WAVES, lds, st>>>(*gs, first, count);
  } else {
    // one workgroup per graph holds row pointers, row sums and nonzero counts in LDS: 12 B per vertex,
    // so the graph set may have at most 160 KB / 12 B = 13,653 vertices (every env kernel stops at
    // ECO_MAX_SPINS = 2048 anyway); larger sets are rejected here rather than failing at launch
    const size_t lds = (size_t)(3 * gs->n_spins + 1) * sizeof(int);
    if (lds > (size_t)160 * 1024)
      return fail(ECO_ERR_ARG, "graphs_prepare: n_spins = " + std::to_string(gs->n_spins) +
                                   " needs " + std::to_string(lds) + " B of LDS (> 160 KB): at most 13653 vertices");
    if (hipFuncSetAttribute((const void*)graphs_prepare_kernel<GP_WAVES>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return fail(ECO_ERR_HIP, "graphs_prepare: cannot raise the dynamic LDS limit");
    graphs_prepare_kernel<GP_WAVES><<<count, 64 * GP_WAVES, lds, st>>>(*gs, first, count);
  }
  int rc = check_launch("graphs_prepare");
  if (rc) return rc;
  if (gs->adjbits && gs->unit_weights && adjbits_applies(gs->n_spins)) return adjbits_build(gs, first, count, st);
  return ECO_OK;
}

extern "C" int eco_graphs_prepare(eco_graph_set* gs, eco_stream_t stream) {
  if (!gs) return fail(ECO_ERR_ARG, "incomplete graph set");
  return graphs_prepare_range(gs, 0, gs->n_graphs, (hipStream_t)stream);
}

extern "C" size_t eco_graphs_adjbits_bytes(int32_t n_spins, int32_t n_graphs) {
  if (n_graphs < 1 || !adjbits_applies(n_spins)) return 0;
  return (size_t)n_graphs * n_spins * adjbits_words_per_node(n_spins) * 4;
}

extern "C" size_t eco_env_state_bytes(const eco_env_config* cfg, int32_t batch) {
  if (validate_cfg(cfg) != ECO_OK || batch < 1) return 0;
  return env_layout(cfg->n_spins, cfg->max_steps, batch).total;
}

static int make_args(EnvArgs& a, const eco_env_config* cfg, const eco_graph_set* gs, void* state, int32_t batch) {
  int rc = validate_cfg(cfg);
  if (rc) return rc;
  if (gs) { rc = validate_gs(gs, cfg->n_spins); if (rc) return rc; }
  if (!state) return fail(ECO_ERR_ARG, "null state");
  if (batch < 1) return fail(ECO_ERR_ARG, "batch must be >= 1");
  a = EnvArgs{};
  a.cfg = *cfg;
  if (gs) a.gs = *gs;
  a.L = env_layout(cfg->n_spins, cfg->max_steps, batch);
  a.state = (uint8_t*)state;
  a.B = batch;
  a.err = err_word();
  if (!a.err) return fail(ECO_ERR_HIP, "cannot allocate error word");
  return ECO_OK;
}

extern "C" int eco_env_reset(const eco_env_config* cfg, const eco_graph_set* gs, void* state, int32_t batch,
                             const int32_t* graph_ids, const int8_t* spins, const uint8_t* reset_mask, uint64_t seed,
                             float* obs_x, double* obs_f64, eco_stream_t stream) {
  EnvArgs a;
  int rc = make_args(a, cfg, gs, state, batch);
  if (rc) return rc;
  if (!gs) return fail(ECO_ERR_ARG, "null graph set");
  if (!graph_ids) return fail(ECO_ERR_ARG, "null graph_ids");
  a.graph_ids = graph_ids; a.spins_in = spins; a.mask = reset_mask; a.seed = seed;
  a.obs_x = obs_x; a.obs_f64 = obs_f64;
  hipStream_t st = (hipStream_t)stream;
  build_time_table_kernel<<<1, 1, 0, st>>>(a.state, a.L.off_tab, cfg->max_steps);
  const int blocks = (batch + 3) / 4;
  const size_t lds = (size_t)4 * cfg->n_spins;
  if (generic_target(cfg)) return env_reset_problem_launch(a, blocks, lds, st);
  ECO_DISPATCH_VPT(cfg->n_spins, (env_reset_kernel<V><<<blocks, 256, lds, st>>>(a)));
  return check_launch("env_reset");
}

#ifdef ECO_PHASE_TIMING
extern "C" int eco_debug_env_ts(unsigned long long* host, int32_t n) {
  if (n > ECO_ENV_TS_EPS * 8) n = ECO_ENV_TS_EPS * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(eco_env_ts), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int eco_check_errors(eco_stream_t stream) {
  int32_t* w = err_word();
  if (!w) return fail(ECO_ERR_HIP, "cannot allocate error word");
  return check_err_word(w, (hipStream_t)stream);
}

extern "C" int eco_error_word_copy(int32_t* dst, eco_stream_t stream) {
  int32_t* w = err_word();
  if (!w) return fail(ECO_ERR_HIP, "cannot allocate error word");
  if (!dst) return fail(ECO_ERR_ARG, "null destination");
  if (hipMemcpyAsync(dst, w, sizeof(int32_t), hipMemcpyDefault, (hipStream_t)stream) != hipSuccess)
    return fail(ECO_ERR_HIP, "error-word copy failed");
  return ECO_OK;
}

extern "C" int eco_env_step(const eco_env_config* cfg, const eco_graph_set* gs, void* state, int32_t batch,
                            const int32_t* actions, double* rewards, uint8_t* dones, float* obs_x, double* obs_f64,
                            eco_stream_t stream) {
  EnvArgs a;
  int rc = make_args(a, cfg, gs, state, batch);
  if (rc) return rc;
  if (!gs) return fail(ECO_ERR_ARG, "null graph set");
  if (!actions || !rewards || !dones) return fail(ECO_ERR_ARG, "null actions/rewards/dones");
  a.actions = actions; a.rewards = rewards; a.dones = dones; a.obs_x = obs_x; a.obs_f64 = obs_f64;
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (batch + 3) / 4;
  if (generic_target(cfg)) return env_step_problem_launch(a, blocks, env_step_lds(cfg->n_spins), st);
  // the DEFAULT_OBSERVABLES fp32-only path (the training / bench configuration) or the general one
  const bool fast = !obs_f64 && obs_x && cfg->n_obs == 7 && cfg->obs_ids[0] == ECO_OBS_SPIN_STATE &&
                    cfg->obs_ids[1] == ECO_OBS_IMMEDIATE_QUALITY_CHANGE && cfg->obs_ids[2] == ECO_OBS_TIME_SINCE_FLIP &&
                    cfg->obs_ids[3] == ECO_OBS_DISTANCE_FROM_BEST_SOLUTION &&
                    cfg->obs_ids[4] == ECO_OBS_DISTANCE_FROM_BEST_STATE &&
                    cfg->obs_ids[5] == ECO_OBS_NUMBER_OF_QUALITY_IMPROVEMENTS &&
                    cfg->obs_ids[6] == ECO_OBS_TERMINATION_IMMANENCY;
  const size_t lds = (size_t)16 * cfg->n_spins;
  if (fast && cfg->n_spins <= 64) env_step_fast_kernel<1><<<blocks, 256, lds, st>>>(a);
  else if (fast && cfg->n_spins <= 128) env_step_fast_kernel<2><<<blocks, 256, lds, st>>>(a);
  else if (fast && cfg->n_spins <= 256) env_step_fast_kernel<4><<<blocks, 256, lds, st>>>(a);
  else if (fast) ECO_DISPATCH_VPT(cfg->n_spins, (env_step_kernel<V, true><<<blocks, 256, lds, st>>>(a)));
  else ECO_DISPATCH_VPT(cfg->n_spins, (env_step_kernel<V, false><<<blocks, 256, lds, st>>>(a)));
  return check_launch("env_step");
}

extern "C" int eco_env_greedy_actions(const eco_env_config* cfg, const eco_graph_set* gs, void* state,
                                      int32_t batch, int32_t* actions, eco_stream_t stream) {
  EnvArgs a;
  int rc = make_args(a, cfg, gs, state, batch);
  if (rc) return rc;
  if (!actions) return fail(ECO_ERR_ARG, "null actions");
  if (cfg->optimisation_target == ECO_TARGET_MIN_DOM_SET && !gs)
    return fail(ECO_ERR_ARG, "MIN_DOM_SET greedy actions need the graph set");
  const int blocks = (batch + 3) / 4;
  hipStream_t st = (hipStream_t)stream;
  if (generic_target(cfg)) return env_greedy_problem_launch(a, actions, blocks, (size_t)4 * cfg->n_spins, st);
  ECO_DISPATCH_VPT(cfg->n_spins, (env_greedy_kernel<V><<<blocks, 256, 0, st>>>(a, actions)));
  return check_launch("env_greedy");
}

extern "C" int eco_env_read(const eco_env_config* cfg, const void* state, int32_t batch, double* scalars,
                            int8_t* spins, int8_t* best_spins, eco_stream_t stream) {
  EnvArgs a;
  int rc = make_args(a, cfg, nullptr, (void*)state, batch);
  if (rc) return rc;
  env_read_kernel<<<batch, 256, 0, (hipStream_t)stream>>>(a, scalars, spins, best_spins);
  return check_launch("env_read");
}
