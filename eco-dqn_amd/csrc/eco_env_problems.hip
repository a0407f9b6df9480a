// Generic-scorer SpinSystem kernels: OptimisationTarget MIN_COVER, MIN_CUT, MAX_IND_SET, MAX_CLIQUE,
// MIN_DOM_SET (src/envs/score_solver.py:232-858) with all 13 observables; same wave-per-episode
// layout as the MaxCut kernels of eco_env.hip.
//
// The reference recomputes every scorer mask densely per step (MinDomSet and MaxClique loop over all
// N flips, each an O(N^2) recount, score_solver.py:692-700, :806-817).  Here each vertex keeps one
// integer neighbour sum F_i, updated along ONE CSR row per flip, and the masks follow in O(1)
// (MinDomSet: one neighbour pass over the row of each vertex):
//
//   target        F_i (x = [s == +1])          quality mask qm_i   invalidity mask im_i
//   MIN_COVER     U_i = sum_j J_ij (1 - x_j)   s_i                 s_i U_i
//   MAX_IND_SET   A_i = sum_j J_ij x_j         -s_i                -s_i A_i
//   MAX_CLIQUE    A_i                          -s_i                x_i ? 2 (A_i - n1 + 1) : 2 (n1 - A_i)
//   MIN_DOM_SET   P_i = sum_j [J_ij > 0] x_j   s_i                 x_i ? [P_i = 0] + S1_i : -[P_i = 0] - S0_i
//   MIN_CUT       h_i = sum_j J_ij s_j         -s_i h_i            0 (no invalidity)
//
// S0_i / S1_i count the positive-weight neighbours k of i with x_k = 0 and P_k = 0 / 1 (vertices a
// flip of i would dominate / leave undominated).  Flipping a changes F_j by coef(J_ja) * s_a(old):
// -2w (h), +w (U), -w (A), -[w > 0] (P).  Scores, masks and observations are then evaluated with the
// reference's float64 operations (MaximizationProblem / MinimizationProblem, :175-229; the generic
// get_score_mask / get_normalized_score_mask, :310-339), so they equal the reference's values.

#include "eco_env_dev.h"

namespace eco {

__device__ __forceinline__ bool target_maximises(int t) {
  return t == ECO_TARGET_MAX_IND_SET || t == ECO_TARGET_MAX_CLIQUE;
}

__device__ __forceinline__ int field_coef(int t, int w) {
  switch (t) {
    case ECO_TARGET_MIN_CUT: return -2 * w;
    case ECO_TARGET_MIN_COVER: return w;
    case ECO_TARGET_MIN_DOM_SET: return w > 0 ? -1 : 0;
    default: return -w;
  }
}

// per-vertex quality / invalidity masks (table above)
__device__ __forceinline__ void vertex_masks(int t, int s, int F, int n1, int S0, int S1, int& qm, int& im) {
  switch (t) {
    case ECO_TARGET_MIN_COVER: qm = s; im = s * F; break;
    case ECO_TARGET_MAX_IND_SET: qm = -s; im = -s * F; break;
    case ECO_TARGET_MAX_CLIQUE: qm = -s; im = s > 0 ? 2 * (F - n1 + 1) : 2 * (n1 - F); break;
    case ECO_TARGET_MIN_DOM_SET: {
      const int alone = F == 0;
      qm = s; im = s > 0 ? alone + S1 : -alone - S0;
      break;
    }
    default: qm = -s * F; im = 0; break;  // MIN_CUT
  }
}

// solution quality (score_solver.py:196-200 / :224-228) of a set of size n1: measure n1, lower bound 0,
// quality normaliser N
__device__ __forceinline__ int set_quality(int t, int n1, int N) { return target_maximises(t) ? n1 : N - n1; }

// MinDomSet neighbour codes: bit0 = (x=0, P=0), bit1 = (x=0, P=1)
__device__ __forceinline__ uint8_t mds_code(int s, int F) {
  return s < 0 ? (uint8_t)((F == 0) | ((F == 1) << 1)) : (uint8_t)0;
}

// S0/S1 of the wave's own vertices from the codes of the whole episode in LDS (one CSR pass)
template <int VPT>
__device__ __forceinline__ void mds_neighbour_counts(const int32_t* rp, const uint32_t* ed, const uint8_t* code,
                                                     int N, int lane, int (&S0)[VPT], int (&S1)[VPT]) {
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    int a0 = 0, a1 = 0;
    if (v < N) {
      const int q1 = rp[v + 1];
      int q = rp[v];
      for (; q + 4 <= q1; q += 4) {  // four independent edge loads in flight
        uint32_t x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = ed[q + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint8_t c = edge_w(x[u]) > 0 ? code[edge_col(x[u])] : (uint8_t)0;
          a0 += c & 1;
          a1 += c >> 1;
        }
      }
      for (; q < q1; ++q) {
        const uint32_t x = ed[q];
        const uint8_t c = edge_w(x) > 0 ? code[edge_col(x)] : (uint8_t)0;
        a0 += c & 1;
        a1 += c >> 1;
      }
    }
    S0[k] = a0;
    S1[k] = a1;
  }
}

// Episode quantities an observation row needs beyond the per-vertex masks.
struct ProbObs {
  double mlr, inorm, dist_best, hamming, nqi, nvi, term, ep_time, gvd, valid;
  int basis;
};

__device__ __forceinline__ double prob_obs_value(int id, const ProbObs& c, int s, int qm, int im, int vm, int tsfk,
                                                 const double* tab, bool cut_like) {
  switch (id) {
    case ECO_OBS_SPIN_STATE: return c.basis == ECO_BASIS_BINARY ? (double)(1 - s) / 2.0 : (double)s;
    case ECO_OBS_IMMEDIATE_QUALITY_CHANGE:
      // MIN_CUT: -(s * (J s)) in f64 (a zero product keeps its sign through the negation)
      return (cut_like ? -((double)s * (double)(-qm * s)) : (double)qm) / c.mlr;
    case ECO_OBS_IMMEDIATE_VALIDITY_DIFFERENCE: return (double)im / c.inorm;
    case ECO_OBS_IMMEDIATE_VALIDITY_CHANGE: return vm ? 1.0 : 0.0;
    case ECO_OBS_TIME_SINCE_FLIP: return tab[tsfk];
    case ECO_OBS_EPISODE_TIME: return c.ep_time;
    case ECO_OBS_TERMINATION_IMMANENCY: return c.term;
    case ECO_OBS_NUMBER_OF_QUALITY_IMPROVEMENTS: return c.nqi;
    case ECO_OBS_NUMBER_OF_VALIDITY_IMPROVEMENTS: return c.nvi;
    case ECO_OBS_DISTANCE_FROM_BEST_SOLUTION: return c.dist_best;
    case ECO_OBS_DISTANCE_FROM_BEST_STATE: return c.hamming;
    case ECO_OBS_GLOBAL_VALIDITY_DIFFERENCE: return c.gvd;
    default: return c.valid;  // ECO_OBS_VALIDITY_BIT
  }
}

template <int VPT>
__device__ __forceinline__ void write_prob_obs(const EnvArgs& a, int e, int lane, const int (&s)[VPT],
                                               const int (&qm)[VPT], const int (&im)[VPT], const int (&vm)[VPT],
                                               const int (&tsf)[VPT], const ProbObs& c, bool cut_like) {
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
        val = prob_obs_value(a.cfg.obs_ids[i], c, s[k], qm[k], im[k], vm[k], tsf[k], tab, cut_like);
        if (a.obs_f64) a.obs_f64[((size_t)e * nobs + i) * N + v] = val;
      }
      xf[i] = (float)val;
    }
    if (a.obs_x) store_obs_row(a.obs_x, (size_t)e * N + v, nobs, xf);
  }
}

// SpinSystemBase.reset (spinsystem.py:183-259) + _reset_state (:283-330) for the generic scorers.
template <int VPT>
__global__ __launch_bounds__(256) void env_reset_problem_kernel(EnvArgs a) {
  extern __shared__ int8_t s_lds[];  // [4 waves][N]: spins, then MinDomSet codes
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int e = uniform_i(blockIdx.x * 4 + wv);
  if (e >= a.B) return;
  if (a.mask && !a.mask[e]) return;
  const int N = a.cfg.n_spins;
  const int tgt = a.cfg.optimisation_target;
  const bool cut_like = tgt == ECO_TARGET_MIN_CUT;
  const EnvLayout& L = a.L;
  int8_t* my_s = s_lds + wv * N;
  const int gid = uniform_i(a.graph_ids[e]);
  // only a cut scorer can see an all-zero local reward mask (the redraw loop, :203-211); the set
  // problems' masks are nonzero on every graph
  if (gid < 0 || gid >= a.gs.n_graphs || (cut_like && !a.gs.valid[gid])) {
    if (lane == 0) atomicCAS(a.err, 0, ECO_ERR_GRAPH);
    return;
  }
  int s[VPT], F[VPT], tsf[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    int sv = 0;
    if (v < N) {
      if (a.spins_in) {
        sv = a.spins_in[(size_t)e * N + v];
        if (sv != 1 && sv != -1) { atomicCAS(a.err, 0, ECO_ERR_BASIS); sv = -1; }
      } else if (a.cfg.reversible_spins) {
        sv = (int)(rng3(a.seed, (uint64_t)e, (uint64_t)v) >> 63) * 2 - 1;
      } else {
        sv = -1;
      }
      my_s[v] = (int8_t)sv;
    }
    s[k] = sv;
    tsf[k] = 0;
  }
  wave_lds_sync();
  const int32_t* rp = a.gs.row_ptr + (size_t)gid * (N + 1);
  const uint32_t* ed = a.gs.edges + a.gs.edge_base[gid];
  long long sumJ = 0, negJ = 0, sx = 0;  // sum J, sum J*(J<0), and sum_i s_i h_i (MIN_CUT) / x_i A_i
  int maxD = INT_MIN, mlr_cut = INT_MIN, inv_part = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    int f = 0;
    if (v < N) {
      int D = 0, h = 0, A = 0, P = 0;
      for (int q = rp[v]; q < rp[v + 1]; ++q) {
        const uint32_t x = ed[q];
        const int w = edge_w(x);
        const int sk = my_s[edge_col(x)];
        D += w;
        h += w * sk;
        if (sk > 0) { A += w; P += w > 0; }
        if (w < 0) negJ += w;
      }
      sumJ += D;
      maxD = max(maxD, D);
      if (D != 0) mlr_cut = max(mlr_cut, -D);  // MIN_CUT: quality mask at s = -1 is -D (:445-453)
      switch (tgt) {
        case ECO_TARGET_MIN_CUT: f = h; sx += (long long)s[k] * h; break;
        case ECO_TARGET_MIN_COVER: f = D - A; if (s[k] < 0) inv_part += f; break;
        case ECO_TARGET_MIN_DOM_SET: f = P; inv_part += (s[k] < 0 && P == 0); break;
        default: f = A; if (s[k] > 0) { sx += A; } break;  // MAX_IND_SET / MAX_CLIQUE
      }
    }
    F[k] = f;
  }
  sumJ = wave_sum_ll(sumJ);
  negJ = wave_sum_ll(negJ);
  sx = wave_sum_ll(sx);
  inv_part = wave_sum_i(inv_part);
  maxD = wave_max_i(maxD);
  mlr_cut = wave_max_i(mlr_cut);
  int n1 = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) n1 += __popcll(__ballot(s[k] > 0));
  // scorer constants (set_max_local_reward before _reset_state; the others after, :213-221)
  double mlr, qn, inorm, lb = 0.0;
  int inv = 0;
  switch (tgt) {
    case ECO_TARGET_MIN_CUT: {
      mlr = (double)mlr_cut;
      const double an = fabs((double)negJ);
      qn = an > 1.0 ? an : 1.0;                              // :439-443
      inorm = 1.0;
      const double h = (double)negJ / 2.0;
      lb = h < 0.0 ? h : 0.0;                                // :455-461
      break;
    }
    case ECO_TARGET_MIN_COVER:
    case ECO_TARGET_MAX_IND_SET:
      mlr = (double)N + (double)maxD;                        // :236-244, :519-523
      qn = (double)N;
      inorm = (double)sumJ / 2.0;                            // :246-252, :513-517
      inv = tgt == ECO_TARGET_MIN_COVER ? inv_part / 2 : (int)(sx / 2);
      break;
    case ECO_TARGET_MAX_CLIQUE:
      mlr = (double)N;
      qn = (double)N;
      inorm = (double)sumJ;                                  // :763-768
      inv = n1 * (n1 - 1) - (int)sx;
      break;
    default:  // MIN_DOM_SET
      mlr = 2.0 * (double)N;
      qn = (double)N;
      inorm = (double)N;
      inv = inv_part;
      break;
  }
  EpScal* sc = scal_ptr(a) + e;
  const double stale_inorm = sc->inorm > 0.0 ? sc->inorm : 1.0;  // normaliser of the previous reset
  int S0[VPT], S1[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) { S0[k] = 0; S1[k] = 0; }
  if (tgt == ECO_TARGET_MIN_DOM_SET) {
    uint8_t* code = (uint8_t*)my_s;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int v = lane + 64 * k;
      if (v < N) code[v] = mds_code(s[k], F[k]);
    }
    wave_lds_sync();
    mds_neighbour_counts<VPT>(rp, ed, code, N, lane, S0, S1);
  }
  int qm[VPT], im[VPT], vm[VPT];
  int nqi = 0, nvi = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    vertex_masks(tgt, s[k], F[k], n1, S0[k], S1[k], qm[k], im[k]);
    vm[k] = (inv + im[k]) == 0;
    nqi += __popcll(__ballot(v < N && qm[k] > 0));
    nvi += __popcll(__ballot(v < N && im[k] > 0));  // '> 0' at reset (:324-325)
  }
  // score / normalized score / solution of the initial spins (:224-226)
  double score, nscore, solution;
  if (cut_like) {
    const double cut = (double)((sumJ - sx) / 4);
    const double q = (qn > 0.0 ? qn : 0.0) - cut;            // max(0, qn) - measure
    score = q;
    nscore = q / qn - 0.0;
    solution = cut;
  } else {
    const int q = set_quality(tgt, n1, N);
    const bool valid = inv == 0;
    score = (double)(valid ? q : 0) - (double)inv;
    nscore = (double)(valid ? q : 0) / qn - (double)inv / inorm;
    solution = valid ? (double)n1 : (target_maximises(tgt) ? 0.0 : (double)N);
  }
  int8_t* gsp = (int8_t*)(a.state + L.off_spins) + (size_t)e * N;
  int32_t* gF = (int32_t*)(a.state + L.off_field) + (size_t)e * N;
  int16_t* gt = (int16_t*)(a.state + L.off_tsf) + (size_t)e * N;
  int8_t* gb = (int8_t*)(a.state + L.off_best) + (size_t)e * N;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) { gsp[v] = (int8_t)s[k]; gF[v] = F[k]; gt[v] = 0; gb[v] = (int8_t)s[k]; }
  }
  uint32_t* vidx = (uint32_t*)(a.state + L.off_vidx) + (size_t)e * L.cap;
  for (int i = lane; i < L.cap; i += 64) vidx[i] = 0u;
  if (lane == 0) {
    sc->score = score; sc->nscore = nscore;
    sc->best_score = score; sc->best_nscore = nscore; sc->best_solution = solution;
    sc->mlr = mlr; sc->qn = qn; sc->lbabs = lb < 0.0 ? -lb : lb;
    sc->hash = 0ull; sc->t = 0; sc->hamming = 0; sc->graph = gid; sc->done = 0; sc->early = 0;
    sc->visit_count = 0;
    sc->inorm = inorm; sc->lb = lb;
    sc->n1 = n1; sc->inv = inv; sc->best_n1 = n1; sc->best_inv = inv;
  }
  ProbObs c;
  c.mlr = mlr; c.inorm = stale_inorm;
  c.dist_best = 0.0; c.hamming = 0.0; c.term = 0.0; c.ep_time = 0.0; c.gvd = 0.0;
  c.nqi = (double)nqi / (double)N;
  c.nvi = (double)nvi / (double)N;
  c.valid = inv == 0 ? 1.0 : 0.0;
  c.basis = a.cfg.spin_basis;
  write_prob_obs<VPT>(a, e, lane, s, qm, im, vm, tsf, c, cut_like);
}

// Score-mask deltas of flipping vertex `act` (spinsystem.py:393-394) from the pre-flip state.
struct FlipDelta { double d, dn; int im; };

__device__ __forceinline__ FlipDelta flip_delta(int tgt, int sa, int Fa, int n1, int inv, int S0a, int S1a, int N,
                                                double qn, double inorm) {
  FlipDelta r;
  int qm, im;
  vertex_masks(tgt, sa, Fa, n1, S0a, S1a, qm, im);
  r.im = im;
  if (tgt == ECO_TARGET_MIN_CUT) {  // score mask = quality mask = -(s * (J s)); normalized: / qn (:495-505)
    const double q = -((double)sa * (double)Fa);
    r.d = q;
    r.dn = q / qn;
    return r;
  }
  const int q = set_quality(tgt, n1, N);
  const bool valid = inv == 0;
  const double score = (double)(valid ? q : 0) - (double)inv;
  const double nscore = (double)(valid ? q : 0) / qn - (double)inv / inorm;
  const int uq = q + qm, ui = inv + im;
  const bool vm = ui == 0;
  r.d = (vm ? (double)uq : 0.0) - (double)ui - score;              // :316-324
  const double uqn = (double)uq / qn;
  r.dn = (vm ? uqn : 0.0 * uqn) - (double)ui / inorm - nscore;      // :331-339
  return r;
}

// SpinSystemBase.step (spinsystem.py:355-559) for the generic scorers.
template <int VPT>
__global__ __launch_bounds__(256) void env_step_problem_kernel(EnvArgs a) {
  extern __shared__ int32_t d_lds[];  // [4 waves][N] row deltas, then [4 waves][N] MinDomSet codes
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int e = uniform_i(blockIdx.x * 4 + wv);
  if (e >= a.B) return;
  const int N = a.cfg.n_spins;
  const int T = a.cfg.max_steps;
  const int tgt = a.cfg.optimisation_target;
  const bool cut_like = tgt == ECO_TARGET_MIN_CUT;
  const EnvLayout& L = a.L;
  uint8_t* c_lds = reinterpret_cast<uint8_t*>(d_lds + 4 * N);
  EpScal* sc = scal_ptr(a) + e;
  const int act = uniform_i(a.actions[e]);  // loaded alongside the done flag
  if (sc->done) {
    if (lane == 0) { a.rewards[e] = 0.0; a.dones[e] = 1; }
    return;
  }
  if (act < 0 || act >= N) {
    if (lane == 0) { atomicCAS(a.err, 0, ECO_ERR_ARG); a.rewards[e] = 0.0; a.dones[e] = 0; }
    return;
  }
  const int t = sc->t + 1;
  int8_t* gsp = (int8_t*)(a.state + L.off_spins) + (size_t)e * N;
  int32_t* gF = (int32_t*)(a.state + L.off_field) + (size_t)e * N;
  int16_t* gt = (int16_t*)(a.state + L.off_tsf) + (size_t)e * N;
  int8_t* gb = (int8_t*)(a.state + L.off_best) + (size_t)e * N;
  const int gid = sc->graph;
  const int32_t* rp = a.gs.row_ptr + (size_t)gid * (N + 1);
  const uint32_t* ed = a.gs.edges + a.gs.edge_base[gid];
  int s[VPT], F[VPT], tsf[VPT], bs[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) { s[k] = gsp[v]; F[k] = gF[v]; tsf[k] = gt[v]; bs[k] = gb[v]; }
    else { s[k] = 0; F[k] = 0; tsf[k] = 0; bs[k] = 0; }
  }
  int sa_old, Fa;
  read_vertex<VPT>(s, F, act, sa_old, Fa);
  const int n1_old = sc->n1, inv_old = sc->inv;
  const double qn = sc->qn, mlr = sc->mlr, inorm = sc->inorm;
  // MinDomSet: the action's neighbour counts from the pre-flip state (lanes split its row)
  int S0a = 0, S1a = 0;
  if (tgt == ECO_TARGET_MIN_DOM_SET) {
    for (int q = rp[act] + lane; q < rp[act + 1]; q += 64) {
      const uint32_t x = ed[q];
      if (edge_w(x) > 0) {
        const int k = edge_col(x);
        const uint8_t c = mds_code(gsp[k], gF[k]);
        S0a += c & 1;
        S1a += c >> 1;
      }
    }
    S0a = wave_sum_i(S0a);
    S1a = wave_sum_i(S1a);
  }
  const FlipDelta fd = flip_delta(tgt, sa_old, Fa, n1_old, inv_old, S0a, S1a, N, qn, inorm);
  const double score = sc->score + fd.d;       // :399
  const double nscore = sc->nscore + fd.dn;    // :400 (accumulated)
  // neighbour sums along the row of `act`
  row_update<VPT>(d_lds + wv * N, ed, rp[act], rp[act + 1], N, lane, F,
                  [&](int w) { return field_coef(tgt, w) * sa_old; });
  uint64_t words[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v == act) { s[k] = -s[k]; tsf[k] = 0; }
    else if (v < N) { tsf[k] = tsf[k] + 1; }
    words[k] = __ballot(s[k] > 0);
  }
  const int n1 = n1_old - sa_old;
  const int inv = cut_like ? 0 : inv_old + fd.im;
  int S0[VPT], S1[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) { S0[k] = 0; S1[k] = 0; }
  if (tgt == ECO_TARGET_MIN_DOM_SET) {
    uint8_t* code = c_lds + wv * N;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int v = lane + 64 * k;
      if (v < N) code[v] = mds_code(s[k], F[k]);
    }
    wave_lds_sync();
    mds_neighbour_counts<VPT>(rp, ed, code, N, lane, S0, S1);
  }
  // masks of the new state (:414-416); the score mask is recomputed from it (integer-valued)
  const int q_new = cut_like ? 0 : set_quality(tgt, n1, N);
  const bool valid = inv == 0;
  const int score_fresh = (valid ? q_new : 0) - inv;
  int qm[VPT], im[VPT], vm[VPT];
  int nqi = 0, nvi = 0, negs = 0;
  bool all_le0 = true;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    vertex_masks(tgt, s[k], F[k], n1, S0[k], S1[k], qm[k], im[k]);
    const int ui = inv + im[k];
    vm[k] = ui == 0;
    const int sm = cut_like ? qm[k] : (vm[k] ? q_new + qm[k] : 0) - ui - score_fresh;
    nqi += __popcll(__ballot(v < N && qm[k] > 0));
    nvi += __popcll(__ballot(v < N && im[k] < 0));  // '< 0' in step (:521-524)
    negs += __popcll(__ballot(v < N && s[k] < 0));
    all_le0 = all_le0 && __ballot(v < N && sm > 0) == 0ull;
  }
  const bool isnew = (a.cfg.has_basin_reward || a.cfg.has_stag_punishment) ? history_update<VPT>(a, e, lane, sc, act, words)
                                                                            : true;
  // reward (:418-457)
  double best_score = sc->best_score, best_nscore = sc->best_nscore;
  double rew = 0.0;
  int early = sc->early + 1;
  const bool improved = score > best_score;
  if (improved) {
    early = 0;
    if (a.cfg.reward_signal == ECO_REWARD_BLS) rew = a.cfg.norm_rewards ? nscore - best_nscore : score - best_score;
  }
  if (a.cfg.reward_signal == ECO_REWARD_DENSE) rew = a.cfg.norm_rewards ? fd.dn : fd.d;
  if (a.cfg.has_stag_punishment && !isnew) rew -= a.cfg.stag_punishment;
  if (a.cfg.has_basin_reward && all_le0 && isnew) rew += a.cfg.basin_reward;
  // best tracking (:459-477)
  double best_solution = sc->best_solution;
  int best_n1 = sc->best_n1, best_inv = sc->best_inv;
  if (improved) {
    best_score = score;
    best_nscore = nscore;
    best_n1 = n1;
    best_inv = inv;
    if (cut_like) best_solution = qn - score;  // cut(best) = max(0, qn) - quality, exact
    else best_solution = valid ? (double)n1 : (target_maximises(tgt) ? 0.0 : (double)N);
#pragma unroll
    for (int k = 0; k < VPT; ++k) bs[k] = s[k];
  }
  int ham = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) ham += __popcll(__ballot(bs[k] != s[k]));
  bool done = (t == T);
  if (a.cfg.stopping == ECO_STOP_EARLY && early == 15) done = true;
  if (a.cfg.stopping == ECO_STOP_QUARTER && t == T / 4) done = true;
  if (!a.cfg.reversible_spins && negs == 0) done = true;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N) {
      gsp[v] = (int8_t)s[k];
      gF[v] = F[k];
      gt[v] = (int16_t)tsf[k];
      if (improved) gb[v] = (int8_t)bs[k];
    }
  }
  if (lane == 0) {
    sc->score = score; sc->nscore = nscore;
    sc->best_score = best_score; sc->best_nscore = best_nscore; sc->best_solution = best_solution;
    sc->t = t; sc->hamming = ham; sc->done = done ? 1 : 0; sc->early = early;
    sc->n1 = n1; sc->inv = inv; sc->best_n1 = best_n1; sc->best_inv = best_inv;
    a.rewards[e] = rew;
    a.dones[e] = done ? 1 : 0;
  }
  ProbObs c;
  c.mlr = mlr; c.inorm = inorm;
  if (cut_like) {
    const double dsc = score - best_score;
    c.dist_best = (dsc < 0.0 ? -dsc : dsc) / mlr;
  } else {
    const int dq = set_quality(tgt, n1, N) - set_quality(tgt, best_n1, N);
    c.dist_best = (double)(dq < 0 ? -dq : dq) / mlr;                      // :516-519
  }
  c.hamming = (double)ham;
  c.nqi = (double)nqi / (double)N;
  c.nvi = (double)nvi / (double)N;
  const double xt = (double)(t - T) / (double)a.cfg.horizon_length + 1.0;
  c.term = xt > 0.0 ? xt : 0.0;
  c.ep_time = tab_ptr(a)[t];
  c.gvd = (double)(inv - best_inv) / inorm;                                // :529-532
  c.valid = valid ? 1.0 : 0.0;
  c.basis = a.cfg.spin_basis;
  write_prob_obs<VPT>(a, e, lane, s, qm, im, vm, tsf, c, cut_like);
}

// Greedy.step (src/agents/solver.py:110-127) on the generic scorers' score mask.
template <int VPT>
__global__ __launch_bounds__(256) void env_greedy_problem_kernel(EnvArgs a, int32_t* actions) {
  extern __shared__ uint8_t c_lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int e = uniform_i(blockIdx.x * 4 + wv);
  if (e >= a.B) return;
  const int N = a.cfg.n_spins;
  const int tgt = a.cfg.optimisation_target;
  const bool cut_like = tgt == ECO_TARGET_MIN_CUT;
  EpScal* sc = scal_ptr(a) + e;
  if (sc->done) {
    if (lane == 0) actions[e] = 0;
    return;
  }
  const int8_t* gsp = (const int8_t*)(a.state + a.L.off_spins) + (size_t)e * N;
  const int32_t* gF = (const int32_t*)(a.state + a.L.off_field) + (size_t)e * N;
  int s[VPT], F[VPT], S0[VPT], S1[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    s[k] = v < N ? gsp[v] : 0;
    F[k] = v < N ? gF[v] : 0;
    S0[k] = 0; S1[k] = 0;
  }
  if (tgt == ECO_TARGET_MIN_DOM_SET) {
    const int gid = sc->graph;
    const int32_t* rp = a.gs.row_ptr + (size_t)gid * (N + 1);
    const uint32_t* ed = a.gs.edges + a.gs.edge_base[gid];
    uint8_t* code = c_lds + wv * N;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int v = lane + 64 * k;
      if (v < N) code[v] = mds_code(s[k], F[k]);
    }
    wave_lds_sync();
    mds_neighbour_counts<VPT>(rp, ed, code, N, lane, S0, S1);
  }
  const int n1 = sc->n1, inv = sc->inv;
  const int q = cut_like ? 0 : set_quality(tgt, n1, N);
  const int score = ((inv == 0) ? q : 0) - inv;
  int best = INT_MIN, bi = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int v = lane + 64 * k;
    if (v < N && (a.cfg.reversible_spins || s[k] < 0)) {
      int qm, im;
      vertex_masks(tgt, s[k], F[k], n1, S0[k], S1[k], qm, im);
      const int ui = inv + im;
      const int sm = cut_like ? qm : (ui == 0 ? q + qm : 0) - ui - score;
      if (sm > best || (sm == best && v < bi)) { best = sm; bi = v; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int ob = __shfl_xor(best, o, 64), oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) {
    if (best < 0 || bi == 0x7fffffff) {
      sc->done = 1;
      actions[e] = 0;
    } else {
      actions[e] = bi;
    }
  }
}

int env_reset_problem_launch(const EnvArgs& a, int blocks, size_t lds, hipStream_t st) {
  ECO_DISPATCH_VPT(a.cfg.n_spins, (env_reset_problem_kernel<V><<<blocks, 256, lds, st>>>(a)));
  return check_launch("env_reset (generic scorer)");
}

int env_step_problem_launch(const EnvArgs& a, int blocks, size_t lds, hipStream_t st) {
  ECO_DISPATCH_VPT(a.cfg.n_spins, (env_step_problem_kernel<V><<<blocks, 256, lds, st>>>(a)));
  return check_launch("env_step (generic scorer)");
}

int env_greedy_problem_launch(const EnvArgs& a, int32_t* actions, int blocks, size_t lds, hipStream_t st) {
  ECO_DISPATCH_VPT(a.cfg.n_spins, (env_greedy_problem_kernel<V><<<blocks, 256, lds, st>>>(a, actions)));
  return check_launch("env_greedy (generic scorer)");
}

}  // namespace eco
