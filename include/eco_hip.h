/*
 * eco_hip.h -- C ABI of libecohip.so, the MI355X (gfx950) engine behind the
 * ECO-DQN MaxCut hot path.
 *
 * The reference (BetterBelle/eco-dqn) is pure Python with no FFI: its boundary is
 * the Python API.  Each entry point below replaces one reference
 * interface, cited as file:line under the reference tree.  The Python host
 * package (eco-dqn_amd/eco_hip) binds these through ctypes and keeps the
 * reference's class/method names; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Every buffer is caller-owned DEVICE memory (PyTorch tensors used as plain
 *     containers: pass tensor.data_ptr()).  The library never allocates or frees
 *     caller memory; scratch is sized by the *_bytes queries.
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream); NULL
 *     means the default stream.  All calls are stream-ordered and asynchronous.
 *   - Every function returns ECO_OK (0) or an error code; eco_last_error() gives
 *     a thread-local message.  Host-side argument errors are reported before any
 *     launch.
 *   - Batched envs that are done are auto-masked: stepping them changes nothing
 *     and `dones` stays 1 until they are reset (the reference never steps a done
 *     env in its batched loops, experiments/utils.py:183-201, dqn.py:558-600).
 */
#ifndef ECO_HIP_H
#define ECO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *eco_stream_t; /* hipStream_t */

/* ---- status codes; the Python wrapper maps them to the reference's exceptions ---- */
enum {
  ECO_OK = 0,
  ECO_ERR_ARG = 1,         /* bad argument (ValueError) */
  ECO_ERR_HIP = 2,         /* HIP runtime error */
  ECO_ERR_PAST_END = 3,    /* step after done: NotImplementedError, spinsystem.py:365-367 */
  ECO_ERR_BASIS = 4,       /* unknown spin basis: Exception, spinsystem.py:600-606 */
  ECO_ERR_TARGET = 5,      /* unsupported optimisation target: NotImplementedError, score_solver.py:885 */
  ECO_ERR_OBSERVABLE = 6,  /* first observable != SPIN_STATE: AssertionError, spinsystem.py:116 */
  ECO_ERR_GRAPH = 7,       /* graph with no nonzero local reward (spinsystem.py:203-211) or bad CSR */
  ECO_ERR_KEY = 8,         /* missing heap / buffer position: KeyError, dqn/utils.py:236,259 */
  ECO_ERR_INDEX = 9        /* rebalance of a heap that is not full: IndexError, dqn/utils.py:196 */
};

/* ---- enums: numerically identical to src/envs/utils.py:10-66 ---- */
enum { ECO_OBS_SPIN_STATE = 1, ECO_OBS_IMMEDIATE_QUALITY_CHANGE = 2, ECO_OBS_IMMEDIATE_VALIDITY_DIFFERENCE = 3,
       ECO_OBS_IMMEDIATE_VALIDITY_CHANGE = 4, ECO_OBS_TIME_SINCE_FLIP = 5, ECO_OBS_EPISODE_TIME = 6,
       ECO_OBS_TERMINATION_IMMANENCY = 7, ECO_OBS_NUMBER_OF_QUALITY_IMPROVEMENTS = 8,
       ECO_OBS_NUMBER_OF_VALIDITY_IMPROVEMENTS = 9, ECO_OBS_DISTANCE_FROM_BEST_SOLUTION = 10,
       ECO_OBS_DISTANCE_FROM_BEST_STATE = 11, ECO_OBS_GLOBAL_VALIDITY_DIFFERENCE = 12, ECO_OBS_VALIDITY_BIT = 13 };
enum { ECO_REWARD_DENSE = 1, ECO_REWARD_BLS = 2, ECO_REWARD_SINGLE = 3, ECO_REWARD_CUSTOM_BLS = 4 };
enum { ECO_BASIS_SIGNED = 1, ECO_BASIS_BINARY = 2 };
enum { ECO_STOP_NORMAL = 1, ECO_STOP_QUARTER = 2, ECO_STOP_EARLY = 3 };
/* OptimisationTarget (src/envs/utils.py:32-39); ENERGY has no scorer (score_solver.py:860-885) */
enum { ECO_TARGET_CUT = 1, ECO_TARGET_ENERGY = 2, ECO_TARGET_MIN_COVER = 3, ECO_TARGET_MIN_CUT = 4,
       ECO_TARGET_MAX_IND_SET = 5, ECO_TARGET_MAX_CLIQUE = 6, ECO_TARGET_MIN_DOM_SET = 7 };

#define ECO_MAX_OBS 16     /* observables per env (all 13 of MAIN_OBSERVABLES, src/envs/utils.py:76-88) */
#define ECO_MPNN_MAX_OBS 16 /* MPNN n_obs_in limit; node-feature rows are ECO_OBS_X_STRIDE(n_obs_in) floats */
/* obs_x row width in floats for n_obs observables: 8 up to 8 observables, else 16 */
#define ECO_OBS_X_STRIDE(n_obs) ((n_obs) <= 8 ? 8 : 16)
#define ECO_MAX_SPINS 2048 /* largest N the env kernels take (wave-per-episode, 32 vertices per lane) */

/* Env configuration: the kwargs of core.make("SpinSystem", gg, max_steps, **env_args)
 * (src/envs/core.py:3-10 -> spinsystem.py:29-48).  OptimisationTarget.CUT is the hot path (its own
 * kernels); MIN_COVER, MIN_CUT, MAX_IND_SET, MAX_CLIQUE and MIN_DOM_SET run the generic scorer kernels
 * (score_solver.py:232-858).  Unbiased graphs, ExtraAction.NONE and memory_length=None only.
 * With CUT / MIN_CUT the validity-mask observables (3, 4, 9) are rejected with ECO_ERR_OBSERVABLE:
 * those scorers return the invalidity mask as a python list and the reference raises TypeError. */
typedef struct {
  int32_t n_spins;                /* N */
  int32_t max_steps;              /* T */
  int32_t n_obs;                  /* number of observables, 1..13 */
  int32_t obs_ids[ECO_MAX_OBS];   /* Observable values; obs_ids[0] == SPIN_STATE */
  int32_t reward_signal;          /* ECO_REWARD_* */
  int32_t norm_rewards;           /* bool */
  int32_t reversible_spins;       /* bool */
  int32_t spin_basis;             /* ECO_BASIS_* (observation row 0 only) */
  int32_t stopping;               /* ECO_STOP_* */
  int32_t has_basin_reward;       /* basin_reward is not None */
  int32_t has_stag_punishment;    /* stag_punishment is not None */
  int32_t horizon_length;         /* horizon_length, or max_steps when None (spinsystem.py:163) */
  int32_t optimisation_target;    /* ECO_TARGET_* */
  double basin_reward;
  double stag_punishment;
} eco_env_config;

/* A set of G graphs with N vertices each, as CSR on the device.
 * Replaces GraphGenerator.get() -> ndarray[N,N] (src/envs/utils.py:121-123): the
 * dense f64 adjacency is never materialised on the hot path.
 * Filled by the caller: n_graphs, n_spins, row_ptr, edge_base, edges.
 * Filled by eco_graphs_prepare: deg, max_deg, meta, valid. */
typedef struct {
  int32_t n_graphs;
  int32_t n_spins;
  const int32_t *row_ptr;   /* [G][N+1] edge offsets local to each graph */
  const int64_t *edge_base; /* [G] offset of graph g's first edge in `edges` */
  const uint32_t *edges;    /* packed edge: column | ((uint8_t)weight << 24); integer weights in [-128,127] */
  int32_t *deg;             /* [G][N] number of nonzero entries per row (mpnn.py:34-38, before the 0->1 clamp) */
  int32_t *max_deg;         /* [G] max over rows of max(deg,1) */
  double *meta;             /* [G][4]: max_local_reward, quality_normalizer, lower_bound, sum(J) */
  int32_t *valid;           /* [G] 1 if the graph has a nonzero local reward */
  int32_t unit_weights;     /* caller: 1 if every stored weight is +-1 (EdgeType.DISCRETE / UNIFORM graphs).
                               Enables the dense-aggregation MPNN kernels for blocks of <= 224 rows; they
                               verify it and report ECO_ERR_GRAPH through eco_check_errors if it is false. */
  uint32_t *adjbits;        /* caller-allocated (eco_graphs_adjbits_bytes) or NULL; filled by eco_graphs_prepare:
                               per graph, node and lane quarter the bitmask adjacency operand of the dense MPNN
                               kernels ([G][N][4][4] u32 up to N = 224, [G][N][4][8] above, to N = 512), so
                               they skip the per-call CSR -> bitmask build */
} eco_graph_set;

/* Graph metadata: MaximumCutUnbiasedScorer normalisers (score_solver.py:347-375)
 * and the MPNN degree normalisation (mpnn.py:34-38), computed on the device. */
int eco_graphs_prepare(eco_graph_set *gs, eco_stream_t stream);

/* Bytes of gs->adjbits for G graphs of N vertices: nonzero only where the dense MPNN path runs one graph
 * per workgroup (104 < N <= 224); 0 means pass adjbits = NULL. */
size_t eco_graphs_adjbits_bytes(int32_t n_spins, int32_t n_graphs);

/* On-device graph generation into graphs [first, first+count) of a set whose edge slots are
 * fixed (edge_base[g] = g * edge_cap): the training-reset graph draws of
 * RandomErdosRenyiGraphGenerator (kind ER, param = p) and RandomBarabasiAlbertGraphGenerator
 * (kind BA, param = m) (src/envs/utils.py:165-236); +-1 weights when discrete_weights, else 1.
 * Runs eco_graphs_prepare afterwards.  An edge-slot overflow is reported by eco_check_errors. */
enum { ECO_GRAPH_ER = 1, ECO_GRAPH_BA = 2 };
size_t eco_graphs_generate_workspace_bytes(int32_t n_spins, int32_t count);
int eco_graphs_generate(eco_graph_set *gs, int32_t first, int32_t count, int32_t kind, double param,
                        int32_t discrete_weights, uint64_t seed, int64_t edge_cap, void *workspace,
                        eco_stream_t stream);

/* ---- batched SpinSystem (spinsystem.py) ---- */

/* Bytes of the opaque per-batch env state buffer (spins, local fields, counters,
 * best-so-far, visited-state sets). */
size_t eco_env_state_bytes(const eco_env_config *cfg, int32_t batch);

/* SpinSystemBase.reset (spinsystem.py:183-259, _reset_state :283-330).
 * graph_ids[B]: graph of each episode.  spins[B][N] (int8, signed +-1) or NULL:
 * NULL draws uniform +-1 spins from a counter-based generator keyed by
 * (seed, episode) (reversible) or all -1 (irreversible, :295-297).
 * reset_mask[B] or NULL (= all): only episodes with mask != 0 are reset.
 * `state` must be zero-filled before its first reset.  As in the reference, the first observation
 * after a reset divides the validity difference by the invalidity normaliser of the episode's
 * previous reset (set_invalidity_normalizer runs after _reset_state, spinsystem.py:216-219), 1 for
 * the first reset of a zero-filled state.
 * Outputs (each may be NULL): obs_x[B][N][ECO_OBS_X_STRIDE(n_obs)] fp32 node features as the MPNN reads
 * them (obs.float(), dqn.py:282), obs_f64[B][n_obs][N] the reference's float64
 * observation rows (get_observation :561-574 without the appended adjacency). */
int eco_env_reset(const eco_env_config *cfg, const eco_graph_set *gs, void *state, int32_t batch,
                  const int32_t *graph_ids, const int8_t *spins, const uint8_t *reset_mask, uint64_t seed,
                  float *obs_x, double *obs_f64, eco_stream_t stream);

/* SpinSystemBase.step (spinsystem.py:355-559) for every episode at once.
 * actions[B] int32 in [0,N); rewards[B] f64; dones[B] u8; obs as in reset. */
int eco_env_step(const eco_env_config *cfg, const eco_graph_set *gs, void *state, int32_t batch,
                 const int32_t *actions, double *rewards, uint8_t *dones, float *obs_x, double *obs_f64,
                 eco_stream_t stream);

/* Greedy solver (src/agents/solver.py:88-131) for every episode: actions[B] = argmax (first index) of
 * the scorer's score mask (allowed vertices only when irreversible); episodes with no non-negative
 * change are marked done (the solver stops). Step with eco_env_step.  `gs` is the set the episodes
 * were reset on (read by MIN_DOM_SET's neighbour counts; may be NULL for the other targets). */
int eco_env_greedy_actions(const eco_env_config *cfg, const eco_graph_set *gs, void *state, int32_t batch,
                           int32_t *actions, eco_stream_t stream);

/* Read-out of the env attributes callers use (dqn.py:564-566, experiments/utils.py:194-197):
 * scalars[B][ECO_ENV_SCALARS] = {current_step, score, normalized_score, best_score,
 *     best_score_normalized, best_solution, hamming_to_best, done, max_local_reward,
 *     solution_quality_normalizer, invalidity_normalizer, lower_bound, set_size (#spins == +1),
 *     invalidity_degree, graph_id, 0};
 * spins / best_spins [B][N] int8 signed (each may be NULL). */
#define ECO_ENV_SCALARS 16
int eco_env_read(const eco_env_config *cfg, const void *state, int32_t batch, double *scalars, int8_t *spins,
                 int8_t *best_spins, eco_stream_t stream);

/* ---- MPNN Q-network (src/networks/mpnn.py) ---- */

/* Parameter count of MPNN(n_obs_in, n_layers=3, n_features=64, n_hid_readout=[])
 * in state_dict order (58,425 for n_obs_in = 7). */
size_t eco_mpnn_param_count(int32_t n_obs_in);
/* Floats of the kernel-side packed parameter image. */
size_t eco_mpnn_packed_count(void);
/* Re-pack the flat state_dict-ordered parameters into the kernel image
 * (after load_state_dict and after every optimiser step). */
int eco_mpnn_pack(const float *params, int32_t n_obs_in, float *packed, eco_stream_t stream);

/* Norm-max scope of EdgeAndNodeEmbeddingLayer (mpnn.py:102): */
enum { ECO_NORM_PER_GRAPH = 0, /* B=1 semantics: act (dqn.py:282) */
       ECO_NORM_PER_CALL = 1,  /* max over the whole call: train_step / batched eval */
       ECO_NORM_PER_CALL_REUSE = 2 /* as PER_CALL, the call maximum taken from this workspace as the previous
                                      PER_CALL forward on the SAME graph ids left it (train_step's online(s)
                                      after the s' pair): skips its reduction launch */ };

/* epsilon-greedy act fused into the forward (dqn.py:453-465, predict :490-512).
 * action = random with probability epsilon (uniform over allowed vertices),
 * else the first argmax of Q over allowed vertices. Irreversible envs allow only
 * vertices whose node feature 0 equals allowed_value (dqn.py:462-464, :505-511). */
typedef struct {
  float epsilon;
  int32_t reversible;      /* 1: every vertex allowed */
  float allowed_value;     /* irreversible: feature-0 value of flippable vertices */
  uint64_t seed;
  uint64_t counter;        /* advance per call; (seed, counter, episode) keys the draws */
} eco_act_config;

size_t eco_mpnn_workspace_bytes(int32_t n_spins, int32_t batch);
/* Bytes of the activations a training forward saves for eco_mpnn_backward. */
size_t eco_mpnn_saved_bytes(int32_t n_spins, int32_t batch);

/* MPNN.forward (mpnn.py:40-77) on B graphs at once.
 * obs_x[B][N][ECO_OBS_X_STRIDE(n_obs_in)]: node features; adjacency = graphs graph_ids[B] of `gs`.
 * Up to 8 features every kernel applies; 9..16 features (MAIN_OBSERVABLES) run the CSR-gather kernels
 * for N <= 512 (the dense-aggregation and N > 512 kernels take 8-float rows).
 * N > 512 with every graph id naming ONE graph of a single-graph set with +-1 weights (the GSet G22
 * best-cut search of experiments/test_eco.py) takes the shared-graph kernels: the aggregation A.[H_1..H_B]
 * from LDS-staged per-episode blocks, N <= 2048; the workspace (eco_mpnn_workspace_bytes) holds their
 * node-major buffers and, across calls, the graph's degree ranking and aggregation tile tables, reused while
 * a 64-bit key of the graph's CSR, N and the batch matches (rebuilt in the call otherwise; any other path that
 * writes the workspace invalidates the key), so a caller may pass the same workspace to every call.
 * q[B][N] fp32 (may be NULL when only actions are wanted).
 * act / actions[B]: optional fused epsilon-greedy action selection.
 * saved: NULL for inference; for the training forward of train_step (dqn.py:437)
 * a buffer of eco_mpnn_saved_bytes that receives the activations. */
int eco_mpnn_forward(const float *packed, int32_t n_obs_in, const eco_graph_set *gs, const int32_t *graph_ids,
                     int32_t batch, const float *obs_x, int32_t norm_scope, float *q, const eco_act_config *act,
                     int32_t *actions, void *saved, void *workspace, eco_stream_t stream);

/* Two networks on the same graphs and node features in one call: the double-DQN pair of dqn.py:416-428
 * (a = online net -> greedy argmax a* over s', b = target net -> Q(s') to gather at a*).  Equivalent to
 * eco_mpnn_forward(packed_a, ..., q_a, act_a, actions_a) followed by eco_mpnn_forward(packed_b, ..., q_b,
 * act_b, actions_b) with saved = NULL; for one-graph dense blocks (ER-200 ... ER-224 with adjbits) it is ONE
 * launch whose workgroups stage each graph once and run both networks on it. */
int eco_mpnn_forward_pair(const float *packed_a, const float *packed_b, int32_t n_obs_in, const eco_graph_set *gs,
                          const int32_t *graph_ids, int32_t batch, const float *obs_x, int32_t norm_scope,
                          float *q_a, const eco_act_config *act_a, int32_t *actions_a, float *q_b,
                          const eco_act_config *act_b, int32_t *actions_b, void *workspace, eco_stream_t stream);

/* Kernel-path policy of the MPNN dispatcher (process-wide, default 0 = the fastest kernel for each shape).
 * Each bit routes the calls it names to another product kernel family that also serves other shapes, with
 * the same results within the fp32 bars of the tests (tests/test_kernel_paths_gpu.py runs every bit):
 *   NO_DENSE  -- blocks the dense-aggregation kernels would take run the CSR-gather kernels instead;
 *   NO_DL     -- one-graph blocks of 224 < N <= 512 run the CSR-gather kernels;
 *   NO_SHARED -- N > 512 single-graph inference runs the per-episode global-memory kernel;
 *   NO_PAIR   -- eco_mpnn_forward_pair runs as two eco_mpnn_forward calls;
 *   DENSE2_FWD -- dense-aggregation forwards and backwards (N <= 224 blocks) run the one-tile-per-wave 16-wave
 *                 kernels instead of the two-tiles-per-wave 8-wave ones (bitwise the same results; A/B and
 *                 cross-check).
 * The library reads no environment variables; this call is the only switch. Returns the previous mask. */
enum { ECO_PATH_NO_DENSE = 1, ECO_PATH_NO_DL = 2, ECO_PATH_NO_SHARED = 4, ECO_PATH_NO_PAIR = 8, ECO_PATH_DENSE2_FWD = 16 };
int32_t eco_set_kernel_paths(int32_t mask);

/* Test probe of the fp16x2 operand split (no reference counterpart; guards the dense kernels' inline-asm
 * v_fma_mix split, which carries its own MFMA wait states -- src/networks/mpnn.py:111-118 is the Linear it feeds).
 * n_blocks blocks of 64 nodes x 16 fp32 activations x[n_blocks][64][16], per-block power-of-two scale sf[n_blocks],
 * one 64-input half of fp16x2 weight fragments w_frags (16 fragments of 512 fp16, the PK_FH layout); order 0 feeds
 * the MFMAs as the dense kernels do, order 1 consumes the lo piece first, order 2 issues the split and the first
 * MFMA reading its lo piece in one asm block (the MFMA straight after the split's own wait states, nothing between
 * them that the compiler could schedule).  out[2][n_blocks][16][64]: the fp32
 * accumulators from the asm split, then from a plain-conversion split -- bitwise equal when the split is sound. */
int eco_probe_split2_mfma(const float *x, const float *sf, const uint16_t *w_frags, int32_t n_blocks, int32_t order,
                          float *out, eco_stream_t stream);

/* ---- DQN train step (dqn.py:403-451) ---- */

size_t eco_mpnn_backward_workspace_bytes(int32_t n_spins, int32_t batch);
/* loss.backward() through the MPNN: grad[flat, state_dict order] = dLoss/dparams
 * for dq[B][N] = dLoss/dQ of the forward that filled `saved` (norm scope per call).
 * grad is overwritten (zero_grad + backward).  Reductions are in a fixed order:
 * results are bitwise reproducible run to run. */
int eco_mpnn_backward(const float *packed, int32_t n_obs_in, const eco_graph_set *gs, const int32_t *graph_ids,
                      int32_t batch, const float *obs_x, const void *saved, const float *dq, float *grad,
                      void *workspace, eco_stream_t stream);

/* Double-DQN TD target and MSE gradient (dqn.py:409-440, reversible env):
 * q_t = q_target_next[b][a_star[b]] (a_star = argmax of the online net on s'),
 * td = r + (1 - done) * gamma * q_t; loss = mean((q_s[b][a_b] - td)^2);
 * dq[B][N] = dloss/dq (zero except at a_b); sqerr[B] scratch; loss[1]. */
int eco_dqn_td(const float *q_s, const float *q_target_next, const int32_t *a_star, const int32_t *actions,
               const float *rewards, const float *dones, int32_t batch, int32_t n_spins, float gamma,
               int32_t clip_q_targets, float *dq, float *sqerr, float *loss, eco_stream_t stream);

/* torch.optim.Adam step (dqn.py:212, optimizer.step() :449) on a flat fp32 buffer.
 * grad_scale multiplies the gradient first (1/world after a multi-GPU sum all-reduce). */
int eco_adam(float *params, const float *grad, float *exp_avg, float *exp_avg_sq, int32_t n, double lr,
             double beta1, double beta2, double eps, double weight_decay, double grad_scale, int64_t step,
             eco_stream_t stream);

/* ReplayBuffer (dqn/utils.py:28-83) as a device ring of compact transitions.  Buffers are
 * caller-owned: xs/xn [capacity][N][x_stride] fp32 node features of s and s'; graph id, action,
 * reward (fp32, dqn.py:299), done (fp32). */
typedef struct {
  int32_t capacity;
  int32_t n_spins;
  int32_t x_stride;  /* floats per node row: ECO_OBS_X_STRIDE(n_obs) (8 or 16; 0 means 8) */
  float *xs;
  float *xn;
  int32_t *gid;
  int32_t *act;
  float *rew;
  float *done;
} eco_replay;

/* ReplayBuffer.add for B transitions into slots (pos + b) % capacity (B <= capacity). */
int eco_replay_push(const eco_replay *rb, int32_t pos, int32_t batch, const float *xs, const float *xn,
                    const int32_t *graph_ids, const int32_t *actions, const double *rewards, const uint8_t *dones,
                    eco_stream_t stream);
/* ReplayBuffer.sample: m DISTINCT uniform slots of the first `size` (random.sample,
 * dqn/utils.py:53), keyed by (seed, counter); gathered into minibatch buffers. */
int eco_replay_sample(const eco_replay *rb, int32_t size, int32_t m, uint64_t seed, uint64_t counter, float *xs,
                      float *xn, int32_t *graph_ids, int32_t *actions, float *rewards, float *dones,
                      eco_stream_t stream);

/* ReplayBuffer (dqn/utils.py:28-83) of MaxCut (OptimisationTarget.CUT) transitions stored as integer env
 * state: ONE state per transition -- per vertex a u32 {spin sign | time-since-flip count | local field
 * (J s)_v as int16} -- plus four float64 observation scalars for s and for s' and graph id / action /
 * reward / done: 4N + 80 bytes per transition.  s' is rebuilt on sample from s, the action and the graph
 * (the env's step), and both states' feature rows are rebuilt with the env's own observation arithmetic
 * (spinsystem.py:486-535), bit-exactly.  Same ReplayBuffer semantics: the newest `capacity` transitions
 * are held, sample = m distinct uniform ones (random.sample, :53).  `pushed` counts the transitions added
 * over the buffer's life (the k-th lives in slot k % (capacity + batch)); push writes each episode's s'
 * straight into the slot of its next transition, so `ring` (caller-owned device memory of
 * eco_replay_compact_bytes()) has `batch` slots more than `capacity`.  Requires |J s| < 2^15 (reported
 * through eco_check_errors), max_steps < 2^15 and n_spins <= ECO_COMPACT_MAX_SPINS. */
#define ECO_COMPACT_MAX_SPINS 8192
size_t eco_replay_compact_bytes(int32_t n_spins, int32_t capacity, int32_t batch);
/* After env reset (all episodes, or those with mask != 0): record their states as the s of the transitions
 * pushed + e. */
int eco_replay_compact_snapshot(const eco_env_config *cfg, const void *env_state, int32_t batch, void *ring,
                                int32_t capacity, int64_t pushed, const uint8_t *mask, eco_stream_t stream);
/* After env step: ReplayBuffer.add of (s, a, r, s', done) for every episode (dqn.py:298-304) as transitions
 * pushed .. pushed + batch - 1; graph ids come from the env state. */
int eco_replay_compact_push(const eco_env_config *cfg, const void *env_state, int32_t batch, void *ring,
                            int32_t capacity, int64_t pushed, const int32_t *actions, const double *rewards,
                            const uint8_t *dones, eco_stream_t stream);
/* ReplayBuffer.sample: m distinct transitions of the newest `size` (keyed like eco_replay_sample: the same
 * keys pick the same transitions as the fp32 feature ring filled by the same pushes) expanded into
 * node-feature rows xs / xn [m][N][ECO_OBS_X_STRIDE(n_obs)] plus graph ids, actions, rewards, dones.
 * env_state / env_batch: the env the ring was filled from (its f64 time table); gs: its graph set. */
int eco_replay_compact_sample(const eco_env_config *cfg, const void *env_state, const eco_graph_set *gs,
                              int32_t env_batch, const void *ring, int32_t capacity, int32_t size, int64_t pushed,
                              int32_t m, uint64_t seed, uint64_t counter, float *xs, float *xn, int32_t *graph_ids,
                              int32_t *actions, float *rewards, float *dones, eco_stream_t stream);

/* PrioritisedReplayBuffer (dqn/utils.py:86-277), rank-based: the binary max-heap of (buffer position,
 * td error) is a native HOST structure (every add / update is a sequential up-/down-heap walk) following
 * the reference's comparisons exactly; transitions stay in HBM in an eco_replay ring at slot = buffer
 * position - 1 and are fetched with eco_replay_gather.  Buffer positions are 1-based like the reference's.
 * These calls are host-only (no stream, no device memory) except eco_replay_gather. */
typedef struct eco_per eco_per;
eco_per *eco_per_create(int32_t capacity, double alpha, double beta0);      /* __init__, :88-111 (NULL: bad capacity) */
void eco_per_destroy(eco_per *per);
int32_t eco_per_len(const eco_per *per);                                   /* __len__, :278 */
double eco_per_beta(const eco_per *per);
int eco_per_full(const eco_per *per);
int eco_per_configure_beta_anneal_time(eco_per *per, double beta_max_at_samples);  /* :275-276 */
/* n consecutive add() calls (:120-142); buffer_positions[n] (nullable) receives the positions written. */
int eco_per_add(eco_per *per, int32_t n, int32_t *buffer_positions);
/* update_priorities (:234-240) in the order given. */
int eco_per_update_priorities(eco_per *per, int32_t n, const int32_t *buffer_positions, const double *td_errors);
/* rebalance (:185-202); ECO_ERR_INDEX unless the heap is full. */
int eco_per_rebalance(eco_per *per);
/* sample (:242-273) without the gather: one rank per partition -- injected (`ranks`, the reference's
 * np.random.randint(low, high) draws) or drawn natively from `seed` when NULL -- giving buffer_positions
 * [batch], float32 importance weights [batch] and (nullable) ranks_out [batch].  = begin + finish; begin
 * refreshes the partitions (:247-254) and writes their boundaries bounds[batch + 1] (nullable; partition k
 * = ranks [bounds[k], bounds[k+1])), so a caller can draw the ranks with its own RNG before finish. */
int eco_per_sample_begin(eco_per *per, int32_t batch, int32_t *bounds);
int eco_per_sample_finish(eco_per *per, int32_t batch, const int64_t *ranks, uint64_t seed, int32_t *buffer_positions,
                          float *weights, int64_t *ranks_out);
int eco_per_sample(eco_per *per, int32_t batch, const int64_t *ranks, uint64_t seed, int32_t *buffer_positions,
                   float *weights, int64_t *ranks_out);
/* Heap positions 1..len: buffer position and td error of each (host arrays of eco_per_len()). */
int eco_per_heap(const eco_per *per, int32_t *buffer_positions, double *td_errors);
/* Current partitions: bounds [n+1] and rank probabilities [len] (both nullable); returns n. */
int32_t eco_per_partitions(const eco_per *per, int32_t *bounds, double *probs);
/* Gather m transitions of an eco_replay ring by explicit slot (DEVICE int32 slots[m], each < capacity). */
int eco_replay_gather(const eco_replay *rb, int32_t m, const int32_t *slots, float *xs, float *xn, int32_t *graph_ids,
                      int32_t *actions, float *rewards, float *dones, eco_stream_t stream);

/* Device-side errors (bad action, invalid graph, non-signed injected spins) are
 * recorded in a device word by the asynchronous kernels; this synchronises
 * `stream`, returns and clears the first one (ECO_OK if none). */
int eco_check_errors(eco_stream_t stream);
/* Asynchronous peek at the same device word: enqueue a copy of it into *dst (pinned host or device memory) on
 * `stream`, without synchronising or clearing it.  A caller that must not block (DQN.learn's per-evaluation check of
 * the regenerated graphs, dqn.py:349-364 cadence) reads *dst once an event behind the copy has fired and calls
 * eco_check_errors only when it is nonzero. */
int eco_error_word_copy(int32_t *dst, eco_stream_t stream);

/* Thread-local text of the last error. */
const char *eco_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* ECO_HIP_H */
