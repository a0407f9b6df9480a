// Shared device/host helpers for libecohip (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/eco_hip.h"

namespace eco {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);
int32_t* err_word();  // device error word shared by all async kernels (eco_check_errors)
int graphs_prepare_range(eco_graph_set* gs, int first, int count, hipStream_t st);  // eco_env.hip

// ---- edge packing: column | (uint8 weight << 24) ----
__device__ __forceinline__ int edge_col(uint32_t e) { return (int)(e & 0xFFFFFFu); }
__device__ __forceinline__ int edge_w(uint32_t e) { return (int)(int8_t)(e >> 24); }

// ---- counter-based RNG (splitmix64 finaliser) ----
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t rng3(uint64_t seed, uint64_t a, uint64_t b) {
  return mix64(mix64(mix64(seed) ^ a) ^ (b * 0xD6E8FEB86659FD93ull));
}
// uniform float in [0,1) from the top 24 bits
__host__ __device__ __forceinline__ float u01(uint64_t r) { return (float)(r >> 40) * (1.0f / 16777216.0f); }

// Zobrist key of vertex v: hash of a flipped-vertex set = XOR of its keys.
__device__ __forceinline__ uint64_t zobrist(int v) { return mix64(0x5EC0DE5EC0DEull + (uint64_t)v) | 1ull; }

// ---- wave (64-lane) reductions ----
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ long long wave_sum_ll(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ---- per-episode scalar record of the batched env ----
struct alignas(16) EpScal {
  double score;          // SpinSystemBase.score (quality = cut + |lb|), exact integer
  double nscore;         // normalized_score, f64 running sum (spinsystem.py:400)
  double best_score;
  double best_nscore;
  double best_solution;  // calculate_cut(best_spins)
  double mlr;            // scorer._max_local_reward
  double qn;             // scorer._solution_quality_normalizer
  double lbabs;          // |min(0, lower_bound)|
  uint64_t hash;         // Zobrist hash of the flipped set (HistoryBuffer key)
  int32_t t;             // current_step
  int32_t hamming;       // count_nonzero(best_spins - spins)
  int32_t graph;
  int32_t done;
  int32_t early;         // early_stopping counter
  int32_t visit_count;   // states inserted in the visited set
  // generic scorer targets (score_solver.py:232-858); unused by the CUT kernels
  double inorm;          // scorer._invalidity_normalizer (0 = never set: a fresh scorer's 1)
  double lb;             // scorer._lower_bound
  int32_t n1;            // set size #(s == +1)
  int32_t inv;           // invalidity degree of the current spins (integer for integer weights)
  int32_t best_n1;       // set size of best_spins
  int32_t best_inv;      // invalidity degree of best_spins
};

// Layout of the opaque env state buffer.
struct EnvLayout {
  int N, T, B, words, cap;
  size_t off_tab, off_scal, off_spins, off_field, off_tsf, off_best, off_vidx, off_vhash, off_vstates, total;
};

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

inline EnvLayout env_layout(int N, int T, int B) {
  EnvLayout L;
  L.N = N; L.T = T; L.B = B;
  L.words = (N + 63) / 64;
  int cap = 16;
  while (cap < 2 * (T + 1)) cap <<= 1;
  L.cap = cap;
  size_t o = 0;
  // [0,256): int32 T the f64 time table was built for; then (T+1) f64 running sums of 1/T
  L.off_tab = o;     o = align_up(o + 256 + sizeof(double) * (size_t)(T + 1), 256);
  L.off_scal = o;    o = align_up(o + sizeof(EpScal) * (size_t)B, 256);
  L.off_spins = o;   o = align_up(o + (size_t)B * N, 256);
  L.off_field = o;   o = align_up(o + (size_t)B * N * 4, 256);
  L.off_tsf = o;     o = align_up(o + (size_t)B * N * 2, 256);
  L.off_best = o;    o = align_up(o + (size_t)B * N, 256);
  L.off_vidx = o;    o = align_up(o + (size_t)B * cap * 4, 256);
  L.off_vhash = o;   o = align_up(o + (size_t)B * cap * 8, 256);
  L.off_vstates = o; o = align_up(o + (size_t)B * (size_t)(T + 1) * L.words * 8, 256);
  L.total = o;
  return L;
}

}  // namespace eco
