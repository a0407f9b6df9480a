// PrioritisedReplayBuffer (src/agents/dqn/utils.py:86-277): rank-based prioritised replay.
//
// The reference keeps a binary max-heap of [buffer_position, td_error, transition] in a Python dict and
// samples one rank per equal-probability partition of P(rank) ~ rank^-alpha.  The heap is a pointer-chasing,
// strictly sequential structure (every add / priority update is an up-/down-heap walk whose path depends on
// the previous one), so it lives here as a native host structure of two flat arrays (buffer position and
// td error per heap position); the transitions stay resident in HBM in the fp32 feature ring (eco_replay,
// slot = buffer position - 1) and a sample is one gather kernel over the chosen slots.  Every heap
// operation follows the reference's comparisons exactly (strict `<` / `>`, the `< size` bound of
// down_heap, the max-td lookup of a heap position that never exists) so the heap layout, partitions,
// probabilities and importance weights match the reference call for call (tests/test_per_cpu.py against
// tests/golden/per.npz, recorded from the reference).
#include <algorithm>
#include <cmath>
#include <vector>

#include "eco_common.h"

using namespace eco;

struct eco_per {
  int32_t capacity;
  double alpha, beta, beta_step;
  std::vector<int32_t> bp;   // heap position (1-based) -> buffer position
  std::vector<double> td;    // heap position -> td error
  std::vector<int32_t> b2h;  // buffer position -> heap position (0: none)
  int32_t size = 0;          // len(priority_heap)
  int32_t position = 1;      // next buffer position (1-based, utils.py:99-100)
  bool full = false;
  int32_t n_parts = 0;       // len(self.partitions)
  bool parts_fixed = false;
  std::vector<int32_t> bounds;  // partition boundaries: n_parts + 1 ranks
  std::vector<double> probs;    // probability of rank r at probs[r - 1]
  uint64_t rng_state = 0x9E3779B97F4A7C15ull;
};

namespace {

// torch's float32 `tensor.pow(python_float)` (utils.py:266): the exponent rounded to float32; 0.5, 2, 3,
// -0.5, -1, -2 are sqrt / square / cube / 1/sqrt / reciprocal / 1/square in float32, any other exponent a
// float32 pow (correctly rounded here; torch's vectorised powf agrees to 1 ulp).
float torch_pow_f32(float x, double exponent) {
  const float e = (float)exponent;
  if (e == 0.5f) return std::sqrt(x);
  if (e == 2.0f) return x * x;
  if (e == 3.0f) return x * x * x;
  if (e == -0.5f) return 1.0f / std::sqrt(x);
  if (e == -1.0f) return 1.0f / x;
  if (e == -2.0f) return 1.0f / (x * x);
  return (float)std::pow((double)x, (double)e);
}

void put(eco_per* p, int32_t h, int32_t b, double t) {  // __update_heap (utils.py:144-149)
  if (h > p->size) p->size = h;
  p->bp[h] = b;
  p->td[h] = t;
  p->b2h[b] = h;
}

void swap_pos(eco_per* p, int32_t i, int32_t j) {
  const int32_t bi = p->bp[i], bj = p->bp[j];
  const double ti = p->td[i], tj = p->td[j];
  put(p, i, bj, tj);
  put(p, j, bi, ti);
}

void up_heap(eco_per* p, int32_t i) {  // utils.py:151-162
  while (i >= 2) {
    const int32_t par = i / 2;
    if (!(p->td[par] < p->td[i])) return;
    swap_pos(p, i, par);
    i = par;
  }
}

void down_heap(eco_per* p, int32_t i) {  // utils.py:164-183 (children must be < size, not <=)
  const int32_t size = p->full ? p->capacity : p->size;
  for (;;) {
    int32_t largest = i;
    const int64_t l = 2 * (int64_t)i, r = l + 1;
    if (l < size && p->td[l] > p->td[largest]) largest = (int32_t)l;
    if (r < size && p->td[r] > p->td[largest]) largest = (int32_t)r;
    if (largest == i) return;
    swap_pos(p, i, largest);
    i = largest;
  }
}

// update_partitions (utils.py:204-232): P(rank) = rank^-alpha / sum, summed in rank order like the
// reference's sum(); boundaries where the running sum first reaches k / num_partitions.
int make_partitions(eco_per* p, int32_t num) {
  const int32_t n = p->size;
  p->probs.assign(n, 0.0);
  double s = 0.0;
  for (int32_t r = 1; r <= n; ++r) {
    p->probs[r - 1] = std::pow((double)r, -p->alpha);
    s += p->probs[r - 1];
  }
  for (int32_t r = 0; r < n; ++r) p->probs[r] /= s;
  p->bounds.assign(1, 1);
  int32_t k = 1, rank = 1;
  double cum = 0.0, next = (double)k / (double)num;
  while (k < num) {
    if (rank > n) return fail(ECO_ERR_KEY, "prioritised replay: partition rank past the heap (KeyError)");
    cum += p->probs[rank - 1];
    ++rank;
    if (cum >= next) {
      p->bounds.push_back(rank);
      ++k;
      next = (double)k / (double)num;
    }
  }
  p->bounds.push_back(n);
  p->n_parts = num;
  return ECO_OK;
}

uint64_t next_u64(uint64_t& s) {  // splitmix64 (ranks drawn natively when the caller injects none)
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

extern "C" eco_per* eco_per_create(int32_t capacity, double alpha, double beta0) {
  if (capacity < 1) {
    set_error("prioritised replay: capacity must be >= 1");
    return nullptr;
  }
  eco_per* p = new eco_per();
  p->capacity = capacity;
  p->alpha = alpha;
  p->beta = beta0;
  p->beta_step = 0.0;
  p->bp.assign((size_t)capacity + 1, 0);
  p->td.assign((size_t)capacity + 1, 0.0);
  p->b2h.assign((size_t)capacity + 1, 0);
  return p;
}

extern "C" void eco_per_destroy(eco_per* p) { delete p; }

extern "C" int32_t eco_per_len(const eco_per* p) { return p->size; }

extern "C" double eco_per_beta(const eco_per* p) { return p->beta; }

extern "C" int eco_per_full(const eco_per* p) { return p->full ? 1 : 0; }

extern "C" int eco_per_configure_beta_anneal_time(eco_per* p, double beta_max_at_samples) {
  if (!(beta_max_at_samples != 0.0)) return fail(ECO_ERR_ARG, "prioritised replay: beta_max_at_samples must be nonzero");
  p->beta_step = (1.0 - p->beta) / beta_max_at_samples;  // utils.py:275-276
  return ECO_OK;
}

// `n` consecutive add() calls (utils.py:120-142): each new transition gets td error 1 (the reference's
// __get_max_td_err reads heap position 0, which is never filled) and the next buffer position; the buffer
// positions written are returned in order (slot = position - 1 in the transition ring).
extern "C" int eco_per_add(eco_per* p, int32_t n, int32_t* buffer_positions) {
  if (n < 0) return fail(ECO_ERR_ARG, "prioritised replay: negative add count");
  for (int32_t k = 0; k < n; ++k) {
    const int32_t b = p->position;
    int32_t h = p->b2h[b];
    if (h != 0) p->full = true;
    else h = b;
    put(p, h, b, 1.0);
    up_heap(p, h);
    if (p->full) down_heap(p, h);
    if (buffer_positions) buffer_positions[k] = b;
    p->position = (p->position % p->capacity) + 1;
  }
  return ECO_OK;
}

// update_priorities (utils.py:234-240), in the order given.
extern "C" int eco_per_update_priorities(eco_per* p, int32_t n, const int32_t* buffer_positions,
                                         const double* td_errors) {
  for (int32_t k = 0; k < n; ++k) {
    const int32_t b = buffer_positions[k];
    if (b < 1 || b > p->capacity || p->b2h[b] == 0)
      return fail(ECO_ERR_KEY, "prioritised replay: buffer position not in the heap (KeyError)");
    const int32_t h = p->b2h[b];
    p->td[h] = td_errors[k];
    down_heap(p, h);
    up_heap(p, h);
  }
  return ECO_OK;
}

// rebalance (utils.py:185-202): stable sort by td error, descending, refill positions 1..capacity, then
// down_heap(i) for i = capacity/2 .. 2 (position 1 is not revisited, as in the reference).
extern "C" int eco_per_rebalance(eco_per* p) {
  if (p->size < p->capacity) return fail(ECO_ERR_INDEX, "prioritised replay: rebalance of a heap that is not full (IndexError)");
  std::vector<int32_t> order(p->size);
  for (int32_t i = 0; i < p->size; ++i) order[i] = i + 1;
  std::stable_sort(order.begin(), order.end(), [p](int32_t a, int32_t b) { return p->td[a] > p->td[b]; });
  std::vector<int32_t> nb(p->size);
  std::vector<double> nt(p->size);
  for (int32_t i = 0; i < p->size; ++i) {
    nb[i] = p->bp[order[i]];
    nt[i] = p->td[order[i]];
  }
  std::fill(p->b2h.begin(), p->b2h.end(), 0);
  for (int32_t i = 0; i < p->capacity; ++i) put(p, i + 1, nb[i], nt[i]);
  for (int32_t i = p->capacity / 2; i > 1; --i) down_heap(p, i);
  return ECO_OK;
}

// sample (utils.py:242-273) minus the transition gather, in two halves so a caller can draw the ranks with
// the reference's own RNG between them:
//   begin  -- the partitions, recomputed unless fixed (they are fixed once the heap is full and the batch
//             size is unchanged); bounds[batch + 1] (nullable) receives the partition boundaries, partition
//             k being the ranks [bounds[k], bounds[k + 1]);
//   finish -- beta annealed, one rank per partition (`ranks` injected: the reference's
//             np.random.randint(low, high) draws; NULL: drawn here from `seed`), and per sample the buffer
//             position and the float32 importance weight (N p)^-beta / max.  ranks_out is nullable.
extern "C" int eco_per_sample_begin(eco_per* p, int32_t batch, int32_t* bounds) {
  if (batch < 1) return fail(ECO_ERR_ARG, "prioritised replay: batch size must be >= 1");
  if (p->size < 1) return fail(ECO_ERR_KEY, "prioritised replay: sample from an empty heap (KeyError)");
  if (batch != p->n_parts || !p->parts_fixed) {
    const int rc = make_partitions(p, batch);
    if (rc != ECO_OK) return rc;
    if (p->full) p->parts_fixed = true;
  }
  if (bounds)
    for (int32_t k = 0; k <= batch; ++k) bounds[k] = p->bounds[k];
  return ECO_OK;
}

extern "C" int eco_per_sample_finish(eco_per* p, int32_t batch, const int64_t* ranks, uint64_t seed,
                                     int32_t* buffer_positions, float* weights, int64_t* ranks_out) {
  if (batch != p->n_parts || (int32_t)p->bounds.size() != batch + 1)
    return fail(ECO_ERR_ARG, "prioritised replay: sample_finish without a matching sample_begin");
  for (int32_t k = 0; k < batch; ++k) {  // validate everything before any state changes
    const int64_t lo = p->bounds[k], hi = p->bounds[k + 1];
    if (ranks ? (ranks[k] < lo || ranks[k] >= hi) : hi <= lo)
      return fail(ECO_ERR_ARG, "prioritised replay: empty partition or injected rank outside its partition");
    if ((ranks ? ranks[k] : hi - 1) > p->size) return fail(ECO_ERR_KEY, "prioritised replay: rank outside the heap (KeyError)");
  }
  p->beta = std::min(p->beta + p->beta_step, 1.0);
  uint64_t s = seed ^ p->rng_state;
  p->rng_state = next_u64(s);
  const float nf = (float)(p->full ? p->capacity : p->size);
  float wmax = 0.f;
  for (int32_t k = 0; k < batch; ++k) {
    const int64_t lo = p->bounds[k], hi = p->bounds[k + 1];
    const int64_t r = ranks ? ranks[k] : lo + (int64_t)(next_u64(s) % (uint64_t)(hi - lo));
    if (ranks_out) ranks_out[k] = r;
    buffer_positions[k] = p->bp[r];
    const float w = torch_pow_f32(nf * (float)p->probs[r - 1], -p->beta);
    weights[k] = w;
    wmax = std::max(wmax, w);
  }
  for (int32_t k = 0; k < batch; ++k) weights[k] /= wmax;
  return ECO_OK;
}

extern "C" int eco_per_sample(eco_per* p, int32_t batch, const int64_t* ranks, uint64_t seed, int32_t* buffer_positions,
                              float* weights, int64_t* ranks_out) {
  const int rc = eco_per_sample_begin(p, batch, nullptr);
  if (rc != ECO_OK) return rc;
  return eco_per_sample_finish(p, batch, ranks, seed, buffer_positions, weights, ranks_out);
}

// Introspection for tests and callers: the heap (positions 1..len) and the current partitions.
extern "C" int eco_per_heap(const eco_per* p, int32_t* buffer_positions, double* td_errors) {
  for (int32_t h = 1; h <= p->size; ++h) {
    buffer_positions[h - 1] = p->bp[h];
    td_errors[h - 1] = p->td[h];
  }
  return ECO_OK;
}

extern "C" int32_t eco_per_partitions(const eco_per* p, int32_t* bounds, double* probs) {
  if (bounds)
    for (size_t i = 0; i < p->bounds.size(); ++i) bounds[i] = p->bounds[i];
  if (probs)
    for (size_t i = 0; i < p->probs.size(); ++i) probs[i] = p->probs[i];
  return p->n_parts;
}

// ---------------------------------------------------------------------------------------- device gather ----
// The sampled transitions out of the fp32 feature ring (eco_replay) by explicit slot: one workgroup per
// sample, float4 copies of the s / s' node-feature rows (HBM-bound: 2 x N x x_stride x 4 B per sample).
__global__ __launch_bounds__(256) void replay_gather_kernel(eco_replay rb, int M, const int32_t* slots, float* xs,
                                                           float* xn, int32_t* gid, int32_t* act, float* rew,
                                                           float* done) {
  const int m = blockIdx.x;
  if (m >= M) return;
  const int xst = rb.x_stride == 16 ? 16 : 8;
  const int slot = slots[m];
  if (slot < 0 || slot >= rb.capacity) return;  // rejected on the host; never read outside the ring
  const int per = rb.n_spins * xst / 4;
  const float4* s4 = reinterpret_cast<const float4*>(rb.xs + (size_t)slot * rb.n_spins * xst);
  const float4* n4 = reinterpret_cast<const float4*>(rb.xn + (size_t)slot * rb.n_spins * xst);
  float4* ds = reinterpret_cast<float4*>(xs + (size_t)m * rb.n_spins * xst);
  float4* dn = reinterpret_cast<float4*>(xn + (size_t)m * rb.n_spins * xst);
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    ds[i] = s4[i];
    dn[i] = n4[i];
  }
  if (threadIdx.x == 0) {
    gid[m] = rb.gid[slot];
    act[m] = rb.act[slot];
    rew[m] = rb.rew[slot];
    done[m] = rb.done[slot];
  }
}

// slots: DEVICE int32 [m], each in [0, capacity) (host-checked by the Python wrapper from the buffer
// positions eco_per_sample returned).
extern "C" int eco_replay_gather(const eco_replay* rb, int32_t m, const int32_t* slots, float* xs, float* xn,
                                 int32_t* graph_ids, int32_t* actions, float* rewards, float* dones,
                                 eco_stream_t stream) {
  if (m < 0 || rb->capacity < 1) return fail(ECO_ERR_ARG, "replay gather: bad size");
  if (m == 0) return ECO_OK;
  replay_gather_kernel<<<m, 256, 0, (hipStream_t)stream>>>(*rb, m, slots, xs, xn, graph_ids, actions, rewards, dones);
  return check_launch("replay_gather");
}
