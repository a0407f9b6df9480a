"""CPU restatement of the reference's rank-based PrioritisedReplayBuffer
(src/agents/dqn/utils.py:86-277).  TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the
native heap (eco_per_* in include/eco_hip.h); nothing in eco-dqn_amd/ imports it.

Pinned against the reference itself: tests/golden/make_per_golden.py runs the reference class through a
scripted sequence of add / update_priorities / sample / rebalance calls and records the heap after every
call (tests/golden/per.npz); tests/test_per_cpu.py replays the script here and on the native heap.

The heap is kept as two flat lists indexed by heap position (1-based, slot 0 unused) instead of the
reference's dict of [buffer_position, td_error, transition]; the transition itself is not part of the
ordering and lives elsewhere (in the product: a device ring indexed by buffer position - 1).
"""
import math

import numpy as np


def torch_pow_f32(x, exponent):
    """torch's float32 `tensor.pow(python_float)`: the exponent is rounded to float32; the exponents
    0.5, 2, 3, -0.5, -1, -2 take sqrt / square / cube / 1/sqrt / reciprocal / 1/square in float32;
    any other is pow with a float32 result (computed here correctly rounded from float64; torch's
    vectorised powf agrees to 1 ulp)."""
    x = np.asarray(x, np.float32)
    e = np.float32(exponent)
    one = np.float32(1)
    special = {0.5: lambda v: np.sqrt(v), 2.0: lambda v: v * v, 3.0: lambda v: v * v * v,
               -0.5: lambda v: one / np.sqrt(v), -1.0: lambda v: one / v, -2.0: lambda v: one / (v * v)}
    if float(e) in special:
        return special[float(e)](x).astype(np.float32)
    return np.power(x.astype(np.float64), np.float64(e)).astype(np.float32)


class PEROracle:
    def __init__(self, capacity=10000, alpha=0.7, beta0=0.5):  # utils.py:88-111
        self.capacity = capacity
        self.bp = [0] * (capacity + 1)      # heap position -> buffer position
        self.td = [0.0] * (capacity + 1)    # heap position -> td error (priority key)
        self.size = 0                       # len(priority_heap)
        self.b2h = {}                       # buffer position -> heap position
        self.position = 1
        self.full = False
        self.alpha = alpha
        self.beta = beta0
        self.beta_step = 0
        self.partitions = []
        self.probabilities = {}
        self.fixed = False

    def _max_td(self):
        # utils.py:113-118: reads heap position 0, which never exists -> always 1
        return 1

    def _set(self, pos, bp, td):  # utils.py:144-149
        if pos > self.size:
            self.size = pos
        self.bp[pos] = bp
        self.td[pos] = td
        self.b2h[bp] = pos

    def _swap(self, i, j):
        bi, ti, bj, tj = self.bp[i], self.td[i], self.bp[j], self.td[j]
        self._set(i, bj, tj)
        self._set(j, bi, ti)

    def add(self):  # utils.py:120-142; returns the buffer position written
        bp = self.position
        heap_pos = self.b2h.get(bp)
        if heap_pos is not None:
            self.full = True
        else:
            heap_pos = bp
        self._set(heap_pos, bp, self._max_td())
        self.up_heap(heap_pos)
        if self.full:
            self.down_heap(heap_pos)
        self.position = (self.position % self.capacity) + 1
        return bp

    def up_heap(self, i):  # utils.py:151-162
        while i >= 2:
            p = i // 2
            if self.td[p] < self.td[i]:
                self._swap(i, p)
                i = p
            else:
                break

    def down_heap(self, i):  # utils.py:164-183 (strict `< size`: heap position `size` is never a child)
        size = self.capacity if self.full else self.size
        while True:
            largest, left, right = i, 2 * i, 2 * i + 1
            if left < size and self.td[left] > self.td[largest]:
                largest = left
            if right < size and self.td[right] > self.td[largest]:
                largest = right
            if largest == i:
                return
            self._swap(i, largest)
            i = largest

    def rebalance(self):  # utils.py:185-202 (needs a full heap: sort_array[count-1] for count <= capacity)
        if self.size < self.capacity:
            raise IndexError("list index out of range")
        items = sorted(zip(self.bp[1:self.size + 1], self.td[1:self.size + 1]), key=lambda x: x[1], reverse=True)
        self.b2h = {}
        for k, (b, t) in enumerate(items[:self.capacity], start=1):
            self._set(k, b, t)
        for i in range(self.capacity // 2, 1, -1):
            self.down_heap(i)

    def update_partitions(self, num_partitions):  # utils.py:204-232
        n = self.size
        pr = [math.pow(rank, -self.alpha) for rank in range(1, n + 1)]
        s = sum(pr)
        probs = {r + 1: p / s for r, p in enumerate(pr)}
        parts = [1]
        k = 1
        cum = 0
        nxt = k / num_partitions
        rank = 1
        while k < num_partitions:
            cum += probs[rank]
            rank += 1
            if cum >= nxt:
                parts.append(rank)
                k += 1
                nxt = k / num_partitions
        parts.append(n)
        return list(zip(parts, parts[1:])), probs

    def update_priorities(self, buffer_positions, td_errors):  # utils.py:234-240
        for b, t in zip(buffer_positions, td_errors):
            h = self.b2h[b]
            self.td[h] = float(t)
            self.down_heap(h)
            self.up_heap(h)

    def sample(self, batch_size, ranks=None):  # utils.py:242-273 (ranks injected or drawn like the reference)
        if batch_size != len(self.partitions) or not self.fixed:
            self.partitions, self.probabilities = self.update_partitions(batch_size)
            if self.full:
                self.fixed = True
        self.beta = min(self.beta + self.beta_step, 1)
        if ranks is None:
            ranks = [np.random.randint(lo, hi) for lo, hi in self.partitions]
        bps = [self.bp[r] for r in ranks]
        n = self.capacity if self.full else self.size
        p = np.array([self.probabilities[r] for r in ranks], dtype=np.float32)
        w = torch_pow_f32(np.float32(n) * p, -self.beta)    # utils.py:266 (N * FloatTensor).pow(-beta)
        w = w / w.max()
        return list(ranks), bps, w

    def configure_beta_anneal_time(self, beta_max_at_samples):  # utils.py:275-276
        self.beta_step = (1 - self.beta) / beta_max_at_samples

    def heap(self):
        return np.array(self.bp[1:self.size + 1]), np.array(self.td[1:self.size + 1])

    def __len__(self):
        return self.size
