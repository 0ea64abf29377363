// Bernoulli pass of rdd.takeSample(False, num, seed) on the GPU
// (kmeans_spark.py:72 initial centroids, :196 empty-cluster replacement).
//
// PySpark's takeSample (RDD.takeSample + RDDSampler, restated host-side in
// sampling.py) keeps row i of partition p when u_i < fraction, u_i the i-th
// double of Python's random.Random(seed ^ p) after ten randint(0, 1) warm-up
// draws.  That stream is MT19937 (init_by_array seeding, genrand_res53
// doubles), one independent stream per partition.  Here one wave owns one
// partition: lane 0 seeds the state, the wave twists 624 words at a time in
// three dependency phases (the twist reads only old words in [0, 227), then
// words of the earlier phase), tempers them into LDS, and lanes test 64 rows
// per step; picks are appended in row order with a ballot prefix.  The
// result is identical to the host restatement (tests/test_gpu_sampling.py).
#include "km_internal.h"

namespace km {

namespace {

constexpr uint32_t MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu, MT_MATRIX = 0x9908b0dfu;

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far) {
  const uint32_t y = (cur & MT_UPPER) | (nxt & MT_LOWER);
  return far ^ (y >> 1) ^ ((y & 1u) ? MT_MATRIX : 0u);
}

// One partition's Bernoulli pass by one wave (64 threads): global row
// indices base + i of the rows kept, in row order, into out[0..cp); the
// number kept (possibly > cp: the caller checks) into *count.
__device__ void bernoulli_partition(uint64_t a, int64_t size, int64_t base, double fraction, int64_t* __restrict__ out,
                                    int cp, int32_t* __restrict__ count) {
  __shared__ uint32_t mt[624];
  __shared__ uint32_t T[624];
  const int lane = threadIdx.x;
  if (lane == 0) {
    // init_genrand(19650218) + init_by_array(key): the key is |seed| in
    // 32-bit words, least significant first (CPython random_seed)
    const uint32_t key[2] = {(uint32_t)a, (uint32_t)(a >> 32)};
    const int kl = (a >> 32) ? 2 : 1;
    mt[0] = 19650218u;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    int i = 1, j = 0;
    for (int k = 624 > kl ? 624 : kl; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      ++i;
      ++j;
      if (i >= 624) {
        mt[0] = mt[623];
        i = 1;
      }
      if (j >= kl) j = 0;
    }
    for (int k = 623; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      ++i;
      if (i >= 624) {
        mt[0] = mt[623];
        i = 1;
      }
    }
    mt[0] = 0x80000000u;
  }
  __syncthreads();

  auto twist = [&]() {
    uint32_t v[4];
    // [0, 227): old words only
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int i = lane + 64 * m;
      if (i < 227) v[m] = mt_mix(mt[i], mt[i + 1], mt[i + 397]);
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int i = lane + 64 * m;
      if (i < 227) mt[i] = v[m];
    }
    __syncthreads();
    // [227, 454): new words [0, 227)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int i = 227 + lane + 64 * m;
      if (i < 454) v[m] = mt_mix(mt[i], mt[i + 1], mt[i - 227]);
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int i = 227 + lane + 64 * m;
      if (i < 454) mt[i] = v[m];
    }
    __syncthreads();
    // [454, 623): new words [227, 396)
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int i = 454 + lane + 64 * m;
      if (i < 623) v[m] = mt_mix(mt[i], mt[i + 1], mt[i - 227]);
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int i = 454 + lane + 64 * m;
      if (i < 623) mt[i] = v[m];
    }
    __syncthreads();
    if (lane == 0) mt[623] = mt_mix(mt[623], mt[0], mt[396]);
    __syncthreads();
    for (int i = lane; i < 624; i += 64) {
      uint32_t y = mt[i];
      y ^= y >> 11;
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= y >> 18;
      T[i] = y;
    }
    __syncthreads();
  };

  int pos = 624;  // next unused tempered word of T (624: twist first)
  // RDDSampler warm-up: ten randint(0, 1) = getrandbits(2) with rejection
  for (int accepted = 0; accepted < 10;) {
    if (pos == 624) {
      twist();
      pos = 0;
    }
    if ((T[pos++] >> 30) < 2u) ++accepted;
  }
  const uint64_t below = (1ull << lane) - 1ull;
  int cnt = 0;
  int64_t row = 0;
  bool carry_on = false;
  uint32_t carry = 0;
  auto take = [&](bool hit, int64_t r) {
    const uint64_t m = __ballot(hit);
    if (hit) {
      const int idx = cnt + __popcll(m & below);
      if (idx < cp) out[idx] = base + r;
    }
    cnt += __popcll(m);
  };
  while (row < size) {
    if (pos == 624) {
      twist();
      pos = 0;
    }
    if (carry_on) {  // a row whose first word ended the previous block
      const uint32_t w0 = carry, w1 = T[pos++];
      const double u = ((double)(w0 >> 5) * 67108864.0 + (double)(w1 >> 6)) * (1.0 / 9007199254740992.0);
      take(lane == 0 && u < fraction, row);
      ++row;
      carry_on = false;
      continue;
    }
    const int64_t nr = min((int64_t)((624 - pos) / 2), size - row);
    for (int64_t q0 = 0; q0 < nr; q0 += 64) {
      const int64_t q = q0 + lane;
      bool hit = false;
      if (q < nr) {
        const uint32_t w0 = T[pos + 2 * q], w1 = T[pos + 2 * q + 1];
        const double u = ((double)(w0 >> 5) * 67108864.0 + (double)(w1 >> 6)) * (1.0 / 9007199254740992.0);
        hit = u < fraction;
      }
      take(hit, row + q);
    }
    row += nr;
    pos += 2 * (int)nr;
    if (row < size && pos == 623) {
      carry = T[623];
      carry_on = true;
      pos = 624;
    }
  }
  if (lane == 0) *count = cnt;
}

__global__ __launch_bounds__(64) void k_bernoulli(const uint64_t* __restrict__ seeds,
                                                  const int64_t* __restrict__ sizes,
                                                  const int64_t* __restrict__ bases, double fraction,
                                                  int64_t* __restrict__ out, int cp, int32_t* __restrict__ counts) {
  const int p = blockIdx.x;
  bernoulli_partition(seeds[p], sizes[p], bases[p], fraction, out + (size_t)p * cp, cp, counts + p);
}

// ---------------------------------------------------------------------------
// Empty-cluster repair on the device (kmeans_spark.py:191-204), inside a
// batch, single rank: rdd.takeSample(False, n_empty, seed = int(time.time()))
// restated as PySpark + CPython do it (sampling.py is the host restatement):
//   fraction = _computeFractionForSampleSize(num, total)      (each pass)
//   picks    = Bernoulli pass, partition p seeded seed ^ p    (k_rep_bernoulli)
//   while len(picks) < num: retry   (p < 5e-5: the batch stops, the host repairs)
//   rand.shuffle(picks); picks[:num]                          (k_rep_finish)
// with rand = random.Random(seed): CPython's MT19937 (init_by_array seeding,
// getrandbits, _randbelow), run by one thread.  The rows replace the empty
// clusters' new centroids in ascending cluster order; their shifts enter
// max_shift (L293-294), then the convergence / NaN decision.
// ---------------------------------------------------------------------------
__device__ void py_seed(uint32_t* __restrict__ mt, uint64_t a) {
  const uint32_t key[2] = {(uint32_t)a, (uint32_t)(a >> 32)};
  const int kl = (a >> 32) ? 2 : 1;
  mt[0] = 19650218u;
  for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  int i = 1, j = 0;
  for (int k = 624 > kl ? 624 : kl; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i;
    ++j;
    if (i >= 624) {
      mt[0] = mt[623];
      i = 1;
    }
    if (j >= kl) j = 0;
  }
  for (int k = 623; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= 624) {
      mt[0] = mt[623];
      i = 1;
    }
  }
  mt[0] = 0x80000000u;
}

__device__ uint32_t py_genrand(uint32_t* __restrict__ mt, int& idx) {
  if (idx >= 624) {
    int kk = 0;
    for (; kk < 624 - 397; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + 397]);
    for (; kk < 623; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + (397 - 624)]);
    mt[623] = mt_mix(mt[623], mt[0], mt[396]);
    idx = 0;
  }
  uint32_t y = mt[idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// CPython random.getrandbits(k), 1 <= k <= 64 (32-bit words, least significant first)
__device__ uint64_t py_getrandbits(uint32_t* __restrict__ mt, int& idx, int k) {
  if (k <= 32) return py_genrand(mt, idx) >> (32 - k);
  const uint64_t w0 = py_genrand(mt, idx);
  const uint64_t w1 = py_genrand(mt, idx) >> (64 - k);
  return w0 | (w1 << 32);
}

// CPython Random._randbelow_with_getrandbits(n), n >= 1
__device__ uint64_t py_randbelow(uint32_t* __restrict__ mt, int& idx, uint64_t n) {
  const int k = 64 - __clzll((long long)n);
  uint64_t r = py_getrandbits(mt, idx, k);
  while (r >= n) r = py_getrandbits(mt, idx, k);
  return r;
}

__device__ double take_sample_fraction(int64_t num, int64_t total, double neg_log_delta) {
#pragma clang fp contract(off)
  // PySpark RandomSampler: _computeFractionForSampleSize (no replacement)
  const double fraction = (double)num / (double)total;
  const double gamma = neg_log_delta / (double)total;
  const double f = fraction + gamma + sqrt(gamma * gamma + 2.0 * gamma * fraction);
  return f < 1.0 ? f : 1.0;
}

// Partition p's Bernoulli pass of the repair: a no-op unless this
// iteration's update left empty clusters (st->n_empty) and the gate is down.
__global__ __launch_bounds__(64) void k_rep_bernoulli(const int* __restrict__ gate, const DevStatus* __restrict__ st,
                                                      int64_t total, double neg_log_delta, uint64_t seed,
                                                      const int64_t* __restrict__ sizes,
                                                      const int64_t* __restrict__ bases, int64_t* __restrict__ picks,
                                                      int cp, int32_t* __restrict__ pcounts) {
  const int num = st->n_empty;
  if (*gate || num == 0 || (int64_t)num >= total) return;
  const int p = blockIdx.x;
  bernoulli_partition(seed ^ (uint64_t)p, sizes[p], bases[p], take_sample_fraction(num, total, neg_log_delta),
                      picks + (size_t)p * cp, cp, pcounts + p);
}

// The rest of the repair, one workgroup: the ascending list of the empty
// clusters, rand = random.Random(seed), the picks in partition order,
// rand.shuffle, the rows into the empty clusters, their shifts, and the
// convergence / NaN decision of the iteration.  A pass with too few picks
// (PySpark would retry with rand.randint(0, sys.maxsize); p < 5e-5 by the
// choice of fraction) or an overflowing partition stops the batch
// (KM_STOP_EMPTY) and the host repairs.
//
// rep_select: the common first part (returns false when the repair is not
// this launch's to do: gate raised, no empties, or a stop for the host).
// It leaves empty[0..num) and samples[0..num) (global rows) in place.
__device__ bool rep_select(const int* __restrict__ gate_ro, int* __restrict__ gate, DevStatus* __restrict__ st,
                           const int64_t* __restrict__ counts, int k, int64_t total, uint64_t seed, int nparts,
                           int cp, int32_t* __restrict__ pcounts, const int64_t* __restrict__ picks,
                           int64_t* __restrict__ samples, int32_t* __restrict__ empty, uint32_t* mt) {
  __shared__ int wsum[4];
  __shared__ int s_total, s_ok;
  const int num = st->n_empty;
  if (*gate_ro || num == 0) return false;
  const int t = threadIdx.x, nt = blockDim.x;
  if ((int64_t)num >= total) {  // takeSample's "every row" branch: left to the host
    if (t == 0) {
      st->stop = KM_STOP_EMPTY;
      *gate = KM_STOP_EMPTY;
    }
    return false;
  }
  // ascending list of the empty clusters (chunk per thread, block prefix)
  {
    const int chunk = (k + nt - 1) / nt;
    const int b0 = t * chunk;
    int v = 0;
    for (int i = 0; i < chunk; ++i)
      if (b0 + i < k && counts[b0 + i] == 0) ++v;
    const int lane = t & 63, w = t >> 6;
    int inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int run = inc - v;
    for (int i = 0; i < w; ++i) run += wsum[i];
    for (int i = 0; i < chunk; ++i)
      if (b0 + i < k && counts[b0 + i] == 0) empty[run++] = b0 + i;
  }
  if (t == 0) {
    int tot = 0, ovf = 0;
    for (int p = 0; p < nparts; ++p) {
      tot += pcounts[p];
      ovf |= pcounts[p] > cp;
    }
    s_total = tot;
    s_ok = (!ovf && tot >= num) ? 1 : 0;
  }
  __syncthreads();
  if (!s_ok) {
    if (t == 0) {
      st->stop = KM_STOP_EMPTY;
      *gate = KM_STOP_EMPTY;
    }
    __syncthreads();
    for (int p = t; p < nparts; p += nt) pcounts[p] = 0;
    return false;
  }
  if (t == 0) {
    // the picks in partition order (rows ascending within a partition), then
    // rand.shuffle (CPython: for i in reversed(range(1, n)): j = _randbelow(i + 1))
    int o = 0;
    for (int p = 0; p < nparts; ++p)
      for (int i = 0; i < pcounts[p]; ++i) samples[o++] = picks[(size_t)p * cp + i];
    py_seed(mt, seed);
    int idx = 624;
    for (int i = s_total - 1; i >= 1; --i) {
      const int j = (int)py_randbelow(mt, idx, (uint64_t)(i + 1));
      const int64_t tmp = samples[i];
      samples[i] = samples[j];
      samples[j] = tmp;
    }
  }
  __syncthreads();
  // the partition counters start at zero for the next repair
  for (int p = t; p < nparts; p += nt) pcounts[p] = 0;
  return true;
}

// rows rows[i] (i < num, from a device buffer or from X) replace the empty
// clusters empty[i] (L196-200); their shifts enter max_shift; then the
// convergence / NaN decision of the iteration
__device__ void rep_apply(int* __restrict__ gate, DevStatus* __restrict__ st, const int32_t* __restrict__ empty,
                          int num, int d, const double* __restrict__ C_old, double* __restrict__ C_new, double tol,
                          const int64_t* __restrict__ samples, const float* __restrict__ X, int64_t row0,
                          int64_t n_local, int dp, const double* __restrict__ rows) {
  __shared__ int s_nf;
  __shared__ unsigned long long s_max;
  const int t = threadIdx.x, nt = blockDim.x;
  if (t == 0) {
    s_nf = 0;
    s_max = 0ull;
  }
  __syncthreads();
  for (int i = t; i < num; i += nt) {
    const int j = empty[i];
    double sh = 0.0;
    int nf = 0;
    const int64_t r = rows ? 0 : samples[i] - row0;
    if (rows || (r >= 0 && r < n_local)) {
      for (int f = 0; f < d; ++f) {
        const double v = rows ? rows[(size_t)i * d + f] : (double)X[(size_t)r * dp + f];
        const double df = v - C_old[(size_t)j * d + f];
        C_new[(size_t)j * d + f] = v;
        sh = fma(df, df, sh);
        nf |= !isfinite(v);
      }
    } else {
      nf = 1;  // cannot happen with every row on this context (km_set_layout)
    }
    atomicMax(&s_max, (unsigned long long)__double_as_longlong(sh));
    if (nf) atomicOr(&s_nf, 1);
  }
  __syncthreads();
  if (t == 0) {
    const double ms = fmax(st->max_shift, sqrt(__longlong_as_double((long long)s_max)));
    st->max_shift = ms;
    st->nonfinite |= s_nf;
    int stop = 0;
    if (st->nonfinite)
      stop = KM_STOP_NONFINITE;
    else if (ms < tol)
      stop = KM_STOP_CONVERGED;
    st->stop = stop;
    st->repaired = 1;
    if (stop) *gate = stop;
  }
}

__global__ __launch_bounds__(256) void k_rep_finish(const int* __restrict__ gate_ro, int* __restrict__ gate,
                                                    DevStatus* __restrict__ st, const int64_t* __restrict__ counts,
                                                    int k, int64_t total, uint64_t seed, int nparts, int cp,
                                                    int32_t* __restrict__ pcounts, const int64_t* __restrict__ picks,
                                                    int64_t* __restrict__ samples, int32_t* __restrict__ empty,
                                                    const float* __restrict__ X, int64_t row0, int64_t n_local,
                                                    int d, int dp, const double* __restrict__ C_old,
                                                    double* __restrict__ C_new, double tol) {
  __shared__ uint32_t mt[624];
  if (!rep_select(gate_ro, gate, st, counts, k, total, seed, nparts, cp, pcounts, picks, samples, empty, mt)) return;
  rep_apply(gate, st, empty, st->n_empty, d, C_old, C_new, tol, samples, X, row0, n_local, dp, nullptr);
}

// Rows spread over ranks (km_set_layout mode 2): every rank runs the same
// Bernoulli passes over ALL partitions (index-level, seeded identically), so
// every rank picks the same rows; k_rep_pick writes the picked rows it holds
// into rows[i] and zeros for the others, the caller sum-all-reduces rows over
// the ranks (stream-ordered), and k_rep_apply puts them in place.  Exact: a
// row plus zeros is the row.
__global__ __launch_bounds__(256) void k_rep_pick(const int* __restrict__ gate_ro, int* __restrict__ gate,
                                                  DevStatus* __restrict__ st, const int64_t* __restrict__ counts,
                                                  int k, int64_t total, uint64_t seed, int nparts, int cp,
                                                  int32_t* __restrict__ pcounts, const int64_t* __restrict__ picks,
                                                  int64_t* __restrict__ samples, int32_t* __restrict__ empty,
                                                  const float* __restrict__ X, int64_t row0, int64_t n_local, int d,
                                                  int dp, double* __restrict__ rows, int32_t* __restrict__ pending) {
  __shared__ uint32_t mt[624];
  const bool go = rep_select(gate_ro, gate, st, counts, k, total, seed, nparts, cp, pcounts, picks, samples, empty, mt);
  if (threadIdx.x == 0) *pending = go ? st->n_empty : 0;
  if (!go) return;
  const int num = st->n_empty;
  for (int e = threadIdx.x; e < num * d; e += blockDim.x) {
    const int i = e / d, f = e - i * d;
    const int64_t r = samples[i] - row0;
    rows[e] = (r >= 0 && r < n_local) ? (double)X[(size_t)r * dp + f] : 0.0;
  }
}

__global__ __launch_bounds__(256) void k_rep_apply(int* __restrict__ gate, DevStatus* __restrict__ st,
                                                   const int32_t* __restrict__ empty, int d,
                                                   const double* __restrict__ C_old, double* __restrict__ C_new,
                                                   double tol, const double* __restrict__ rows,
                                                   const int32_t* __restrict__ pending) {
  const int num = *pending;  // 0: no repair this iteration (or a stop already raised)
  if (num == 0 || *gate) return;
  rep_apply(gate, st, empty, num, d, C_old, C_new, tol, nullptr, nullptr, 0, 0, 0, rows);
}

}  // namespace

hipError_t launch_repair(int* gate, const int64_t* counts, const Geometry& g, int64_t total, double neg_log_delta,
                         uint64_t seed, int32_t* empty, int32_t* pcounts, int64_t* picks, int64_t* samples, int cp,
                         const int64_t* sizes, const int64_t* bases, int nparts, const float* X, int64_t row0,
                         const double* C_old, double* C_new, DevStatus* st, double tol, hipStream_t s) {
  hipLaunchKernelGGL(k_rep_bernoulli, dim3(nparts), dim3(64), 0, s, gate, st, total, neg_log_delta, seed, sizes,
                     bases, picks, cp, pcounts);
  hipLaunchKernelGGL(k_rep_finish, dim3(1), dim3(256), 0, s, gate, gate, st, counts, g.k, total, seed, nparts, cp,
                     pcounts, picks, samples, empty, X, row0, g.n, g.d, g.dp, C_old, C_new, tol);
  return hipGetLastError();
}

hipError_t launch_repair_pick(int* gate, const int64_t* counts, const Geometry& g, int64_t total,
                              double neg_log_delta, uint64_t seed, int32_t* empty, int32_t* pcounts, int64_t* picks,
                              int64_t* samples, int cp, const int64_t* sizes, const int64_t* bases, int nparts,
                              const float* X, int64_t row0, DevStatus* st, double* rows, int32_t* pending,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_rep_bernoulli, dim3(nparts), dim3(64), 0, s, gate, st, total, neg_log_delta, seed, sizes,
                     bases, picks, cp, pcounts);
  hipLaunchKernelGGL(k_rep_pick, dim3(1), dim3(256), 0, s, gate, gate, st, counts, g.k, total, seed, nparts, cp,
                     pcounts, picks, samples, empty, X, row0, g.n, g.d, g.dp, rows, pending);
  return hipGetLastError();
}

hipError_t launch_repair_apply(int* gate, const Geometry& g, const int32_t* empty, const double* C_old,
                               double* C_new, DevStatus* st, double tol, const double* rows, const int32_t* pending,
                               hipStream_t s) {
  hipLaunchKernelGGL(k_rep_apply, dim3(1), dim3(256), 0, s, gate, st, empty, g.d, C_old, C_new, tol, rows, pending);
  return hipGetLastError();
}

hipError_t launch_bernoulli(const uint64_t* seeds, const int64_t* sizes, const int64_t* bases, int nparts,
                            double fraction, int64_t* out, int cp, int32_t* counts, hipStream_t s) {
  if (nparts <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bernoulli, dim3(nparts), dim3(64), 0, s, seeds, sizes, bases, fraction, out, cp, counts);
  return hipGetLastError();
}

}  // namespace km
