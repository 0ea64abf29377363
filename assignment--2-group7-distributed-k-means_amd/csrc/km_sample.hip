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

__global__ __launch_bounds__(64) void k_bernoulli(const uint64_t* __restrict__ seeds,
                                                  const int64_t* __restrict__ sizes,
                                                  const int64_t* __restrict__ bases, double fraction,
                                                  int64_t* __restrict__ out, int cp, int32_t* __restrict__ counts) {
  __shared__ uint32_t mt[624];
  __shared__ uint32_t T[624];
  const int p = blockIdx.x;
  const int lane = threadIdx.x;
  const uint64_t a = seeds[p];
  const int64_t size = sizes[p], base = bases[p];
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
      if (idx < cp) out[(size_t)p * cp + idx] = base + r;
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
  if (lane == 0) counts[p] = cnt;
}

}  // namespace

hipError_t launch_bernoulli(const uint64_t* seeds, const int64_t* sizes, const int64_t* bases, int nparts,
                            double fraction, int64_t* out, int cp, int32_t* counts, hipStream_t s) {
  if (nparts <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bernoulli, dim3(nparts), dim3(64), 0, s, seeds, sizes, bases, fraction, out, cp, counts);
  return hipGetLastError();
}

}  // namespace km
