// HIP/CDNA4 (gfx950) kernels for the Lloyd-iteration hot path of
// kmeans_spark.py (reference: ersanjay16/Assignment--2-Group7-distributed-K-means).
//
// Exactness contract (DESIGN.md "Exactness"): a label is the reference's
//   np.argmin(np.linalg.norm(C - x, axis=1))          kmeans_spark.py:153-156
// computed in float64 with first-minimum tie-break.  The fast kernels only
// SCREEN candidates in fp32 / bf16x3; a rigorous per-point error bound decides
// whether the screened best is provably the float64 best, whether the top-2
// must be re-ranked in float64, or whether a full float64 scan is needed.
// Neither path ever returns a label the float64 argmin would not.
#include "km_internal.h"

#include <float.h>

namespace km {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

static constexpr float U24 = 5.9604644775390625e-08f;  // 2^-24, fp32 unit roundoff
static constexpr float U16 = 1.52587890625e-05f;       // 2^-16, bf16x2 split residual

__host__ __device__ inline int ceil_log2(int v) {
  int b = 0;
  while ((1 << b) < v) ++b;
  return b;
}

// top-3 smallest keys, k1 <= k2 <= k3 (v_min_f32 + 2x v_med3_f32)
__device__ __forceinline__ void top3_insert(float& k1, float& k2, float& k3, float v) {
  const float n1 = fminf(k1, v);
  const float n2 = __builtin_amdgcn_fmed3f(k1, k2, v);
  const float n3 = __builtin_amdgcn_fmed3f(k2, k3, v);
  k1 = n1;
  k2 = n2;
  k3 = n3;
}

__device__ __forceinline__ float key_of(float score, uint32_t idx, uint32_t mask) {
  return __uint_as_float((__float_as_uint(score) & ~mask) | idx);
}

// ||x - c||^2 in float64 (x fp32 row with stride, c float64 row)
__device__ inline double d2_exact(const float* __restrict__ x, const double* __restrict__ c, int d) {
  double s = 0.0;
  for (int f = 0; f < d; ++f) {
    const double t = (double)x[f] - c[f];
    s = fma(t, t, s);
  }
  return s;
}

// Full float64 scan, first minimum wins (np.argmin, kmeans_spark.py:156).
__device__ inline int exact_argmin(const float* __restrict__ x, const double* __restrict__ C64, int k, int d) {
  double best = d2_exact(x, C64, d);
  int lab = 0;
  for (int j = 1; j < k; ++j) {
    const double v = d2_exact(x, C64 + (size_t)j * d, d);
    if (v < best) {
      best = v;
      lab = j;
    }
  }
  return lab;
}

__device__ inline int exact_pick2(const float* __restrict__ x, const double* __restrict__ C64, int d, int a,
                                  int b) {
  const double va = d2_exact(x, C64 + (size_t)a * d, d);
  const double vb = d2_exact(x, C64 + (size_t)b * d, d);
  if (va < vb) return a;
  if (vb < va) return b;
  return a < b ? a : b;
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ inline float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------------------
// Centroid preparation: float64 centroids -> fp32 copy (direct screening),
// bf16 hi/lo split of -2c (MFMA screening), fp32 ||c||^2, max ||c||.
// Padded rows (k <= j < kp) are zero with ||c||^2 = 1e30 (never selected).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_prep_centroids(const double* __restrict__ C64, int k, int d, int dp,
                                                       float* __restrict__ C32, __bf16* __restrict__ Chi,
                                                       __bf16* __restrict__ Clo, float* __restrict__ cn2,
                                                       float* __restrict__ cmax) {
  const int j = blockIdx.x;
  const int lane = threadIdx.x;
  double nn = 0.0;
  for (int f = lane; f < dp; f += 64) {
    const double c = (j < k && f < d) ? C64[(size_t)j * d + f] : 0.0;
    nn = fma(c, c, nn);
    const float c32 = (float)c;
    C32[(size_t)j * dp + f] = c32;
    const float m2 = -2.0f * c32;
    const __bf16 hi = (__bf16)m2;
    const __bf16 lo = (__bf16)(m2 - (float)hi);
    Chi[(size_t)j * dp + f] = hi;
    Clo[(size_t)j * dp + f] = lo;
  }
  nn = wave_sum(nn);
  if (lane == 0) {
    cn2[j] = (j < k) ? (float)nn : 1e30f;
    if (j < k) {
      const float cn = sqrtf((float)nn) * 1.0001f + 1e-30f;
      atomicMax((unsigned int*)cmax, __float_as_uint(cn));
    }
  }
}

hipError_t launch_prep_centroids(const double* C64, const Geometry& g, float* C32, __bf16* Chi, __bf16* Clo,
                                 float* cn2, float* cmax, hipStream_t s) {
  hipError_t e = hipMemsetAsync(cmax, 0, sizeof(float), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_prep_centroids, dim3(g.kp), dim3(64), 0, s, C64, g.k, g.d, g.dp, C32, Chi, Clo, cn2, cmax);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Small k*d path (c1/c2 shapes).  One point per lane, centroids broadcast
// from LDS, direct-form fp32 distances (error relative to the distance
// itself), exact float64 re-rank in-thread when the bound cannot separate the
// candidates, fused partial statistics into an LDS float64 table replicated
// per lane (no same-address atomics inside a 32-lane group).
// ---------------------------------------------------------------------------
static constexpr int SMALL_MAX_K = 32;
static constexpr int SMALL_LDS = 60 * 1024;

template <int DP>
__global__ __launch_bounds__(256) void k_assign_small(const float* __restrict__ X, int64_t n, int d, int k,
                                                      const float* __restrict__ C32,
                                                      const double* __restrict__ C64,
                                                      const float* __restrict__ cmaxp, int32_t* __restrict__ labels,
                                                      double* __restrict__ stats, int fuse, int R) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sC = reinterpret_cast<float*>(smem);
  double* tab = reinterpret_cast<double*>(smem + ((k * DP * 4 + 15) / 16) * 16);
  const int d1 = d + 1;
  for (int i = threadIdx.x; i < k * DP; i += blockDim.x) sC[i] = C32[i];
  if (fuse)
    for (int i = threadIdx.x; i < k * d1 * R; i += blockDim.x) tab[i] = 0.0;
  __syncthreads();

  const int b = ceil_log2(k);
  const uint32_t mask = (1u << b) - 1u;
  const float cm = *cmaxp;
  // direct-form bound: |D~ - D| <= a*D~ + beta*sqrt(D~) + g0   (DESIGN.md), x2 safety
  const float alpha = 2.0f * (float)(DP + 6 + (2 << b)) * U24;
  const float beta = 2.0f * 2.5f * U24 * cm;
  const float g0 = 2.0f * 8.0f * U24 * U24 * cm * cm;
  const int rep = threadIdx.x & (R - 1);

  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < n;
       row += (int64_t)gridDim.x * blockDim.x) {
    const float* xr = X + row * DP;
    float x[DP];
#pragma unroll
    for (int f = 0; f < DP; f += 4) {
      const float4 v = *reinterpret_cast<const float4*>(xr + f);
      x[f] = v.x;
      x[f + 1] = v.y;
      x[f + 2] = v.z;
      x[f + 3] = v.w;
    }
    float k1 = FLT_MAX, k2 = FLT_MAX, k3 = FLT_MAX;
    for (int j = 0; j < k; ++j) {
      const float* c = sC + j * DP;
      float acc = 0.0f;
#pragma unroll
      for (int f = 0; f < DP; ++f) {
        const float t = x[f] - c[f];
        acc = fmaf(t, t, acc);
      }
      top3_insert(k1, k2, k3, key_of(acc, (uint32_t)j, mask));
    }
    int lab = (int)(__float_as_uint(k1) & mask);
    const int i2 = (int)(__float_as_uint(k2) & mask);
    const float B1 = alpha * k1 + beta * sqrtf(k1) + g0;
    const float B2 = alpha * k2 + beta * sqrtf(k2) + g0;
    const float B3 = alpha * k3 + beta * sqrtf(k3) + g0;
    const bool need_full = (k >= 3) && !((k3 > 64.0f * U24 * U24 * cm * cm) && (k3 - B3 > k1 + B1));
    const bool need_two = (k >= 2) && !(k2 - B2 > k1 + B1);
    if (need_full || need_two) {
      // exact float64 distances with the point held in registers
      double best = 0.0;
      int bl = -1;
      const int jn = need_full ? k : 2;
      for (int jj = 0; jj < jn; ++jj) {
        const int j = need_full ? jj : (jj == 0 ? (lab < i2 ? lab : i2) : (lab < i2 ? i2 : lab));
        const double* c = C64 + (size_t)j * d;
        double s = 0.0;
#pragma unroll
        for (int f = 0; f < DP; ++f) {
          if (f < d) {
            const double t = (double)x[f] - c[f];
            s = fma(t, t, s);
          }
        }
        if (bl < 0 || s < best) {
          best = s;
          bl = j;
        }
      }
      lab = bl;
    }
    if (lab >= k) lab = 0;  // only reachable with non-finite data (np.argmin of NaNs -> 0)
    labels[row] = lab;
    if (fuse) {
      double* t = tab + (size_t)lab * d1 * R + rep;
#pragma unroll
      for (int f = 0; f < DP; ++f)
        if (f < d) atomicAdd(t + (size_t)f * R, (double)x[f]);
      atomicAdd(t + (size_t)d * R, 1.0);
    }
  }
  if (fuse) {
    __syncthreads();
    for (int e = threadIdx.x; e < k * d1; e += blockDim.x) {
      double s = 0.0;
      for (int r = 0; r < R; ++r) s += tab[(size_t)e * R + r];
      if (s != 0.0) atomicAdd(stats + e, s);
    }
  }
}

static int small_replicas(const Geometry& g) {
  const size_t cbytes = ((size_t)g.k * g.dp * 4 + 15) / 16 * 16;
  int R = 32;
  while (R > 1 && cbytes + (size_t)g.k * (g.d + 1) * 8 * R > SMALL_LDS) R >>= 1;
  return R;
}

bool small_path_ok(const Geometry& g) {
  if (g.k > SMALL_MAX_K || g.dp > 64) return false;
  const size_t cbytes = ((size_t)g.k * g.dp * 4 + 15) / 16 * 16;
  return cbytes + (size_t)g.k * (g.d + 1) * 8 <= SMALL_LDS;
}

hipError_t launch_assign_small(const float* X, const Geometry& g, const float* C32, const double* C64,
                               const float* cmax, int32_t* labels, double* stats, int fuse, int n_cu,
                               hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  const int R = small_replicas(g);
  const size_t lds = ((size_t)g.k * g.dp * 4 + 15) / 16 * 16 + (fuse ? (size_t)g.k * (g.d + 1) * 8 * R : 0);
  int64_t blocks = (g.n + 255) / 256;
  const int64_t cap = (int64_t)n_cu * 4;
  if (blocks > cap) blocks = cap;
  switch (g.dp) {
    case 16:
      hipLaunchKernelGGL(k_assign_small<16>, dim3((unsigned)blocks), dim3(256), lds, s, X, g.n, g.d, g.k, C32, C64,
                         cmax, labels, stats, fuse, R);
      break;
    case 32:
      hipLaunchKernelGGL(k_assign_small<32>, dim3((unsigned)blocks), dim3(256), lds, s, X, g.n, g.d, g.k, C32, C64,
                         cmax, labels, stats, fuse, R);
      break;
    case 48:
      hipLaunchKernelGGL(k_assign_small<48>, dim3((unsigned)blocks), dim3(256), lds, s, X, g.n, g.d, g.k, C32, C64,
                         cmax, labels, stats, fuse, R);
      break;
    case 64:
      hipLaunchKernelGGL(k_assign_small<64>, dim3((unsigned)blocks), dim3(256), lds, s, X, g.n, g.d, g.k, C32, C64,
                         cmax, labels, stats, fuse, R);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// MFMA screening path (c3/c4/c5 shapes).
//
// scores S[j][p] = ||c_j||^2 - 2 c_j.x_p on v_mfma_f32_32x32x16_bf16 with a
// bf16x3 split (-2c = ch + cl, x = xh + xl; ch*xh + ch*xl + cl*xh), A operand
// = 32 centroids from LDS, B operand = 32 points held in registers, the
// accumulator initialised with ||c||^2.  C/D layout: column (point) on the
// lane, rows (centroids) in registers, so each lane keeps a running top-3 of
// (score | centroid index in the low mantissa bits) with min/med3.  The two
// lane halves hold disjoint centroid rows and are merged at the end.
// ---------------------------------------------------------------------------
static constexpr int MFMA_LDS_SMALL = 80 * 1024;   // 2+ workgroups of 4 waves per CU
static constexpr int MFMA_LDS_LARGE = 160 * 1024;  // 1 workgroup of 8 waves per CU

template <int NS>
__device__ __forceinline__ int phys_chunk(int c, int row) {
  constexpr int C = 2 * NS;  // 16-byte chunks per bf16 row
  if constexpr ((C & (C - 1)) == 0) {
    return c ^ ((row >> 1) & (C - 1));
  } else {
    return c;
  }
}

template <int NS, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_assign_mfma(const float* __restrict__ X, int64_t n, int k,
                                                              int kp, const __bf16* __restrict__ Chi,
                                                              const __bf16* __restrict__ Clo,
                                                              const float* __restrict__ cn2,
                                                              const float* __restrict__ cmaxp,
                                                              int32_t* __restrict__ labels, QEntry* __restrict__ queue,
                                                              uint32_t* __restrict__ qcount, int KC) {
  constexpr int DP = 16 * NS;
  constexpr int ROWB = DP * 2;  // bytes per bf16 row
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sHi = smem;
  char* sLo = smem + (size_t)KC * ROWB;
  float* sCn = reinterpret_cast<float*>(smem + 2 * (size_t)KC * ROWB);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int b = ceil_log2(kp);
  const uint32_t mask = (1u << b) - 1u;
  const float cm = *cmaxp;
  const int nchunks = (kp + KC - 1) / KC;
  const int64_t ntiles = (n + 31) / 32;
  const int64_t nwt = (ntiles + WAVES - 1) / WAVES;

  auto stage = [&](int ch) {
    const int kc = min(KC, kp - ch * KC);
    const int nc = kc * 2 * NS;
    const char* gh = reinterpret_cast<const char*>(Chi + (size_t)ch * KC * DP);
    const char* gl = reinterpret_cast<const char*>(Clo + (size_t)ch * KC * DP);
    for (int id = threadIdx.x; id < nc; id += WAVES * 64) {
      const int row = id / (2 * NS);
      const int c = id % (2 * NS);
      const size_t dst = (size_t)row * ROWB + (size_t)phys_chunk<NS>(c, row) * 16;
      *reinterpret_cast<uint4*>(sHi + dst) = *reinterpret_cast<const uint4*>(gh + (size_t)id * 16);
      *reinterpret_cast<uint4*>(sLo + dst) = *reinterpret_cast<const uint4*>(gl + (size_t)id * 16);
    }
    for (int id = threadIdx.x; id < kc; id += WAVES * 64) sCn[id] = cn2[(size_t)ch * KC + id];
  };

  if (nchunks == 1) {
    stage(0);
    __syncthreads();
  }

  for (int64_t wt = blockIdx.x; wt < nwt; wt += gridDim.x) {
    const int64_t tile = wt * WAVES + wave;
    if (nchunks == 1 && tile >= ntiles) break;  // no barriers below in this mode
    const int64_t row = tile * 32 + r;
    const bool valid = row < n;
    const int64_t rl = valid ? row : (n - 1);
    const float* xr = X + rl * DP + 8 * h;

    bf16x8 bh[NS], bl[NS];
    float xx = 0.0f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const float4 v0 = *reinterpret_cast<const float4*>(xr + 16 * s);
      const float4 v1 = *reinterpret_cast<const float4*>(xr + 16 * s + 4);
      const float xv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const __bf16 hi = (__bf16)xv[e];
        bh[s][e] = hi;
        bl[s][e] = (__bf16)(xv[e] - (float)hi);
        xx = fmaf(xv[e], xv[e], xx);
      }
    }
    xx += __shfl_xor(xx, 32);

    float k1 = FLT_MAX, k2 = FLT_MAX, k3 = FLT_MAX;
    for (int ch = 0; ch < nchunks; ++ch) {
      if (nchunks > 1) {
        __syncthreads();
        stage(ch);
        __syncthreads();
      }
      const int kc = min(KC, kp - ch * KC);
      for (int blk = 0; blk < kc / 32; ++blk) {
        f32x16 acc;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 cv = *reinterpret_cast<const float4*>(sCn + blk * 32 + 8 * g4 + 4 * h);
          acc[4 * g4 + 0] = cv.x;
          acc[4 * g4 + 1] = cv.y;
          acc[4 * g4 + 2] = cv.z;
          acc[4 * g4 + 3] = cv.w;
        }
        const int crow = blk * 32 + r;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const size_t off = (size_t)crow * ROWB + (size_t)phys_chunk<NS>(2 * s + h, crow) * 16;
          const bf16x8 ah = *reinterpret_cast<const bf16x8*>(sHi + off);
          const bf16x8 al = *reinterpret_cast<const bf16x8*>(sLo + off);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[s], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[s], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[s], acc, 0, 0, 0);
        }
        const uint32_t jb = (uint32_t)(ch * KC + blk * 32 + 4 * h);
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const uint32_t j = jb + (uint32_t)((reg & 3) + 8 * (reg >> 2));
          top3_insert(k1, k2, k3, key_of(acc[reg], j, mask));
        }
      }
    }
    if (nchunks > 1 && tile >= ntiles) continue;

    // merge the two lane halves (disjoint centroid rows of the same point)
    {
      const float p1 = __shfl_xor(k1, 32);
      const float p2 = __shfl_xor(k2, 32);
      const float p3 = __shfl_xor(k3, 32);
      top3_insert(k1, k2, k3, p1);
      top3_insert(k1, k2, k3, p2);
      top3_insert(k1, k2, k3, p3);
    }
    // rigorous screening bound on |S~ - S| (DESIGN.md "Exactness"), x2 safety
    const float xn = sqrtf(xx) * 1.0001f;
    const float B0 = 2.0f * ((6.5f * U16 + (float)(6 * DP + 8) * U24) * xn * cm +
                             (float)(3 * DP + 4) * U24 * cm * cm +
                             __builtin_ldexpf(1.0f, b - 23) * (cm * cm + 2.0f * xn * cm));
    const uint32_t i1 = __float_as_uint(k1) & mask;
    const uint32_t i2 = __float_as_uint(k2) & mask;
    // negated tests: a NaN (non-finite data) falls through to the full float64
    // scan, whose np.argmin semantics then pick the first index
    uint32_t kind = 0;
    if (!(k3 - k1 > 2.0f * B0))
      kind = 2;
    else if (!(k2 - k1 > 2.0f * B0))
      kind = 1;
    int lab = (i1 < (uint32_t)k) ? (int)i1 : 0;
    if (h == 0 && valid) labels[row] = lab;
    const bool enq = (h == 0) && valid && (kind != 0);
    const uint64_t m = __ballot(enq);
    if (m) {
      const int cnt = __popcll(m);
      const int leader = __ffsll((long long)m) - 1;
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(qcount, (uint32_t)cnt);
      base = __shfl(base, leader);
      if (enq) {
        const int pos = __popcll(m & ((1ull << lane) - 1ull));
        QEntry q;
        q.row = (uint32_t)row;
        q.i1 = i1;
        q.i2 = i2;
        q.kind = kind;
        queue[base + pos] = q;
        if (kind == 2) atomicAdd(qcount + 1, 1u);
      }
    }
  }
}

static int mfma_kc(const Geometry& g, int* waves) {
  const size_t per = (size_t)g.dp * 4 + 4;
  if ((size_t)g.kp * per <= MFMA_LDS_SMALL) {
    *waves = 4;
    return g.kp;
  }
  *waves = 8;
  if ((size_t)g.kp * per <= MFMA_LDS_LARGE) return g.kp;
  return (int)((MFMA_LDS_LARGE / per) / 32 * 32);
}

bool mfma_path_ok(const Geometry& g) {
  switch (g.dp) {
    case 16: case 32: case 48: case 64: case 96: case 128: case 192: case 256:
      return g.kp >= 32 && g.kp % 32 == 0 && g.kp <= (1 << 20);
    default:
      return false;
  }
}

template <int NS>
static void launch_mfma_ns(int waves, int blocks, size_t lds, hipStream_t s, const float* X, const Geometry& g,
                           const __bf16* Chi, const __bf16* Clo, const float* cn2, const float* cmax,
                           int32_t* labels, QEntry* queue, uint32_t* qcount, int KC) {
  if (waves == 4)
    hipLaunchKernelGGL((k_assign_mfma<NS, 4>), dim3(blocks), dim3(256), lds, s, X, g.n, g.k, g.kp, Chi, Clo, cn2,
                       cmax, labels, queue, qcount, KC);
  else
    hipLaunchKernelGGL((k_assign_mfma<NS, 8>), dim3(blocks), dim3(512), lds, s, X, g.n, g.k, g.kp, Chi, Clo, cn2,
                       cmax, labels, queue, qcount, KC);
}

hipError_t launch_assign_mfma(const float* X, const Geometry& g, const __bf16* Chi, const __bf16* Clo,
                              const float* cn2, const float* cmax, int32_t* labels, QEntry* queue,
                              uint32_t* qcount, int n_cu, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  int waves = 4;
  const int KC = mfma_kc(g, &waves);
  if (KC < 32) return hipErrorInvalidValue;
  const size_t lds = 2 * (size_t)KC * g.dp * 2 + (size_t)KC * 4;
  const int64_t ntiles = (g.n + 31) / 32;
  const int64_t nwt = (ntiles + waves - 1) / waves;
  const int per_cu = (waves == 4) ? (int)(MFMA_LDS_LARGE / lds > 4 ? 4 : MFMA_LDS_LARGE / lds) : 1;
  int64_t blocks = (int64_t)n_cu * (per_cu < 1 ? 1 : per_cu);
  if (blocks > nwt) blocks = nwt;
  const int nb = (int)blocks;
  switch (g.dp / 16) {
    case 1: launch_mfma_ns<1>(waves, nb, lds, s, X, g, Chi, Clo, cn2, cmax, labels, queue, qcount, KC); break;
    case 2: launch_mfma_ns<2>(waves, nb, lds, s, X, g, Chi, Clo, cn2, cmax, labels, queue, qcount, KC); break;
    case 3: launch_mfma_ns<3>(waves, nb, lds, s, X, g, Chi, Clo, cn2, cmax, labels, queue, qcount, KC); break;
    case 4: launch_mfma_ns<4>(waves, nb, lds, s, X, g, Chi, Clo, cn2, cmax, labels, queue, qcount, KC); break;
    case 6: launch_mfma_ns<6>(waves, nb, lds, s, X, g, Chi, Clo, cn2, cmax, labels, queue, qcount, KC); break;
    case 8: launch_mfma_ns<8>(waves, nb, lds, s, X, g, Chi, Clo, cn2, cmax, labels, queue, qcount, KC); break;
    case 12: launch_mfma_ns<12>(waves, nb, lds, s, X, g, Chi, Clo, cn2, cmax, labels, queue, qcount, KC); break;
    case 16: launch_mfma_ns<16>(waves, nb, lds, s, X, g, Chi, Clo, cn2, cmax, labels, queue, qcount, KC); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Exact float64 resolution of the queued ambiguous points.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_resolve(const float* __restrict__ X, int dp, int d, int k,
                                                 const double* __restrict__ C64, const QEntry* __restrict__ queue,
                                                 const uint32_t* __restrict__ qcount, int32_t* __restrict__ labels) {
  const uint32_t cnt = qcount[0];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
    const QEntry q = queue[i];
    const float* x = X + (size_t)q.row * dp;
    int lab;
    if (q.kind == 2 || q.i1 >= (uint32_t)k || q.i2 >= (uint32_t)k)
      lab = exact_argmin(x, C64, k, d);
    else
      lab = exact_pick2(x, C64, d, (int)q.i1, (int)q.i2);
    labels[q.row] = lab;
  }
}

hipError_t launch_resolve(const float* X, const Geometry& g, const double* C64, const QEntry* queue,
                          const uint32_t* qcount, int32_t* labels, int n_cu, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_resolve, dim3(n_cu * 2), dim3(256), 0, s, X, g.dp, g.d, g.k, C64, queue, qcount, labels);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Partial statistics (reduceByKey, kmeans_spark.py:169-173): per cluster
// sum of x and count, float64, into an LDS table; a workgroup owns a range of
// clusters (blockIdx.y) and a range of rows (blockIdx.x); one float64 global
// atomic per non-zero table entry at the end.
// ---------------------------------------------------------------------------
static constexpr int STATS_LDS = 156 * 1024;

__global__ __launch_bounds__(1024) void k_stats(const float* __restrict__ X, int64_t n, int d, int dp, int k,
                                                const int32_t* __restrict__ labels, double* __restrict__ stats,
                                                int kr, int64_t rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* tab = reinterpret_cast<double*>(smem);
  const int d1 = d + 1;
  const int c0 = blockIdx.y * kr;
  const int c1 = min(k, c0 + kr);
  const int nent = (c1 - c0) * d1;
  for (int i = threadIdx.x; i < nent; i += blockDim.x) tab[i] = 0.0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  int dpp = 1;
  while (dpp < d1) dpp <<= 1;
  if (dpp <= 64) {
    const int P = 64 / dpp;
    const int q = lane / dpp;
    const int f = lane % dpp;
    for (int64_t base = r0 + (int64_t)wave * P; base < r1; base += (int64_t)nwaves * P) {
      const int64_t row = base + q;
      if (row < r1 && f < d1) {
        const int lab = labels[row];
        if (lab >= c0 && lab < c1) {
          const float v = (f < d) ? X[row * dp + f] : 1.0f;
          atomicAdd(tab + (lab - c0) * d1 + f, (double)v);
        }
      }
    }
  } else {
    for (int64_t row = r0 + wave; row < r1; row += nwaves) {
      const int lab = labels[row];
      if (lab >= c0 && lab < c1) {
        double* t = tab + (lab - c0) * d1;
        for (int f = lane; f < d1; f += 64) {
          const float v = (f < d) ? X[row * dp + f] : 1.0f;
          atomicAdd(t + f, (double)v);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nent; i += blockDim.x) {
    const double v = tab[i];
    if (v != 0.0) atomicAdd(stats + (size_t)c0 * d1 + i, v);
  }
}

hipError_t launch_stats(const float* X, const Geometry& g, const int32_t* labels, double* stats, int n_cu,
                        hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  const int d1 = g.d + 1;
  int kr = (int)(STATS_LDS / ((size_t)d1 * 8));
  if (kr < 1) return hipErrorInvalidValue;
  if (kr > g.k) kr = g.k;
  const int ranges = (g.k + kr - 1) / kr;
  const size_t lds = (size_t)kr * d1 * 8;
  int per_cu = (int)((160 * 1024) / (lds + 1024));
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 2) per_cu = 2;
  int64_t bx = (int64_t)n_cu * per_cu / ranges;
  if (bx < 1) bx = 1;
  const int64_t min_rows = 2048;
  if (bx > (g.n + min_rows - 1) / min_rows) bx = (g.n + min_rows - 1) / min_rows;
  const int64_t rpb = (g.n + bx - 1) / bx;
  hipLaunchKernelGGL(k_stats, dim3((unsigned)bx, (unsigned)ranges), dim3(1024), lds, s, X, g.n, g.d, g.dp, g.k,
                     labels, stats, kr, rpb);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Centroid update (kmeans_spark.py:176-206 + 278-294): new = sum / count,
// empties keep the old centroid (host replaces them, L191-204), per-cluster
// squared shift, SSE via the closed form
//   SSE = sum_p ||x_p - mu||^2 - 2 sum_j (c_j - mu).(S_j - n_j mu) + sum_j n_j ||c_j - mu||^2
// with c_j the PRE-update centroids (L279 uses centroids_bc).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_update(const double* __restrict__ stats, const double* __restrict__ old,
                                               const double* __restrict__ mu, int k, int d,
                                               double* __restrict__ out, double* __restrict__ work,
                                               int64_t* __restrict__ counts) {
  const int j = blockIdx.x;
  const int lane = threadIdx.x;
  const int d1 = d + 1;
  const double cnt = stats[(size_t)j * d1 + d];
  double sh = 0.0, t = 0.0, nf = 0.0;
  for (int f = lane; f < d; f += 64) {
    const double S = stats[(size_t)j * d1 + f];
    const double o = old[(size_t)j * d + f];
    const double nv = (cnt > 0.0) ? S / cnt : o;
    out[(size_t)j * d + f] = nv;
    const double df = nv - o;
    sh = fma(df, df, sh);
    if (!isfinite(nv)) nf = 1.0;
    if (cnt > 0.0) {
      const double cmu = o - mu[f];
      t += -2.0 * cmu * (S - cnt * mu[f]) + cnt * cmu * cmu;
    }
  }
  sh = wave_sum(sh);
  t = wave_sum(t);
  nf = wave_sum(nf);
  if (lane == 0) {
    work[j] = sh;
    work[k + j] = t;
    work[2 * k + j] = nf;
    counts[j] = (int64_t)cnt;
  }
}

__global__ __launch_bounds__(256) void k_finalize(const double* __restrict__ work, const int64_t* __restrict__ counts,
                                                  int k, const double* __restrict__ sse_base,
                                                  const uint32_t* __restrict__ qcount, DevStatus* __restrict__ st) {
  __shared__ double s_max[256], s_sum[256];
  __shared__ int s_emp[256], s_nf[256];
  double mx = 0.0, sm = 0.0;
  int emp = 0, nf = 0;
  for (int j = threadIdx.x; j < k; j += 256) {
    mx = fmax(mx, work[j]);
    sm += work[k + j];
    nf |= (work[2 * k + j] != 0.0);
    emp += (counts[j] == 0);
  }
  s_max[threadIdx.x] = mx;
  s_sum[threadIdx.x] = sm;
  s_emp[threadIdx.x] = emp;
  s_nf[threadIdx.x] = nf;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      s_max[threadIdx.x] = fmax(s_max[threadIdx.x], s_max[threadIdx.x + o]);
      s_sum[threadIdx.x] += s_sum[threadIdx.x + o];
      s_emp[threadIdx.x] += s_emp[threadIdx.x + o];
      s_nf[threadIdx.x] |= s_nf[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    st->max_shift = sqrt(s_max[0]);
    st->sse = *sse_base + s_sum[0];
    st->n_empty = s_emp[0];
    st->nonfinite = s_nf[0];
    st->q_full = (int32_t)qcount[1];
    st->q_rerank = (int32_t)(qcount[0] - qcount[1]);
  }
}

hipError_t launch_update(const double* stats, const double* C64_old, const double* mu, const Geometry& g,
                         double* C64_new, double* work, int64_t* counts, const double* sse_base,
                         const uint32_t* qcount, DevStatus* status, hipStream_t s) {
  hipLaunchKernelGGL(k_update, dim3(g.k), dim3(64), 0, s, stats, C64_old, mu, g.k, g.d, C64_new, work, counts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(256), 0, s, work, counts, g.k, sse_base, qcount, status);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Data moments (once per load): sum_p x_p and sum_p ||x_p - mu||^2, float64.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sum_x(const float* __restrict__ X, int64_t n, int d, int dp,
                                               double* __restrict__ out) {
  const int fl = threadIdx.x & 63;
  const int rg = threadIdx.x >> 6;
  for (int f0 = 0; f0 < d; f0 += 64) {
    const int f = f0 + fl;
    double acc = 0.0;
    if (f < d)
      for (int64_t row = (int64_t)blockIdx.x * 4 + rg; row < n; row += (int64_t)gridDim.x * 4)
        acc += (double)X[row * dp + f];
    if (f < d && acc != 0.0) atomicAdd(out + f, acc);
  }
}

__global__ __launch_bounds__(256) void k_sq_dev(const float* __restrict__ X, int64_t n, int d, int dp,
                                                const double* __restrict__ mu, double* __restrict__ out) {
  __shared__ double red[4];
  const int fl = threadIdx.x & 63;
  const int rg = threadIdx.x >> 6;
  double acc = 0.0;
  for (int f0 = 0; f0 < d; f0 += 64) {
    const int f = f0 + fl;
    if (f < d) {
      const double m = mu[f];
      for (int64_t row = (int64_t)blockIdx.x * 4 + rg; row < n; row += (int64_t)gridDim.x * 4) {
        const double t = (double)X[row * dp + f] - m;
        acc = fma(t, t, acc);
      }
    }
  }
  acc = wave_sum(acc);
  if (fl == 0) red[rg] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

hipError_t launch_sum_x(const float* X, const Geometry& g, double* out, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  int64_t blocks = (g.n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_sum_x, dim3((unsigned)blocks), dim3(256), 0, s, X, g.n, g.d, g.dp, out);
  return hipGetLastError();
}

hipError_t launch_sq_dev(const float* X, const Geometry& g, const double* mu, double* out, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  int64_t blocks = (g.n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_sq_dev, dim3((unsigned)blocks), dim3(256), 0, s, X, g.n, g.d, g.dp, mu, out);
  return hipGetLastError();
}

__global__ void k_gather_rows(const float* __restrict__ X, int dp, int d, const int64_t* __restrict__ idx, int32_t n,
                              double* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n * d) return;
  const int i = (int)(t / d);
  const int f = (int)(t % d);
  out[t] = (double)X[idx[i] * dp + f];
}

hipError_t launch_gather_rows(const float* X, const Geometry& g, const int64_t* idx, int32_t n, double* out,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t tot = (int64_t)n * g.d;
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, X, g.dp, g.d, idx, n, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Synthetic Gaussian blobs, counter-based so that a row's
// value depends only on (seed, global row, feature): shard-invariant.
// ---------------------------------------------------------------------------
__host__ __device__ inline uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_gen_blobs(float* __restrict__ X, int64_t n, int d, int dp, int64_t row_offset, int n_centers,
                            float box, float stddev, uint64_t seed) {
  const int64_t tot = n * dp;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t / dp;
    const int f = (int)(t % dp);
    if (f >= d) {
      X[t] = 0.0f;
      continue;
    }
    const uint64_t g = (uint64_t)(row + row_offset);
    const uint64_t cid = splitmix64(seed ^ (g * 0xD1B54A32D192ED03ull)) % (uint64_t)n_centers;
    const uint64_t hc = splitmix64((seed + 0x5851F42D4C957F2Dull) ^ (cid * 0x2545F4914F6CDD1Dull + (uint64_t)f));
    const float u = (float)((hc >> 40) + 0.5) * (1.0f / 16777216.0f);
    const float center = box * (2.0f * u - 1.0f);
    const uint64_t hn = splitmix64((seed + 0x14057B7EF767814Full) ^ (g * 0x9E3779B97F4A7C15ull + (uint64_t)f * 0x632BE59BD9B4E019ull));
    const float u1 = (float)(((hn >> 40) & 0xFFFFFF) + 0.5) * (1.0f / 16777216.0f);
    const float u2 = (float)(((hn >> 8) & 0xFFFFFF) + 0.5) * (1.0f / 16777216.0f);
    const float z = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
    X[t] = center + stddev * z;
  }
}

hipError_t launch_gen_blobs(float* X, const Geometry& g, int64_t row_offset, int32_t n_centers, float box,
                            float stddev, uint64_t seed, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  int64_t blocks = (g.n * g.dp + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(k_gen_blobs, dim3((unsigned)blocks), dim3(256), 0, s, X, g.n, g.d, g.dp, row_offset, n_centers,
                     box, stddev, seed);
  return hipGetLastError();
}

}  // namespace km
