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
#include "km_exact.h"
#include "km_internal.h"

#include <float.h>
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>

// waves per k_assign_mfma workgroup for dp <= 64 (8, 12 or 16) and for
// 64 < dp < 192 (4, 8 or 12)
#ifndef KM_NARROW_WAVES
#define KM_NARROW_WAVES 16
#endif
#ifndef KM_WIDE_WAVES
#define KM_WIDE_WAVES 12
#endif
// k_rerank2 runs on KM_RERANK_PCT percent of n_cu workgroups
#ifndef KM_RERANK_PCT
#define KM_RERANK_PCT 100
#endif

namespace km {

thread_local LaunchTiming g_timing;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static constexpr float U24 = 5.9604644775390625e-08f;  // 2^-24, fp32 unit roundoff

__host__ __device__ inline int ceil_log2(int v) {
  int b = 0;
  while ((1 << b) < v) ++b;
  return b;
}

// top-3 smallest keys, k1 <= k2 <= k3 (v_min_f32 + 2x v_med3_f32)
__device__ __forceinline__ void top3_insert(float& k1, float& k2, float& k3, float v) {
  // min as med3(k1, v, -FLT_MAX): no NaN-canonicalising v_max in front (fminf has one)
  const float n1 = __builtin_amdgcn_fmed3f(k1, v, -FLT_MAX);
  const float n2 = __builtin_amdgcn_fmed3f(k1, k2, v);
  const float n3 = __builtin_amdgcn_fmed3f(k2, k3, v);
  k1 = n1;
  k2 = n2;
  k3 = n3;
}

__device__ __forceinline__ float key_of(float score, uint32_t idx, uint32_t mask) {
  return __uint_as_float((__float_as_uint(score) & ~mask) | idx);
}

// Cross-lane exchanges of the 16x16 MFMA layouts (lane l: column l & 15,
// quarter l >> 4).  perm_quarters: lo = value of lane (l & ~16), hi = value of
// lane (l | 16).  swap_halves(v0, v1): lanes 0-31 get v0 of lanes l and
// l + 32, lanes 32-63 get v1 of lanes l - 32 and l (the lower lane's first):
// v_permlane32_swap exchanges the upper half of its first operand with the
// lower half of its second.
__device__ __forceinline__ void perm_halves(uint32_t v, uint32_t& lo, uint32_t& hi) {
  // lo = value of lane (l & 31), hi = value of lane (l | 32), in every lane
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  lo = p[0];
  hi = p[1];
}
__device__ __forceinline__ void perm_quarters(uint32_t v, uint32_t& lo, uint32_t& hi) {
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  lo = p[0];
  hi = p[1];
}
__device__ __forceinline__ void swap_halves(uint32_t v0, uint32_t v1, uint32_t& lo, uint32_t& hi) {
  const auto p = __builtin_amdgcn_permlane32_swap(v0, v1, false, false);
  lo = p[0];
  hi = p[1];
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


// Screening bound B0 (scaled units, see DESIGN.md "Exactness") for a point of
// scaled norm xn_s, centroids of scaled max norm cm_s, and the scaled
// per-feature maxima product pm_s = (cabs s)(xabs s):
//   fp16x3 split residuals + fp64->fp32 rounding of c + ||c||^2 rounding:
//       (6.5 2^-22 + 0.5 u) xn cm + u cm^2
//   accumulation, per MFMA (3 dp/16 of them in a block chain): one final
//       rounding u |D| <= u (cm^2 + 2 xn cm) plus the in-group alignment
//       truncation of the v_mfma_f32_32x32x16_f16 product sum, <= 14 u times
//       the largest product <= 2 pm (characterised in
//       scripts/probes/mfma_align.hip: terms > 25 bits below their 8-product
//       group's maximum are dropped; worst observed U|D| + 3.7 u max|term|)
//   fp16 underflow: u sqrt(dp) (xn + 2 cm)
// times a 1.5 safety factor.
// The same terms for v_mfma_f32_16x16x32_f16 (k_fused16; characterised in
// scripts/probes/mfma_align16.hip): its 32 products form four 8-product
// groups, each aligned to its own maximum (terms > 25 bits below it dropped,
// <= 7 u per group and max product), and the four group sums enter the
// accumulator one after the other, each rounded (a group sum 24 bits below
// the running value is lost, one above it is exact).  Per MFMA: <= 4
// roundings of a partial sum bounded like |D| and 28 u max|product|; a block
// chain has 3 dp/32 of them.  In units of the 32x32x16 model: nr = rounding
// terms per chain, nt = truncation terms (28 u * 2 pm each).
struct ChainErr {
  float nr, nt;
};
__host__ __device__ inline ChainErr chain_err(int dp, int shape16) {
  const float nm32 = 3.0f * (float)dp / 16.0f;  // 32x32x16 MFMAs per block chain
  return shape16 ? ChainErr{2.0f * nm32, nm32} : ChainErr{nm32, nm32};
}
// B0 = screen_slope * xn_s + screen_icpt (affine in xn_s)
__host__ __device__ inline float screen_slope(float cm_s, int dp, int shape16 = 0) {
  const ChainErr ce = chain_err(dp, shape16);
  return 1.5f * ((6.5f * 2.384185791015625e-07f + 0.5f * U24) * cm_s + ce.nr * 2.0f * U24 * cm_s +
                 U24 * sqrtf((float)dp));
}
__host__ __device__ inline float screen_icpt(float cm_s, float pm_s, int dp, int shape16 = 0) {
  const ChainErr ce = chain_err(dp, shape16);
  return 1.5f * (U24 * cm_s * cm_s + ce.nr * U24 * cm_s * cm_s + ce.nt * 28.0f * U24 * pm_s +
                 2.0f * U24 * sqrtf((float)dp) * cm_s);
}
__host__ __device__ inline float screen_b0(float xn_s, float cm_s, float pm_s, int dp, int shape16 = 0) {
  return fmaf(screen_slope(cm_s, dp, shape16), xn_s, screen_icpt(cm_s, pm_s, dp, shape16));
}

// The same bound for the one-MFMA screen (k_assign_mfma16<..., ONE>): the
// image RN16(-2 s c') and the row RN16(s x) are single fp16 parts, so the
// product error is (2 u16 + u16^2) |a||b| per feature (Cauchy-Schwarz:
// 2 (2 u16 + u16^2) cm xn), fp16 subnormals add 2^-25 sqrt(dp) (xn + 2 cm)
// (1 + u16), c vs c' 2 u cm xn, the norm u cm^2, and the 16x16x32
// accumulation model of dp / 32 MFMAs per chain (4 u |D| and 28 u of the
// largest product each), times 1.5 like screen_b0.
__host__ __device__ inline float screen_b0_one(float xn_s, float cm_s, float pm_s, int dp) {
  constexpr float U16 = 4.8828125e-04f;
  const float nmf = (float)dp / 32.0f, sq = sqrtf((float)dp) * (1.0f + U16);
  const float slope = (2.0f * U24 + 2.0f * (2.0f * U16 + U16 * U16) + 8.0f * nmf * U24) * cm_s +
                      2.98023223876953125e-08f * sq;
  const float icpt = (1.0f + 4.0f * nmf) * U24 * cm_s * cm_s + 56.2f * nmf * U24 * pm_s +
                     5.9604644775390625e-08f * sq * cm_s;
  return 1.5f * fmaf(slope, xn_s, icpt);
}

// Per-key screening bounds (scaled units), used where the global-cmax test
// above cannot separate the candidates (e.g. far-away centroids inflate
// cmax).  Every term of screen_b0 is a function of the candidate's own scaled
// norm r (cmax -> r, the per-feature product maximum pm -> r * xabs), so a
// centroid of norm r has screen error E(r) = e2 r^2 + e1 r + e0 for this
// point (x = its scaled norm bound), and its exact score S = s^2(||c||^2 -
// 2 c.x) >= r^2 - 2 r x.  For a key k (score with truncated mantissa, rho):
//   upper(k): the centroid holding k has S <= k+ + E(R), R the largest r with
//             r^2 - 2 r x <= k+ + E(r)   (k+ = k + rho |k|);
//   lower(k): every centroid whose key is >= k has S >= min_r max(k- - E(r),
//             r^2 - 2 r x): at the crossing r* >= x of the two curves, else -x^2.
// Rounding of these fp32 evaluations is covered by explicit slack terms.
struct KeyBounds {
  float e2, e1, e0, x, rho;
  __device__ __forceinline__ float upper(float k) const {
    const float kp = k + rho * fabsf(k);
    const float a = 1.0f - e2, b = 2.0f * x + e1;
    const float disc = fmaxf(b * b + 4.0f * a * (e0 + kp), 0.0f);
    const float R = (b + sqrtf(disc)) / (2.0f * a) * (1.0f + 8.0f * U24);
    const float E = (e2 * R + e1) * R + e0;
    return kp + E + 8.0f * U24 * (fabsf(kp) + E + R * (R + 2.0f * x));
  }
  __device__ __forceinline__ float lower(float k) const {
    const float km = k - rho * fabsf(k);
    const float a = 1.0f + e2, b = 2.0f * x - e1;
    const float disc = b * b + 4.0f * a * (km - e0);
    const float floor_ = -x * x * (1.0f + 8.0f * U24);
    if (!(disc >= 0.0f)) return floor_;
    const float r = (b + sqrtf(disc)) / (2.0f * a);
    if (!(r >= x)) return floor_;
    const float E = (e2 * r + e1) * r + e0;
    const float f = km - E, g = r * (r - 2.0f * x);
    return fmaxf(fminf(f, g) - 8.0f * U24 * (fabsf(km) + E + r * (r + 2.0f * x)), floor_);
  }
};

// E(r) of screen_b0_one (cm -> r, pm -> r min(xn, xabs))
__device__ __forceinline__ KeyBounds key_bounds_one(float xn_s, float xabs_s, int dp, float rho) {
  constexpr float U16 = 4.8828125e-04f;
  const float nmf = (float)dp / 32.0f, sq = sqrtf((float)dp) * (1.0f + U16);
  KeyBounds kb;
  kb.e2 = 1.5f * U24 * (1.0f + 4.0f * nmf);
  kb.e1 = 1.5f * ((2.0f * U24 + 2.0f * (2.0f * U16 + U16 * U16) + 8.0f * nmf * U24) * xn_s +
                  56.2f * nmf * U24 * fminf(xn_s, xabs_s) + 5.9604644775390625e-08f * sq);
  kb.e0 = 1.5f * 2.98023223876953125e-08f * sq * xn_s;
  kb.x = xn_s;
  kb.rho = rho * 1.01f + 2.0f * U24;
  return kb;
}

// E(r) coefficients for a point of scaled norm bound xn_s (xabs_s: scaled
// max |x_f| over the data), the terms of screen_b0 with the same 1.5 safety
__device__ __forceinline__ KeyBounds key_bounds(float xn_s, float xabs_s, int dp, float rho, int shape16 = 0) {
  const ChainErr ce = chain_err(dp, shape16);
  const float sq = sqrtf((float)dp);
  KeyBounds kb;
  kb.e2 = 1.5f * U24 * (1.0f + ce.nr);
  kb.e1 = 1.5f * ((6.5f * 2.384185791015625e-07f + 0.5f * U24 + 2.0f * ce.nr * U24) * xn_s +
                  28.0f * ce.nt * U24 * fminf(xn_s, xabs_s) + 2.0f * U24 * sq);
  kb.e0 = 1.5f * U24 * sq * xn_s;
  kb.x = xn_s;
  kb.rho = rho * 1.01f + 2.0f * U24;
  return kb;
}

// ---------------------------------------------------------------------------
// Centroid preparation: float64 centroids -> fp32 copy (direct screening),
// bf16 hi/lo split of -2c (MFMA screening), fp32 ||c||^2, max ||c||.
// Padded rows (k <= j < kp) are zero with ||c||^2 = 1e30 (never selected).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_prep_centroids(const double* __restrict__ C64, int k, int d, int dp,
                                                       float* __restrict__ C32, float* __restrict__ cn2,
                                                       float* __restrict__ cmax, float* __restrict__ cabs,
                                                       double* __restrict__ C64T, double* __restrict__ C64P, const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  const int j = blockIdx.x;
  const int lane = threadIdx.x;
  double nn = 0.0;
  float am = 0.0f;
  for (int f = lane; f < dp; f += 64) {
    const double c = (j < k && f < d) ? C64[(size_t)j * d + f] : 0.0;
    if (j < k && f < d) C64T[(size_t)f * k + j] = c;
    C64P[(size_t)j * dp + f] = c;
    nn = fma(c, c, nn);
    const float c32 = (float)c;
    C32[(size_t)j * dp + f] = c32;
    am = (fabsf(c32) > am || c32 != c32) ? fabsf(c32) : am;
  }
  nn = wave_sum(nn);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float t = __shfl_xor(am, o);
    am = (t > am || t != t) ? t : am;
  }
  if (lane == 0 && j < k) atomicMax((unsigned int*)cabs, __float_as_uint(am));
  if (lane == 0) {
    cn2[j] = (j < k) ? (float)nn : 1e30f;
    if (j < k) {
      const float cn = sqrtf((float)nn) * 1.0001f + 1e-30f;
      atomicMax((unsigned int*)cmax, __float_as_uint(cn));
    }
  }
}

// Small path (k <= 32, dp <= 64): its only centroid images -- the fp32 copy
// [kp][dp] and max ||c|| -- in one workgroup (the MFMA path's prep is four
// launches: maxima, copies + norms, fp16 split, bound constants)
__global__ __launch_bounds__(256) void k_prep_small(const double* __restrict__ C64, int k, int d, int dp, int kp,
                                                    float* __restrict__ C32, float* __restrict__ cmax,
                                                    const int* __restrict__ gate) {
  if (*gate) return;
  __shared__ unsigned int red[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned int mx = 0u;  // max of non-negative floats (or NaN) as bits, like the atomicMax of k_prep_centroids
  for (int j = wave; j < kp; j += 4) {
    double nn = 0.0;
    for (int f = lane; f < dp; f += 64) {
      const double c = (j < k && f < d) ? C64[(size_t)j * d + f] : 0.0;
      nn = fma(c, c, nn);
      C32[(size_t)j * dp + f] = (float)c;
    }
    nn = wave_sum(nn);
    if (lane == 0 && j < k) {
      const float cn = sqrtf((float)nn) * 1.0001f + 1e-30f;
      mx = max(mx, __float_as_uint(cn));
    }
  }
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  if (threadIdx.x == 0) *cmax = __uint_as_float(max(max(red[0], red[1]), max(red[2], red[3])));
}

hipError_t launch_prep_small(const double* C64, const Geometry& g, float* C32, float* cmax, const int* gate,
                             hipStream_t s) {
  hipLaunchKernelGGL(k_prep_small, dim3(1), dim3(256), 0, s, C64, g.k, g.d, g.dp, g.kp, C32, cmax, gate);
  return hipGetLastError();
}

__global__ void k_zero_maxima(float* __restrict__ cmax, float* __restrict__ cabs, const int* __restrict__ gate) {
  if (*gate) return;
  if (threadIdx.x == 0) {
    *cmax = 0.0f;
    *cabs = 0.0f;
  }
}

hipError_t launch_prep_centroids(const double* C64, const Geometry& g, float* C32, float* cn2, float* cmax,
                                 float* cabs, double* C64T, double* C64P, const int* gate, hipStream_t s) {
  // the two maxima are zeroed by a gated kernel (a memset would run in a
  // stopped batch and leave the live images' bound inputs at zero)
  hipLaunchKernelGGL(k_zero_maxima, dim3(1), dim3(64), 0, s, cmax, cabs, gate);
  hipLaunchKernelGGL(k_prep_centroids, dim3(g.kp), dim3(64), 0, s, C64, g.k, g.d, g.dp, C32, cn2, cmax, cabs, C64T,
                     C64P, gate);
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
static constexpr int SMALL_QW = 32;  // queued rows a wave resolves itself (LDS); more go to the last workgroup
static constexpr int SMALL_LDS = 60 * 1024;

// The rows the direct-form bound cannot settle (rare: q_rerank 0 at c2 in
// steady state) are queued instead of re-ranked in-thread: the float64
// re-rank's registers held the kernel at 4 waves per SIMD (125 VGPRs) while
// it never ran.  The last workgroup to finish (done counter) resolves the
// queue -- the reference's float64 norms in NumPy's order, np.argmin's
// tie-break -- adds those rows' sums, counts and residuals, and, when the
// iteration is local (one rank: no all-reduce between the sums and the
// update), runs the one-workgroup update itself, so an iteration is one
// launch (update_one_body; launch_assign_small's SmallTail).

template <bool COHERENT>
__device__ void update_one_body(double* __restrict__ stats, const double* __restrict__ old, int k, int d,
                                double* __restrict__ out, int64_t* __restrict__ counts, const double* __restrict__ sse,
                                const uint32_t* __restrict__ qcount, uint32_t nq, DevStatus* __restrict__ st,
                                int* __restrict__ gate, double stop_tol, int dev_repair, int clear,
                                float* __restrict__ C32, float* __restrict__ cmax, int dp, int kp, int corr = 0);

// waves per SIMD at dp = 16 (KM_SMALL_WPE; c2 on one MI355X: 4 waves with the
// row prefetch 146-147 us, 8 waves without it 154-161 us), the compiler's
// choice above (a row and its prefetch are 2 dp VGPRs)
#ifndef KM_SMALL_WPE
#define KM_SMALL_WPE 4
#endif
// A/B knobs, c2 on one MI355X (profiles/r5_c2_small_ab.json):
//   KM_SMALL_SERP serpentine sweep: 153-155 -> 145 us (6,450 -> 6,840 it/s)
//   KM_SMALL_SC   centroids as scalar operands: 141-142 -> 135-136 us
//   KM_SMALL_PF2  two rows prefetched (4 waves): +4-5 us, off
//   KM_SMALL_PF8  the one-row prefetch at 6 waves per SIMD: +5 us, off
//   KM_SMALL_NTL  non-temporal label stores: -1 us; 32 statistics replicas +5 us
#ifndef KM_SMALL_PF2
#define KM_SMALL_PF2 0
#endif
#ifndef KM_SMALL_SC
#define KM_SMALL_SC 1
#endif
#ifndef KM_SMALL_PF8
#define KM_SMALL_PF8 0
#endif
#ifndef KM_SMALL_SERP
#define KM_SMALL_SERP 1
#endif
#ifndef KM_SMALL_NTL  // labels stored non-temporal: +1% (the 40 MB of labels leave the cache to X)
#define KM_SMALL_NTL 1
#endif
template <int DP, bool SSE, int WPE = (DP <= 16 ? KM_SMALL_WPE : 1)>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_assign_small(const float* __restrict__ X, int64_t n, int d, int k, const float* __restrict__ C32,
                    const double* __restrict__ C64, const float* __restrict__ cmaxp, int32_t* __restrict__ labels,
                    double* __restrict__ stats, int fuse, int R, const int* __restrict__ gate, SmallTail T) {
  constexpr bool want_sse = SSE;
  if (*gate) {  // a stopped batch (km_update_async): the rest of it is a no-op
    if (T.fold && blockIdx.x == 0 && threadIdx.x == 0) {
      T.st->ran = 0;
      T.st->stop = 0;
    }
    return;
  }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sC = reinterpret_cast<float*>(smem);
  double* tab = reinterpret_cast<double*>(smem + ((k * DP * 4 + 15) / 16) * 16);
  const int d1 = d + 1;
  const int lane = threadIdx.x & 63;
  if (!KM_SMALL_SC)
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

  // rows strided over the grid; the next row is prefetched into registers
  // while this one is processed (the loop is otherwise latency-bound)
  const int64_t rstride = (int64_t)gridDim.x * blockDim.x;
  int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double sacc = 0.0;  // this lane's SSE residuals (want_sse)
  // this wave's queued rows (LDS, after the statistics table)
  uint32_t* wq = reinterpret_cast<uint32_t*>(smem + ((k * DP * 4 + 15) / 16) * 16 + (fuse ? (size_t)k * d1 * R * 8 : 0)) +
                 (threadIdx.x >> 6) * SMALL_QW;
  uint32_t wq_n = 0;
  // PF: the next row prefetched into registers while this one is processed
  // (at 8 waves per SIMD the other waves hide the latency instead: no
  // prefetch, 2 dp fewer VGPRs); PF2: two rows ahead (KM_SMALL_PF2)
  constexpr bool PF = WPE < 8 || KM_SMALL_PF8;
  constexpr bool PF2 = PF && KM_SMALL_PF2 && DP <= 16;
  // serpentine sweep: every other launch visits the rows from the last one
  // down, so its first ~200 MB are the previous launch's last reads, still in
  // the 256 MiB Infinity Cache (same rows, same per-row work; only the order)
  const bool rev = KM_SMALL_SERP && T.rev;
  auto at = [&](int64_t v) { return rev ? n - 1 - v : v; };
  float4 nx[DP / 4], nx2[DP / 4];
  if (PF && row < n) {
#pragma unroll
    for (int f = 0; f < DP; f += 4) nx[f / 4] = *reinterpret_cast<const float4*>(X + at(row) * DP + f);
  }
  if (PF2 && row + rstride < n) {
#pragma unroll
    for (int f = 0; f < DP; f += 4) nx2[f / 4] = *reinterpret_cast<const float4*>(X + at(row + rstride) * DP + f);
  }
  auto row_body = [&](const float (&x)[DP], int64_t row) {
    float k1 = FLT_MAX, k2 = FLT_MAX, k3 = FLT_MAX;
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    bool amb;
    {
      // packed fp32 (v_pk_add_f32 / v_pk_fma_f32): even and odd features in
      // two partial sums, half the VALU issue of the scalar loop; the
      // direct-form bound (DP sequential terms) covers two sums of DP / 2
#pragma unroll 2
      for (int j = 0; j < k; ++j) {
        // KM_SMALL_SC: the centroid through uniform (scalar) loads from C32,
        // operands from SGPRs, instead of LDS reads into VGPRs
        const f32x2* c2 = reinterpret_cast<const f32x2*>((KM_SMALL_SC ? C32 : sC) + j * DP);
        f32x2 acc2 = {0.0f, 0.0f};
#pragma unroll
        for (int f = 0; f < DP; f += 2) {
          const f32x2 xv = {x[f], x[f + 1]};
          const f32x2 t = xv - c2[f / 2];
          acc2 = __builtin_elementwise_fma(t, t, acc2);
        }
        top3_insert(k1, k2, k3, key_of(acc2.x + acc2.y, (uint32_t)j, mask));
      }
      const float B1 = alpha * k1 + beta * sqrtf(k1) + g0;
      const float B2 = alpha * k2 + beta * sqrtf(k2) + g0;
      amb = (k >= 2) && !(k2 - B2 > k1 + B1);  // k1 not provably the float64 argmin
    }
    int lab = (int)(__float_as_uint(k1) & mask);
    if (lab >= k) lab = 0;  // only reachable with non-finite data (np.argmin of NaNs -> 0)
    // a queued row's label is written by the last workgroup only (two
    // writers of one label in one launch could reach memory in either order)
    if (!amb) {
      if (KM_SMALL_NTL)
        __builtin_nontemporal_store(lab, labels + row);  // keep the Infinity Cache for X (serpentine sweep)
      else
        labels[row] = lab;
    }
    const uint64_t qm = __ballot(amb);
    if (qm) {  // rare: the wave's own LDS queue, past SMALL_QW rows the launch's queue
      const uint32_t pos = wq_n + (uint32_t)__popcll(qm & ((1ull << lane) - 1ull));
      if (amb) {
        if (pos < SMALL_QW) {
          wq[pos] = (uint32_t)row;
        } else {
          // write-through (sc1) store: the last workgroup may sit on another XCD
          const uint32_t g = atomicAdd(T.qctr, 1u);
          __hip_atomic_store(T.queue + g, (uint32_t)row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      wq_n += (uint32_t)__popcll(qm);
    }
    if (amb) return;
    if (want_sse) {
      // min(norm)**2 of compute_partition_sse (kmeans_spark.py:231-233): the
      // residual to the pre-update centroid, each difference and square in
      // float64 (no cancellation, unlike ||x||^2 - 2 x.c + ||c||^2)
      const double* c = C64 + (size_t)lab * d;
      double r = 0.0;
#pragma unroll
      for (int f = 0; f < DP; ++f)
        if (f < d) {
          const double t = (double)x[f] - c[f];
          r = fma(t, t, r);
        }
      sacc += r;
    }
    if (fuse) {
      double* t = tab + (size_t)lab * d1 * R + rep;
#pragma unroll
      for (int f = 0; f < DP; ++f)
        if (f < d) atomicAdd(t + (size_t)f * R, (double)x[f]);
      atomicAdd(t + (size_t)d * R, 1.0);
    }
  };
  auto unpack = [&](const float4 (&v)[DP / 4], float (&x)[DP]) {
#pragma unroll
    for (int f = 0; f < DP; f += 4) {
      x[f] = v[f / 4].x;
      x[f + 1] = v[f / 4].y;
      x[f + 2] = v[f / 4].z;
      x[f + 3] = v[f / 4].w;
    }
  };
  auto load_row = [&](float4 (&v)[DP / 4], int64_t r) {
#pragma unroll
    for (int f = 0; f < DP; f += 4) v[f / 4] = *reinterpret_cast<const float4*>(X + r * DP + f);
  };
  if constexpr (PF2) {
    for (; row < n; row += 2 * rstride) {
      float x[DP];
      unpack(nx, x);
      if (row + 2 * rstride < n) load_row(nx, at(row + 2 * rstride));
      row_body(x, at(row));
      if (row + rstride >= n) break;
      unpack(nx2, x);
      if (row + 3 * rstride < n) load_row(nx2, at(row + 3 * rstride));
      row_body(x, at(row + rstride));
    }
  } else {
    for (; row < n; row += rstride) {
      float x[DP];
      if constexpr (PF) {
        unpack(nx, x);
        if (row + rstride < n) load_row(nx, at(row + rstride));
      } else {
        float4 v[DP / 4];
        load_row(v, at(row));
        unpack(v, x);
      }
      row_body(x, at(row));
    }
  }
  // A queued row, resolved by one wave, lanes over centroids: the
  // reference's float64 norms (kmeans_spark.py:153) in NumPy's pairwise
  // order, np.argmin's tie-break across the lanes; the row's sums go to the
  // LDS table (in_lds) or straight to the global statistics; returns its
  // residual (want_sse) in every lane
  auto resolve = [&](int64_t r, bool in_lds) {
    const float* xr = X + r * DP;
    double v = 0.0;
    int j = -1;
    if (lane < k) {
      v = np_norm_d<0>([&](int f) { return np_sq(C64[(size_t)lane * d + f], xr[f]); }, d);  // d <= 64: one block
      j = lane;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {  // first NaN, else the smallest, lowest index
      const double ov = __shfl_xor(v, o);
      const int oj = __shfl_xor(j, o);
      bool take = false;
      if (oj >= 0) {
        if (j < 0) {
          take = true;
        } else {
          const bool on = ov != ov, mn = v != v;
          take = (on && !mn) || (on == mn && (on ? oj < j : (ov < v || (ov == v && oj < j))));
        }
      }
      v = take ? ov : v;  // select form
      j = take ? oj : j;
    }
    const int lab = j < 0 ? 0 : j;
    if (lane == 0) {
      if (in_lds)
        labels[r] = lab;
      else  // write-through: no other writer of this label in the launch, but keep it out of this XCD's L2
        __hip_atomic_store(labels + r, lab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    double rr = 0.0;
    for (int f = lane; f < d; f += 64) {
      const double x = (double)xr[f];
      if (fuse) {
        if (in_lds)
          atomicAdd(tab + ((size_t)lab * d1 + f) * R, x);
        else
          atomicAdd(stats + (size_t)lab * d1 + f, x);
      }
      const double t = x - C64[(size_t)lab * d + f];
      rr = fma(t, t, rr);
    }
    if (fuse && lane == 0) {
      if (in_lds)
        atomicAdd(tab + ((size_t)lab * d1 + d) * R, 1.0);
      else
        atomicAdd(stats + (size_t)lab * d1 + d, 1.0);
    }
    return want_sse ? wave_sum(rr) : 0.0;
  };
  {
    const uint32_t nall = (uint32_t)__builtin_amdgcn_readfirstlane(wq_n);
    if (nall && lane == 0) atomicAdd(T.done + 1, nall);  // queued rows of the launch (status q_rerank)
    const uint32_t nw = min(nall, (uint32_t)SMALL_QW);
    for (uint32_t i = 0; i < nw; ++i) {
      const double rs = resolve(wq[i], true);
      if (lane == 0) sacc += rs;
    }
  }
  if (want_sse) {
    sacc = wave_sum(sacc);
    if (lane == 0 && sacc != 0.0) atomicAdd(stats + (size_t)k * d1, sacc);
  }
  if (fuse) {
    __syncthreads();
    for (int e = threadIdx.x; e < k * d1; e += blockDim.x) {
      double s = 0.0;
      for (int r = 0; r < R; ++r) s += tab[(size_t)e * R + r];
      if (s != 0.0) atomicAdd(stats + e, s);
    }
  }
  // ---- the last workgroup: queued rows, then (fold) the update ----
  // Hand-off without an L2 write-back (cdna_hip_programming.md section 6,
  // the counter form with write-through data): everything the last
  // workgroup reads was written by device-scope atomics (sums, counter) or
  // sc1 stores (queue); each wave drains them (vmcnt), then one relaxed
  // agent-scope ticket per workgroup; the last reads with sc1 loads.
  // (__threadfence() here -- a full XCD L2 write-back per workgroup -- made
  // the c2 launch 3.5x slower.)
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // (one ticket per workgroup on one counter; per-group counters and 16
  // copies of the sums, merged by the last workgroup, measured 7% slower)
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(T.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
  __syncthreads();
  if (!s_last) return;
  const uint32_t nq = __hip_atomic_load(T.qctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the rows past the waves' own queues: one per wave
  const int wave = threadIdx.x >> 6;
  double qs = 0.0;
  for (uint32_t i = wave; i < nq; i += blockDim.x >> 6)
    qs += resolve(__hip_atomic_load(T.queue + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), false);
  if (want_sse && lane == 0 && qs != 0.0) atomicAdd(stats + (size_t)k * d1, qs);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the queued rows' sums are in before the update reads them
  __syncthreads();
  if (T.fold) {
    update_one_body<true>(stats, T.old, k, d, T.out, T.counts, stats + (size_t)k * d1, nullptr, 0u, T.st, T.gate,
                          T.stop_tol, T.dev_repair, 1, T.C32n, T.cmaxn, DP, T.kp);
    if (threadIdx.x == 0)
      T.st->q_rerank = (int32_t)__hip_atomic_load(T.done + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (T.qout && threadIdx.x == 0) {
    // the separate update launch reports the queued rows from qcount (one segment)
    T.qout[0] = __hip_atomic_load(T.done + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    T.qout[1] = 0u;
  }
  if (threadIdx.x == 0) {
    T.done[0] = 0u;
    T.done[1] = 0u;
    *T.qctr = 0u;
  }
}

// tuning knobs: defaults measured on MI355X; environment overrides exist only
// in the diagnostic build (make diag) for sweeps and ablations
int diag_env(const char* name, int dflt) {
#ifdef KM_DIAG
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

// statistics replicas: as many as fit the LDS share of one of the 8
// workgroups a CU holds at 8 waves per SIMD (20 KiB each), at most 32
#ifndef KM_SMALL_LDS
#define KM_SMALL_LDS (20 * 1024)
#endif
#ifndef KM_SMALL_BPC
#define KM_SMALL_BPC 8
#endif
static constexpr int SMALL_WG_LDS = KM_SMALL_LDS;
static int small_replicas(const Geometry& g) {
  const size_t cbytes = ((size_t)g.k * g.dp * 4 + 15) / 16 * 16;
  static const int rmax = diag_env("KM_SMALL_R", 32);
  static const int budget = diag_env("KM_SMALL_LDS", SMALL_WG_LDS);
  int R = rmax;
  while (R > 1 && cbytes + (size_t)g.k * (g.d + 1) * 8 * R > (size_t)budget) R >>= 1;
  return R;
}

bool small_path_ok(const Geometry& g) {
  if (g.k > SMALL_MAX_K || g.dp > 64) return false;
  const size_t cbytes = ((size_t)g.k * g.dp * 4 + 15) / 16 * 16;
  return cbytes + (size_t)g.k * (g.d + 1) * 8 <= SMALL_LDS;
}

hipError_t launch_assign_small(const float* X, const Geometry& g, const float* C32, const double* C64,
                               const float* cmax, int32_t* labels, double* stats, int fuse, int want_sse, int n_cu,
                               const int* gate, hipStream_t s, const SmallTail& tail) {
  if (g.n == 0) return hipSuccess;
  if (!tail.queue || !tail.qctr || !tail.done) return hipErrorInvalidValue;
  const int R = small_replicas(g);
  const size_t lds = ((size_t)g.k * g.dp * 4 + 15) / 16 * 16 + (fuse ? (size_t)g.k * (g.d + 1) * 8 * R : 0) +
                     (size_t)4 * SMALL_QW * 4;
  int64_t blocks = (g.n + 255) / 256;
  static const int bpc = diag_env("KM_SMALL_BPC", KM_SMALL_BPC);
  const int64_t cap = (int64_t)n_cu * bpc;
  if (blocks > cap) blocks = cap;
#define KM_SMALL_CASE(DP_)                                                                                 \
  case DP_:                                                                                                \
    if (want_sse)                                                                                          \
      KM_TIMED_LAUNCH((k_assign_small<DP_, true>), dim3((unsigned)blocks), dim3(256), lds, s, X, g.n, g.d,  \
                      g.k, C32, C64, cmax, labels, stats, fuse, R, gate, tail);                            \
    else                                                                                                   \
      KM_TIMED_LAUNCH((k_assign_small<DP_, false>), dim3((unsigned)blocks), dim3(256), lds, s, X, g.n,      \
                      g.d, g.k, C32, C64, cmax, labels, stats, fuse, R, gate, tail);                       \
    break;
  switch (g.dp) {
    KM_SMALL_CASE(16) KM_SMALL_CASE(32) KM_SMALL_CASE(48) KM_SMALL_CASE(64)
    default:
      return hipErrorInvalidValue;
  }
#undef KM_SMALL_CASE
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// MFMA screening path (c3/c4/c5 shapes).
//
// Scores S[j][p] = ||c_j||^2 - 2 c_j.x_p on v_mfma_f32_32x32x16_f16 with an
// fp16x3 split: with a power-of-two scale s (data and centroids into
// |.| < 2^14), -2cs = ch + cl and xs = xh + xl (fp16 halves, 22 bits), and
// S s^2 ~ ||cs||^2 + ch.xl + cl.xh + ch.xh accumulated in fp32.  A operand =
// 32 centroids (LDS), B operand = 32 points (registers), accumulator
// initialised with ||c||^2 s^2.  C/D layout: column (point) on the lane,
// centroid rows in registers; each lane keeps four independent running
// top-3 chains of (score | j>>2 in the low mantissa bits) with v_med3, the
// chain id carrying j & 3.  Blocks of 32 centroids are software-pipelined in
// pairs so one block's key updates overlap the next block's MFMAs.
// ---------------------------------------------------------------------------
static constexpr int MFMA_LDS_LARGE = 160 * 1024;  // LDS per CU

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
// lo = RN_f16(xs - hi) for a pair, hi = RN_f16(xs) (the fp16x3 row split).
// Written in C: the compiler turns it into v_fma_mix forms with the scale
// folded in and pads the VALU -> MFMA operand hazard itself.  The
// inline-asm form (KM_SPLIT_ASM=1, one v_fma_mix per element, rounds 1-3)
// is not safe: hipcc placed an asm v_fma_mixhi_f16 one wait state before the
// MFMA that reads its register as the B operand -- compiler-emitted VALU
// writes get two -- and k_fused16 then read stale row halves (567 of 20,000
// labels wrong in the far-from-origin test, 0 with this form; DESIGN.md
// section 4).  k_fused's asm happened to be scheduled two or more apart.
#ifndef KM_SPLIT_ASM
#define KM_SPLIT_ASM 0
#endif
__device__ __forceinline__ f16x2 split_lo(f16x2 hp, float xs0, float xs1) {
#if !KM_SPLIT_ASM
  // xs - hi is exact in fp32; the compiler emits its own v_fma_mix form
  // (with the scale folded in) and sees the writes it must pad
  const f16x2 lo = {(_Float16)(xs0 - (float)hp[0]), (_Float16)(xs1 - (float)hp[1])};
  return lo;
#else
  uint32_t lp;
  asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lp) : "v"(__builtin_bit_cast(uint32_t, hp)), "v"(xs0));
  asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "+v"(lp)
      : "v"(__builtin_bit_cast(uint32_t, hp)), "v"(xs1));
  return __builtin_bit_cast(f16x2, lp);
#endif
}


// power-of-two scale: max(|x|, |c|) * s < 2^14 (so |-2cs| < 2^15 < 65504);
// 1 for non-finite or all-zero data (the keys then force the exact path)
__device__ __forceinline__ float mfma_scale(float xabs, float cabs) {
  const float m = fmaxf(xabs, cabs);
  if (!(m > 0.0f) || !(m < 3.0e38f)) return 1.0f;
  int e;
  (void)frexpf(m, &e);  // m < 2^e
  return ldexpf(1.0f, 14 - e);
}

__global__ __launch_bounds__(64) void k_prep_split(const float* __restrict__ C32, int kp, int dp,
                                                   const float* __restrict__ cn2, const float* __restrict__ xabs,
                                                   const float* __restrict__ cabs, _Float16* __restrict__ Chi,
                                                   _Float16* __restrict__ Clo, float* __restrict__ cn2s, int k, const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  const int j = blockIdx.x;
  const float s = mfma_scale(*xabs, *cabs);
  for (int f = threadIdx.x; f < dp; f += 64) {
    const float m2 = -2.0f * C32[(size_t)j * dp + f] * s;
    const _Float16 hi = (_Float16)m2;
    Chi[(size_t)j * dp + f] = hi;
    Clo[(size_t)j * dp + f] = (_Float16)(m2 - (float)hi);
  }
  if (threadIdx.x == 0) cn2s[j] = (j < k) ? cn2[j] * s * s : 1e30f;
}

// top-3 insert carrying the index of the two best (a candidate equal to a
// kept key does not displace it)
__device__ __forceinline__ void top3p_insert(float& k1, float& k2, float& k3, uint32_t& p1, uint32_t& p2, float v,
                                             uint32_t pv) {
  const bool lt1 = v < k1, lt2 = v < k2, lt3 = v < k3;
  const float n3 = lt2 ? k2 : (lt3 ? v : k3);
  const float n2 = lt1 ? k1 : (lt2 ? v : k2);
  const uint32_t q2 = lt1 ? p1 : (lt2 ? pv : p2);
  k1 = lt1 ? v : k1;
  p1 = lt1 ? pv : p1;
  k2 = n2;
  p2 = q2;
  k3 = n3;
}

static constexpr int CAND_REC = 16;  // candidate record: count + up to 15 centroid indices, ascending
int cand_rec_words() { return CAND_REC; }

template <int NS, int WAVES>
constexpr int mfma_min_waves() {
  return WAVES == 4 ? 1 : (WAVES == 16 ? 4 : (WAVES == 12 ? 3 : (NS <= 4 ? 4 : 2)));
}

struct MfmaArgs {
  const float* X;
  int64_t n;
  int k, kp, KC;
  uint32_t seg;
  const _Float16* Chi;
  const _Float16* Clo;
  const float* cn2s;
  const float* cmax;
  const float* xabs;
  const float* cabs;
  int32_t* labels;
  QEntry* queue;
  uint32_t* qcount;
  const int* gate;  // nonzero: a stopped batch, the launch is a no-op
  uint32_t* cand;      // candidate pool (kind-4 entries): CAND_REC words per record, nullptr: off
  uint32_t* cand_ctr;  // records taken this launch (zeroed before it)
  uint32_t cand_cap;   // records
  int one = 0;         // k_assign_mfma16: one fp16 MFMA per product (KM_SCREEN_ONE)
  const float* C32 = nullptr;  // ONE: fp32 centroids [kp][dp], the in-kernel pair re-score
  // delta statistics (k_assign_mfma16): the previous labels are read; a
  // decided row whose label changed is written and appended to its wave's
  // change-list segment {row, old << 16 | new} ([wave][seg], count in
  // chg_cnt[wave]); queued rows keep their previous label for the resolvers
  uint2* chg = nullptr;
  uint32_t* chg_cnt = nullptr;
};

// LDS image of a centroid chunk: for block b (32 centroids) and K-step t the
// A fragment is one contiguous 1 KiB piece, lane l at byte 16*l (rows
// 32b + (l&31), features 16t + 8(l>>5) .. +8): lane-linear, bank-conflict
// free, and every read of a block is base + immediate offset.
// T2: chains keep their best two keys (3 VALU per score instead of 4; for
// small d, where the key updates, not the MFMAs, bound the loop); a point
// whose best two share a chain then has no re-rank certificate (full scan).
template <int NS, int WAVES, bool T2 = false>
__global__ __launch_bounds__(WAVES * 64, (mfma_min_waves<NS, WAVES>())) void k_assign_mfma(MfmaArgs A) {
  if (*A.gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  constexpr int DP = 16 * NS;
  constexpr int BLKB = NS * 1024;  // bytes of one block's fragments (one of hi / lo)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KC = A.KC;
  const size_t himg = (size_t)(KC / 32) * BLKB;
  // one chunk image: hi, lo, ||c||^2 s^2; with several chunks two of them
  // (double buffer, filled by LDS-DMA while the other is read)
  const size_t bufsz = ((2 * himg + (size_t)KC * 4) + 15) / 16 * 16;
  char* sHi = smem;
  char* sLo = smem + himg;
  float* sCn = reinterpret_cast<float*>(smem + 2 * himg);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int kp = A.kp;
  const int64_t n = A.n;
  const int b = ceil_log2(kp);  // kp is a multiple of 64: b >= 6
  const uint32_t maskq = (1u << (b - 2)) - 1u;
  const float s = mfma_scale(*A.xabs, *A.cabs);
  const float cm = *A.cmax * s;
  const float pm = (*A.cabs * s) * (*A.xabs * s) * 1.0001f;
  const float rho = __builtin_ldexpf(1.0f, b - 2 - 23) * 1.01f;  // key truncation (relative)
  const int nchunks = (kp + KC - 1) / KC;
  const int64_t ntiles = (n + 31) / 32;
  const int64_t nwt = (ntiles + WAVES - 1) / WAVES;

  auto stage = [&](int ch) {
    const int kc = min(KC, kp - ch * KC);
    const int npieces = (kc / 32) * NS * 64;  // 16-byte pieces per image
    const char* gh = reinterpret_cast<const char*>(A.Chi + (size_t)ch * KC * DP);
    const char* gl = reinterpret_cast<const char*>(A.Clo + (size_t)ch * KC * DP);
    for (int id = threadIdx.x; id < npieces; id += WAVES * 64) {
      const int l = id & 63;
      const int bt = id >> 6;  // blk * NS + t
      const int blk = bt / NS, t = bt - blk * NS;
      const size_t src = ((size_t)(blk * 32 + (l & 31)) * DP + 16 * t + 8 * (l >> 5)) * 2;
      *reinterpret_cast<uint4*>(sHi + (size_t)id * 16) = *reinterpret_cast<const uint4*>(gh + src);
      *reinterpret_cast<uint4*>(sLo + (size_t)id * 16) = *reinterpret_cast<const uint4*>(gl + src);
    }
    for (int id = threadIdx.x; id < kc; id += WAVES * 64) sCn[id] = A.cn2s[(size_t)ch * KC + id];
  };

  // several chunks: chunk images through LDS-DMA (global_load_lds, 16 B per
  // lane, no VGPRs), one 1 KiB fragment piece per wave-instruction, into the
  // buffer the waves are not reading; the barrier at each chunk start drains
  // the wave's own DMA (vmcnt) and then everyone's
  auto stage_async = [&](int ch, int bf) {
    const int kc = min(KC, kp - ch * KC);
    const int npc = (kc / 32) * NS;  // 1 KiB pieces per image
    char* dHi = smem + (size_t)bf * bufsz;
    char* dLo = dHi + himg;
    char* dCn = dHi + 2 * himg;
    const char* gh = reinterpret_cast<const char*>(A.Chi + (size_t)ch * KC * DP);
    const char* gl = reinterpret_cast<const char*>(A.Clo + (size_t)ch * KC * DP);
    for (int pc = wave; pc < npc; pc += WAVES) {
      const int blk = pc / NS, t = pc - blk * NS;
      const size_t src = ((size_t)(blk * 32 + r) * DP + 16 * t + 8 * h) * 2;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(gh + src),
                                       (__attribute__((address_space(3))) void*)(dHi + (size_t)pc * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(gl + src),
                                       (__attribute__((address_space(3))) void*)(dLo + (size_t)pc * 1024), 16, 0, 0);
    }
    // ||c||^2 s^2 of the chunk: kc * 4 bytes, 1 KiB per wave-instruction
    const char* gc = reinterpret_cast<const char*>(A.cn2s + (size_t)ch * KC);
    for (int pc = wave; pc * 1024 < kc * 4; pc += WAVES)
      if (pc * 1024 + lane * 16 < kc * 4)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(gc + pc * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(dCn + pc * 1024), 16, 0, 0);
  };

  int cbuf = 0;  // buffer the current chunk is in (several chunks)
  if (nchunks == 1) {
    stage(0);
    __syncthreads();
  } else if ((int64_t)blockIdx.x < nwt) {
    stage_async(0, 0);
  }

  // per-wave queue segment: no global counter (one hot address would
  // serialise every wave at the memory side)
  const uint32_t gw = blockIdx.x * WAVES + wave;
  QEntry* wq = A.queue + (size_t)gw * A.seg;
  uint32_t qn = 0, qf = 0;
  const char* laneHi = sHi + lane * 16;
  const char* laneLo = sLo + lane * 16;
  const float* laneCn = sCn + 4 * h;
  auto point_at = [&](int bf) {
    laneHi = smem + (size_t)bf * bufsz + lane * 16;
    laneLo = laneHi + himg;
    laneCn = reinterpret_cast<const float*>(smem + (size_t)bf * bufsz + 2 * himg) + 4 * h;
  };

  for (int64_t wt = blockIdx.x; wt < nwt; wt += gridDim.x) {
    const int64_t tile = wt * WAVES + wave;
    if (nchunks == 1 && tile >= ntiles) break;  // no barriers below in this mode
    const int64_t row = tile * 32 + r;
    const bool valid = row < n;
    const float* xr = A.X + (valid ? row : (n - 1)) * DP + 8 * h;

    // B operand: lane (r, h) holds features [16t + 8h, 16t + 8h + 8) of point r
    f16x8 bh[NS], bl[NS];
    float xx = 0.0f;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const float4 v0 = *reinterpret_cast<const float4*>(xr + 16 * t);
      const float4 v1 = *reinterpret_cast<const float4*>(xr + 16 * t + 4);
      const float xv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xs = xv[e] * s;
        const _Float16 hi = (_Float16)xs;
        bh[t][e] = hi;
        bl[t][e] = (_Float16)(xs - (float)hi);
        xx = fmaf(xs, xs, xx);
      }
    }
    xx += __shfl_xor(xx, 32);

    float a1[4], a2[4], a3[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a1[c] = a2[c] = a3[c] = FLT_MAX;

    auto init_acc = [&](int blk) {
      f32x16 acc;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 cv = *reinterpret_cast<const float4*>(laneCn + blk * 32 + 8 * g4);
        acc[4 * g4 + 0] = cv.x;
        acc[4 * g4 + 1] = cv.y;
        acc[4 * g4 + 2] = cv.z;
        acc[4 * g4 + 3] = cv.w;
      }
      return acc;
    };
    struct Frag {
      f16x8 hi, lo;
    };
    auto load_frag = [&](int blk, int t) {
      const size_t off = (size_t)blk * BLKB + (size_t)t * 1024;
      Frag f;
      f.hi = *reinterpret_cast<const f16x8*>(laneHi + off);
      f.lo = *reinterpret_cast<const f16x8*>(laneLo + off);
      return f;
    };
    auto mfma3 = [&](f32x16 acc, const Frag& f, int t) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.hi, bl[t], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.lo, bh[t], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.hi, bh[t], acc, 0, 0, 0);
      return acc;
    };
    // register reg of block blk holds centroid j = 32*blk + 4h + (reg&3) + 8*(reg>>2);
    // chain reg&3 stores j >> 2 = (8*blk + h) | 2*(reg>>2) in the key
    uint32_t jg[4];
    auto set_jg = [&](uint32_t jq) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        jg[g] = jq | (uint32_t)(2 * g);
        asm volatile("" : "+v"(jg[g]));  // keep it a register: one v_and_or per key
      }
    };
    auto key_update = [&](const f32x16& acc, int reg) {
      const float key = __uint_as_float((__float_as_uint(acc[reg]) & ~maskq) | jg[reg >> 2]);
      if constexpr (T2) {
        const int c = reg & 3;
        const float n1 = __builtin_amdgcn_fmed3f(a1[c], key, -FLT_MAX);
        a2[c] = __builtin_amdgcn_fmed3f(a1[c], a2[c], key);
        a1[c] = n1;
      } else {
        top3_insert(a1[reg & 3], a2[reg & 3], a3[reg & 3], key);
      }
    };
    // top-2 chains: registers ra = 8 (pp >> 2) + (pp & 3) and ra + 4 (one
    // chain) folded in together, 5 VALU per 2 keys (as in k_fused)
    auto key_pair = [&](const f32x16& acc, int pp) {
      const int c = pp & 3, ra = 8 * (pp >> 2) + c, rb = ra + 4;
      const float ka = __uint_as_float((__float_as_uint(acc[ra]) & ~maskq) | jg[ra >> 2]);
      const float kb = __uint_as_float((__float_as_uint(acc[rb]) & ~maskq) | jg[rb >> 2]);
      const float tm = __builtin_amdgcn_fmed3f(a1[c], ka, kb);
      a1[c] = __builtin_fminf(__builtin_fminf(a1[c], ka), kb);
      a2[c] = __builtin_fminf(a2[c], tm);
    };
    // MFMAs of block `blk` into `cur` while the 16 key updates of the
    // previous block (`prev`, index words already in jg) fill the gaps.  A
    // fragments are prefetched one K-step ahead (into the next block at the
    // last step) so no MFMA waits on its own LDS read.
    Frag fr = load_frag(0, 0);
    auto overlapped = [&](f32x16& cur, int blk, int nblk, const f32x16& prev) {
      cur = init_acc(blk);
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        const Frag nx = (t + 1 < NS) ? load_frag(blk, t + 1) : load_frag(blk + 1 < nblk ? blk + 1 : blk, 0);
        cur = mfma3(cur, fr, t);
        if constexpr (T2) {
#pragma unroll
          for (int pp = 0; pp < 8; ++pp)
            if (pp * NS / 8 == t) key_pair(prev, pp);
        } else {
#pragma unroll
          for (int rr = 0; rr < 16; ++rr)
            if (rr * NS / 16 == t) key_update(prev, rr);
        }
        fr = nx;
      }
    };

    for (int ch = 0; ch < nchunks; ++ch) {
      if (nchunks > 1) {
        // this chunk's DMA landed: LDS-DMA completion is tracked only by the
        // issuing wave's vmcnt, and a workgroup barrier on gfx950 does not
        // drain it (the compiler inserts no vmcnt wait before s_barrier), so
        // every wave waits for its own pieces first, then for everyone's
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // ... and the other buffer is no longer read
        point_at(cbuf);
        if (ch + 1 < nchunks)
          stage_async(ch + 1, cbuf ^ 1);
        else if (wt + gridDim.x < nwt)
          stage_async(0, cbuf ^ 1);  // the next tile group starts over at chunk 0
        cbuf ^= 1;
        fr = load_frag(0, 0);
      }
      const int nb = min(KC, kp - ch * KC) / 32;  // even: kp and KC are multiples of 64
      const uint32_t jq0 = (uint32_t)((ch * KC) >> 2) + (uint32_t)h;
      f32x16 accA = init_acc(0), accB;
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        const Frag nx = (t + 1 < NS) ? load_frag(0, t + 1) : load_frag(1, 0);
        accA = mfma3(accA, fr, t);
        fr = nx;
      }
      int blk = 1;
      for (; blk + 1 < nb; blk += 2) {
        set_jg(jq0 + 8u * (uint32_t)(blk - 1));
        overlapped(accB, blk, nb, accA);
        set_jg(jq0 + 8u * (uint32_t)blk);
        overlapped(accA, blk + 1, nb, accB);
      }
      set_jg(jq0 + 8u * (uint32_t)(blk - 1));
      overlapped(accB, blk, nb, accA);
      set_jg(jq0 + 8u * (uint32_t)blk);
      if constexpr (T2) {
#pragma unroll
        for (int pp = 0; pp < 8; ++pp) key_pair(accB, pp);
      } else {
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) key_update(accB, rr);
      }
    }
    if (nchunks > 1 && tile >= ntiles) continue;

    // exact merge of the 4 chains, carrying full indices of the best two
    float k1 = FLT_MAX, k2 = FLT_MAX, k3 = FLT_MAX;
    uint32_t p1 = 0, p2 = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      top3p_insert(k1, k2, k3, p1, p2, a1[c], ((__float_as_uint(a1[c]) & maskq) << 2) | (uint32_t)c);
      top3p_insert(k1, k2, k3, p1, p2, a2[c], ((__float_as_uint(a2[c]) & maskq) << 2) | (uint32_t)c);
      // a 3rd never enters the top two; with T2 the chain's dropped keys are
      // only known to be >= its second, which stands in for its third
      top3p_insert(k1, k2, k3, p1, p2, T2 ? a2[c] : a3[c], 0u);
    }
    {  // the two lane halves hold disjoint centroid rows of the same point
      const float q1 = __shfl_xor(k1, 32), q2 = __shfl_xor(k2, 32), q3 = __shfl_xor(k3, 32);
      const uint32_t r1 = __shfl_xor(p1, 32), r2 = __shfl_xor(p2, 32);
      top3p_insert(k1, k2, k3, p1, p2, q1, r1);
      top3p_insert(k1, k2, k3, p1, p2, q2, r2);
      top3p_insert(k1, k2, k3, p1, p2, q3, 0u);
    }
    // Rigorous bound on |K_j - s^2 (||x - c_j||^2 - ||x||^2)| (DESIGN.md
    // "Exactness"): fp16x3 split residuals, fp64->fp32 rounding of c, fp32
    // accumulation, ||c||^2 rounding, fp16 underflow (B0); plus the key
    // truncation rho*|K|.  x1.5 safety.
    const float xn = sqrtf(xx) * 1.0001f;
    const float B0 = screen_b0(xn, cm, pm, DP);
    const float thr3 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k3));
    const float thr2 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k2));
    // negated tests: NaN (non-finite data) falls through to the full float64
    // scan, whose np.argmin semantics then pick the first index
    uint32_t kind = 0;
    bool same_chain = false;
    if constexpr (T2) {
      // p1, p2 in one chain (same j & 7): no certificate for the pair
      same_chain = ((p1 ^ p2) & 7u) == 0u;
      if (!(k2 - k1 > thr2)) kind = (same_chain || !(k3 - k1 > thr3)) ? 2u : 1u;
    } else {
      if (!(k3 - k1 > thr3))
        kind = 2;
      else if (!(k2 - k1 > thr2))
        kind = 1;
    }
    // per-key bounds where the global test failed (wave-uniform branch)
    if (__ballot(kind != 0u) != 0ull && kind != 0u) {
      const KeyBounds kb = key_bounds(xn, *A.xabs * s, DP, rho);
      const float u1 = kb.upper(k1);
      if (u1 < kb.lower(k2))
        kind = 0u;  // every other centroid (key >= k2) is provably worse
      else if (kind == 2u && !same_chain && kb.lower(k3) > u1)
        kind = 1u;  // the rest (key >= k3) is worse than i1: the answer is i1 or i2
    }
    // Candidate lists (kind 4) instead of full scans.  A kind-2 point has more
    // than two keys within the bound of k1, but each chain keeps its best keys
    // with their indices (top 3: two indexed, T2: one) and knows that every key
    // it dropped is >= its guard (third, T2: second).  When no chain's guard is
    // within the bound, every centroid that can be the argmin is one of the kept
    // keys within it: those few are re-ranked in float64 (k_rerank2) instead
    // of a scan over all k.  Exactness as for kind 1: the true argmin j* has
    // S_j* <= S_p1, so its key passes the same two tests that exclude the others.
    if (A.cand != nullptr && __ballot(kind == 2u) != 0ull) {
      uint32_t cj[8];  // this lane half's kept candidates (0xffffffff: none)
      bool over = !(k1 == k1) || !(fabsf(k1) < 3.0e38f);
      if (kind == 2u) {
        const KeyBounds kb = key_bounds(xn, *A.xabs * s, DP, rho);
        const float u1 = kb.upper(k1);
        auto maybe = [&](float v) {  // v's centroid may be the argmin (NaN: yes)
          return !(v - k1 > 2.0f * B0 + rho * (fabsf(k1) + fabsf(v))) && !(kb.lower(v) > u1);
        };
        auto idx = [&](float v, int c) { return ((__float_as_uint(v) & maskq) << 2) | (uint32_t)c; };
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float g = T2 ? a2[c] : a3[c];
          over |= maybe(g);
          cj[2 * c] = maybe(a1[c]) ? idx(a1[c], c) : 0xffffffffu;
          cj[2 * c + 1] = (!T2 && maybe(a2[c])) ? idx(a2[c], c) : 0xffffffffu;
        }
      } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) cj[c] = 0xffffffffu;
      }
      // the other lane half's chains (same point)
      uint32_t co[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) co[c] = __shfl_xor(cj[c], 32);
      over |= __shfl_xor((int)over, 32) != 0;
      int nc = 0;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        nc += cj[c] < (uint32_t)A.k;
        nc += co[c] < (uint32_t)A.k;
      }
      const bool want = h == 0 && valid && kind == 2u && !over && nc >= 1 && nc < CAND_REC;
      const uint64_t m4 = __ballot(want);
      if (m4) {
        const int leader = __ffsll((unsigned long long)m4) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(A.cand_ctr, (uint32_t)__popcll(m4));
        base = __shfl(base, leader);
        const uint32_t slot = base + (uint32_t)__popcll(m4 & ((1ull << lane) - 1ull));
        if (want && slot < A.cand_cap) {
          // ascending index order (np.argmin's tie-break in k_rerank2)
          uint32_t v[16];
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            v[c] = cj[c] < (uint32_t)A.k ? cj[c] : 0xffffffffu;
            v[8 + c] = co[c] < (uint32_t)A.k ? co[c] : 0xffffffffu;
          }
#pragma unroll
          for (int i = 1; i < 16; ++i)
#pragma unroll
            for (int j2 = i; j2 > 0; --j2) {
              const uint32_t lo = min(v[j2 - 1], v[j2]), hi = max(v[j2 - 1], v[j2]);
              v[j2 - 1] = lo;
              v[j2] = hi;
            }
          uint32_t* rec = A.cand + (size_t)slot * CAND_REC;
          rec[0] = (uint32_t)nc;
#pragma unroll
          for (int i = 0; i < CAND_REC - 1; ++i) rec[1 + i] = v[i];
          kind = 4u;
          p2 = slot;
        }
      }
    }
    const int lab = (p1 < (uint32_t)A.k) ? (int)p1 : 0;
    if (h == 0 && valid) A.labels[row] = lab;
    const bool enq = (h == 0) && valid && (kind != 0);
    const uint64_t m = __ballot(enq);
    if (m) {
      // re-rank and candidate-list entries fill the wave's segment from the
      // front, full scans from the back (resolved by different kernels)
      const uint64_t m1 = __ballot(enq && (kind == 1 || kind == 4));
      const uint64_t m2 = m & ~m1;
      const uint64_t below = (1ull << lane) - 1ull;
      if (enq) {
        QEntry q;
        q.row = (uint32_t)row;
        q.i1 = p1;
        q.i2 = p2;
        q.kind = kind;
        const uint32_t pos = (kind == 1 || kind == 4) ? qn + (uint32_t)__popcll(m1 & below)
                                                      : A.seg - 1u - (qf + (uint32_t)__popcll(m2 & below));
        wq[pos] = q;
      }
      qn += (uint32_t)__popcll(m1);
      qf += (uint32_t)__popcll(m2);
    }
  }
  if (lane == 0) {
    A.qcount[2 * gw] = qn;
    A.qcount[2 * gw + 1] = qf;
  }
}

// ---------------------------------------------------------------------------
// Screening for rows wider than 256 features (kmeans_spark.py:153 takes any
// row length), where the x tile no longer fits the registers whole.  Pieces of
// WIDE_KC = 256 centroids x WIDE_FW = 64 features (8 MFMA blocks x 4 K-steps,
// the lane-linear fp16 hi/lo image of k_assign_mfma, 64 KiB + the chunk's
// ||c||^2) stream through two LDS buffers by LDS-DMA, one piece ahead, with one
// barrier per piece; 8 waves (2 per SIMD), each on its own 32 rows, run the 3
// MFMAs per block and K-step into 8 accumulators (128 VGPRs) carried across
// the feature pieces, the rows' next feature slice loaded one piece ahead.
// Keys, chains, the rigorous bound and the queue are those of k_assign_mfma
// (top-3 chains).  X is read once per centroid chunk (once for k <= 256).
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// k_assign_mfma16: k_assign_mfma on v_mfma_f32_16x16x32_f16 (dp a multiple of
// 32).  Same chunked LDS images, LDS-DMA and queue / candidate-list logic, the
// same 32 rows per wave; a block of 32 centroids is two 16-centroid halves
// (cb) x two 16-row groups (pg), and an image piece (blk, cb NS/2 + sl) holds,
// lane l, the 8 halves of centroid 32 blk + 16 cb + (l & 15), features
// 32 sl + 8 (l >> 4).  On the MFMA-only ablation at c5 (12 waves) the shape
// runs 2.12 vs 1.92 GHz at equal MFMA busy: 109 vs 121 ms (DESIGN.md
// section 4).  Chains are (j & 3, quarter q = l >> 4) per row group: 16 per
// row; after the chunks the row groups are reduce-scattered over the lane
// halves and merged over quarter pairs (as k_fused16), so lanes l and l ^ 16
// own row (l & 15) + 16 (l >> 5).  The bound is screen_b0's 16x16x32 model.
// ---------------------------------------------------------------------------
template <int NS, int WAVES, bool T2 = false, bool ONE = false>
__global__ __launch_bounds__(WAVES * 64, (mfma_min_waves<NS, WAVES>())) void k_assign_mfma16(MfmaArgs A) {
  if (*A.gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  static_assert(NS % 2 == 0, "dp a multiple of 32");
  constexpr int DP = 16 * NS;
  constexpr int NS2 = NS / 2;      // 32-feature slabs
  constexpr int BLKB = NS * 1024;  // bytes of one block's fragments (one of hi / lo)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KC = A.KC;
  const size_t himg = (size_t)(KC / 32) * BLKB;
  const size_t bufsz = ((2 * himg + (size_t)KC * 4) + 15) / 16 * 16;
  char* sHi = smem;
  char* sLo = smem + himg;
  float* sCn = reinterpret_cast<float*>(smem + 2 * himg);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c16 = lane & 15;
  const int q = lane >> 4;
  const int pgo = lane >> 5;           // the row group this lane owns after the merge
  const int prow = c16 + 16 * pgo;     // its row within the tile
  const int kp = A.kp;
  const int64_t n = A.n;
  const int b = ceil_log2(kp);  // kp is a multiple of 64: b >= 6
  const uint32_t maskq = (1u << (b - 2)) - 1u;
  const float s = mfma_scale(*A.xabs, *A.cabs);
  const float cm = *A.cmax * s;
  const float pm = (*A.cabs * s) * (*A.xabs * s) * 1.0001f;
  const float rho = __builtin_ldexpf(1.0f, b - 2 - 23) * 1.01f;  // key truncation (relative)
  const int nchunks = (kp + KC - 1) / KC;
  const int64_t ntiles = (n + 31) / 32;
  const int64_t nwt = (ntiles + WAVES - 1) / WAVES;

  // piece pc = blk NS + tt of a chunk, tt = cb NS2 + sl: lane l's 16 bytes
  auto piece_src = [&](int pc, int l) {
    const int blk = pc / NS, tt = pc - blk * NS;
    const int cb = tt / NS2, sl = tt - cb * NS2;
    return ((size_t)(blk * 32 + 16 * cb + (l & 15)) * DP + 32 * sl + 8 * (l >> 4)) * 2;
  };
  auto stage = [&](int ch) {
    const int kc = min(KC, kp - ch * KC);
    const int npieces = (kc / 32) * NS * 64;
    const char* gh = reinterpret_cast<const char*>(A.Chi + (size_t)ch * KC * DP);
    const char* gl = reinterpret_cast<const char*>(A.Clo + (size_t)ch * KC * DP);
    for (int id = threadIdx.x; id < npieces; id += WAVES * 64) {
      const size_t src = piece_src(id >> 6, id & 63);
      *reinterpret_cast<uint4*>(sHi + (size_t)id * 16) = *reinterpret_cast<const uint4*>(gh + src);
      if constexpr (!ONE) *reinterpret_cast<uint4*>(sLo + (size_t)id * 16) = *reinterpret_cast<const uint4*>(gl + src);
    }
    for (int id = threadIdx.x; id < kc; id += WAVES * 64) sCn[id] = A.cn2s[(size_t)ch * KC + id];
  };
  auto stage_async = [&](int ch, int bf) {
    const int kc = min(KC, kp - ch * KC);
    const int npc = (kc / 32) * NS;
    char* dHi = smem + (size_t)bf * bufsz;
    char* dLo = dHi + himg;
    char* dCn = dHi + 2 * himg;
    const char* gh = reinterpret_cast<const char*>(A.Chi + (size_t)ch * KC * DP);
    const char* gl = reinterpret_cast<const char*>(A.Clo + (size_t)ch * KC * DP);
    for (int pc = wave; pc < npc; pc += WAVES) {
      const size_t src = piece_src(pc, lane);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(gh + src),
                                       (__attribute__((address_space(3))) void*)(dHi + (size_t)pc * 1024), 16, 0, 0);
      if constexpr (!ONE)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(gl + src),
                                         (__attribute__((address_space(3))) void*)(dLo + (size_t)pc * 1024), 16, 0, 0);
    }
    const char* gc = reinterpret_cast<const char*>(A.cn2s + (size_t)ch * KC);
    for (int pc = wave; pc * 1024 < kc * 4; pc += WAVES)
      if (pc * 1024 + lane * 16 < kc * 4)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(gc + pc * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(dCn + pc * 1024), 16, 0, 0);
  };

  int cbuf = 0;
  if (nchunks == 1) {
    stage(0);
    __syncthreads();
  } else if ((int64_t)blockIdx.x < nwt) {
    stage_async(0, 0);
  }

  const uint32_t gw = blockIdx.x * WAVES + wave;
  QEntry* wq = A.queue + (size_t)gw * A.seg;
  uint32_t qn = 0, qf = 0, cc = 0;
  uint2* wc = A.chg != nullptr ? A.chg + (size_t)gw * A.seg : nullptr;
  const char* laneHi = sHi + lane * 16;
  const char* laneLo = sLo + lane * 16;
  const float* laneCn = sCn + 4 * q;
  auto point_at = [&](int bf) {
    laneHi = smem + (size_t)bf * bufsz + lane * 16;
    laneLo = laneHi + himg;
    laneCn = reinterpret_cast<const float*>(smem + (size_t)bf * bufsz + 2 * himg) + 4 * q;
  };

  for (int64_t wt = blockIdx.x; wt < nwt; wt += gridDim.x) {
    const int64_t tile = wt * WAVES + wave;
    if (nchunks == 1 && tile >= ntiles) break;  // no barriers below in this mode
    const int64_t row = tile * 32 + prow;       // the row this lane owns after the merge
    const bool valid = row < n;
    // delta statistics: the row's previous label, loaded now (used at the end)
    const int32_t old_raw = (wc != nullptr && valid) ? A.labels[row] : 0;

    // B operands: lane l holds features 32 sl + 8 q .. + 8 of rows 16 pg + (l & 15)
    f16x8 bh[2][NS2], bl[2][NS2];
    float xx[2] = {0.0f, 0.0f};
#pragma unroll
    for (int pg = 0; pg < 2; ++pg) {
      const int64_t rg = tile * 32 + 16 * pg + c16;
      const float* xr = A.X + (rg < n ? rg : (n - 1)) * DP + 8 * q;
#pragma unroll
      for (int sl = 0; sl < NS2; ++sl) {
        const float4 v0 = *reinterpret_cast<const float4*>(xr + 32 * sl);
        const float4 v1 = *reinterpret_cast<const float4*>(xr + 32 * sl + 4);
        const float xv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xs = xv[e] * s;
          const _Float16 hi = (_Float16)xs;
          bh[pg][sl][e] = hi;
          bl[pg][sl][e] = (_Float16)(xs - (float)hi);
          xx[pg] = fmaf(xs, xs, xx[pg]);
        }
      }
    }
#pragma unroll
    for (int pg = 0; pg < 2; ++pg) {  // the four quarters hold disjoint features of a row
      xx[pg] += __shfl_xor(xx[pg], 16);
      xx[pg] += __shfl_xor(xx[pg], 32);
    }

    float a1[2][4], a2[2][4], a3[2][4];
#pragma unroll
    for (int pg = 0; pg < 2; ++pg)
#pragma unroll
      for (int c = 0; c < 4; ++c) a1[pg][c] = a2[pg][c] = a3[pg][c] = FLT_MAX;

    struct Acc {
      f32x4 v[2][2];  // [cb][pg]
    };
    auto init_acc = [&](int blk) {
      Acc a;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const float4 cv = *reinterpret_cast<const float4*>(laneCn + blk * 32 + 16 * cb);
        const f32x4 c4 = {cv.x, cv.y, cv.z, cv.w};
        a.v[cb][0] = c4;
        a.v[cb][1] = c4;
      }
      return a;
    };
    struct Frag {
      f16x8 hi, lo;
    };
    auto load_frag = [&](int blk, int tt) {
      const size_t off = (size_t)blk * BLKB + (size_t)tt * 1024;
      Frag f;
      f.hi = *reinterpret_cast<const f16x8*>(laneHi + off);
      if constexpr (!ONE) f.lo = *reinterpret_cast<const f16x8*>(laneLo + off);
      return f;
    };
    // piece tt = cb NS2 + sl: the half cb's contribution of slab sl, both row groups
    auto mfma_step = [&](Acc& a, const Frag& f, int tt) {
      const int cb = tt / NS2, sl = tt - (tt / NS2) * NS2;
      if constexpr (!ONE) {
#pragma unroll
        for (int pg = 0; pg < 2; ++pg)
          a.v[cb][pg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.hi, bl[pg][sl], a.v[cb][pg], 0, 0, 0);
#pragma unroll
        for (int pg = 0; pg < 2; ++pg)
          a.v[cb][pg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.lo, bh[pg][sl], a.v[cb][pg], 0, 0, 0);
      }
#pragma unroll
      for (int pg = 0; pg < 2; ++pg)
        a.v[cb][pg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.hi, bh[pg][sl], a.v[cb][pg], 0, 0, 0);
    };
    // register i of accumulator (cb, pg): centroid j = 32 blk + 16 cb + 4 q + i;
    // chain (i, q) of row group pg stores j >> 2 = 8 blk + 4 cb + q in the key
    uint32_t jg[2];
    auto set_jg = [&](uint32_t jq) {  // jq = j >> 2 of the block's cb = 0, q = 0 (+ q added)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        jg[cb] = jq + 4u * (uint32_t)cb + (uint32_t)q;
        asm volatile("" : "+v"(jg[cb]));  // keep it a register: one v_and_or per key
      }
    };
    auto key_of2 = [&](float v, int cb) { return __uint_as_float((__float_as_uint(v) & ~maskq) | jg[cb]); };
    // update u of the block's 16 (T2: 8 pairs): pg = u >> 3, c = u & 3 (T2: u = 4 pg + c)
    auto key_update = [&](const Acc& a, int u) {
      const int pg = u >> 3, cb = (u >> 2) & 1, c = u & 3;
      top3_insert(a1[pg][c], a2[pg][c], a3[pg][c], key_of2(a.v[cb][pg][c], cb));
    };
    auto key_pair = [&](const Acc& a, int u) {
      const int pg = u >> 2, c = u & 3;
      const float ka = key_of2(a.v[0][pg][c], 0);
      const float kb = key_of2(a.v[1][pg][c], 1);
      const float tm = __builtin_amdgcn_fmed3f(a1[pg][c], ka, kb);
      a1[pg][c] = __builtin_fminf(__builtin_fminf(a1[pg][c], ka), kb);
      a2[pg][c] = __builtin_fminf(a2[pg][c], tm);
    };
    Frag fr = load_frag(0, 0);
    auto overlapped = [&](Acc& cur, int blk, int nblk, const Acc& prev) {
      cur = init_acc(blk);
#pragma unroll
      for (int tt = 0; tt < NS; ++tt) {
        const Frag nx = (tt + 1 < NS) ? load_frag(blk, tt + 1) : load_frag(blk + 1 < nblk ? blk + 1 : blk, 0);
        mfma_step(cur, fr, tt);
        if constexpr (T2) {
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (u * NS / 8 == tt) key_pair(prev, u);
        } else {
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (u * NS / 16 == tt) key_update(prev, u);
        }
        fr = nx;
      }
    };

    for (int ch = 0; ch < nchunks; ++ch) {
      if (nchunks > 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces (see k_assign_mfma)
        __syncthreads();
        point_at(cbuf);
        if (ch + 1 < nchunks)
          stage_async(ch + 1, cbuf ^ 1);
        else if (wt + gridDim.x < nwt)
          stage_async(0, cbuf ^ 1);
        cbuf ^= 1;
        fr = load_frag(0, 0);
      }
      const int nb = min(KC, kp - ch * KC) / 32;  // even
      const uint32_t jq0 = (uint32_t)((ch * KC) >> 2);
      Acc accA = init_acc(0), accB;
#pragma unroll
      for (int tt = 0; tt < NS; ++tt) {
        const Frag nx = (tt + 1 < NS) ? load_frag(0, tt + 1) : load_frag(1, 0);
        mfma_step(accA, fr, tt);
        fr = nx;
      }
      int blk = 1;
      for (; blk + 1 < nb; blk += 2) {
        set_jg(jq0 + 8u * (uint32_t)(blk - 1));
        overlapped(accB, blk, nb, accA);
        set_jg(jq0 + 8u * (uint32_t)blk);
        overlapped(accA, blk + 1, nb, accB);
      }
      set_jg(jq0 + 8u * (uint32_t)(blk - 1));
      overlapped(accB, blk, nb, accA);
      set_jg(jq0 + 8u * (uint32_t)blk);
      if constexpr (T2) {
#pragma unroll
        for (int u = 0; u < 8; ++u) key_pair(accB, u);
      } else {
#pragma unroll
        for (int u = 0; u < 16; ++u) key_update(accB, u);
      }
    }
    if (nchunks > 1 && tile >= ntiles) continue;

    // per row group: this lane's 4 chains merged, full indices of the best two
    auto idx = [&](float v, int c) { return ((__float_as_uint(v) & maskq) << 2) | (uint32_t)c; };
    float g1[2], g2[2], g3[2];
    uint32_t gp1[2], gp2[2];
#pragma unroll
    for (int pg = 0; pg < 2; ++pg) {
      float k1 = FLT_MAX, k2 = FLT_MAX, k3 = FLT_MAX;
      uint32_t p1 = 0, p2 = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        top3p_insert(k1, k2, k3, p1, p2, a1[pg][c], idx(a1[pg][c], c));
        top3p_insert(k1, k2, k3, p1, p2, a2[pg][c], idx(a2[pg][c], c));
        top3p_insert(k1, k2, k3, p1, p2, T2 ? a2[pg][c] : a3[pg][c], 0u);
      }
      g1[pg] = k1;
      g2[pg] = k2;
      g3[pg] = k3;
      gp1[pg] = p1;
      gp2[pg] = p2;
    }
    float k1, k2, k3;
    uint32_t p1, p2;
    {  // reduce-scatter over the lane halves, then the quarter pairs (lower lane's side first)
      uint32_t K1, Q1, K2, Q2, K3, Q3, P1, R1, P2, R2;
      swap_halves(__float_as_uint(g1[0]), __float_as_uint(g1[1]), K1, Q1);
      swap_halves(__float_as_uint(g2[0]), __float_as_uint(g2[1]), K2, Q2);
      swap_halves(__float_as_uint(g3[0]), __float_as_uint(g3[1]), K3, Q3);
      swap_halves(gp1[0], gp1[1], P1, R1);
      swap_halves(gp2[0], gp2[1], P2, R2);
      k1 = __uint_as_float(K1);
      k2 = __uint_as_float(K2);
      k3 = __uint_as_float(K3);
      p1 = P1;
      p2 = P2;
      top3p_insert(k1, k2, k3, p1, p2, __uint_as_float(Q1), R1);
      top3p_insert(k1, k2, k3, p1, p2, __uint_as_float(Q2), R2);
      top3p_insert(k1, k2, k3, p1, p2, __uint_as_float(Q3), 0u);
    }
    {
      uint32_t K1, Q1, K2, Q2, K3, Q3, P1, R1, P2, R2;
      perm_quarters(__float_as_uint(k1), K1, Q1);
      perm_quarters(__float_as_uint(k2), K2, Q2);
      perm_quarters(__float_as_uint(k3), K3, Q3);
      perm_quarters(p1, P1, R1);
      perm_quarters(p2, P2, R2);
      k1 = __uint_as_float(K1);
      k2 = __uint_as_float(K2);
      k3 = __uint_as_float(K3);
      p1 = P1;
      p2 = P2;
      top3p_insert(k1, k2, k3, p1, p2, __uint_as_float(Q1), R1);
      top3p_insert(k1, k2, k3, p1, p2, __uint_as_float(Q2), R2);
      top3p_insert(k1, k2, k3, p1, p2, __uint_as_float(Q3), 0u);
    }
    const float xn = sqrtf(xx[pgo]) * 1.0001f;
    const float B0 = ONE ? screen_b0_one(xn, cm, pm, DP) : screen_b0(xn, cm, pm, DP, 1);
    const float thr3 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k3));
    const float thr2 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k2));
    uint32_t kind = 0;
    bool same_chain = false;
    if constexpr (T2) {
      same_chain = ((p1 ^ p2) & 15u) == 0u;  // chain (j & 3, quarter): j & 15
      if (!(k2 - k1 > thr2)) kind = (same_chain || !(k3 - k1 > thr3)) ? 2u : 1u;
    } else {
      if (!(k3 - k1 > thr3))
        kind = 2;
      else if (!(k2 - k1 > thr2))
        kind = 1;
    }
    float u1 = FLT_MAX;
    if (__ballot(kind != 0u) != 0ull && kind != 0u) {
      const KeyBounds kb = ONE ? key_bounds_one(xn, *A.xabs * s, DP, rho) : key_bounds(xn, *A.xabs * s, DP, rho, 1);
      u1 = kb.upper(k1);
      if (u1 < kb.lower(k2))
        kind = 0u;
      else if (kind == 2u && !same_chain && kb.lower(k3) > u1)
        kind = 1u;
    }
    if constexpr (ONE) {
      // The one-part bound leaves many pairs to the float64 re-rank (13% of
      // c5 rows): re-score the pair in fp32 here first.  The two owner lanes
      // of a row take half of its features each; bounds of ||x - c||
      // (unscaled): |Dt - D'| <= (dp/2 + 4) u D' for the lane sums and their
      // sum, sqrt(D') = r (1 +- (dp/4 + 2 + 4) u) with v_sqrt_f32 (2 ulp),
      // widened by 8 u, and ||x - c|| = sqrt(D') +- u cmax (c vs its fp32 c').
      // Below 2^-96 the hardware sqrt loses accuracy: U takes sqrt(2^-96),
      // L takes 0.  Decided when one candidate's upper bound is below the
      // other's lower bound; otherwise the pair stays for k_rerank2.
      if (A.C32 != nullptr && __ballot(kind == 1u && valid) != 0ull) {
        const bool act = kind == 1u && valid;
        constexpr int HF = DP / 2;  // features per owner lane
        const int hb = (q & 1) * HF;
        const float4* xr = reinterpret_cast<const float4*>(A.X + (size_t)(act ? row : 0) * DP + hb);
        const float4* c1 = reinterpret_cast<const float4*>(A.C32 + (size_t)(act ? p1 : 0) * DP + hb);
        const float4* c2 = reinterpret_cast<const float4*>(A.C32 + (size_t)(act ? p2 : 0) * DP + hb);
        float d1 = 0.0f, d2 = 0.0f;
#pragma unroll 1
        for (int u = 0; u < HF / 4; ++u) {
          const float4 xv = xr[u], a = c1[u], b = c2[u];
          float t;
          t = xv.x - a.x; d1 = fmaf(t, t, d1);
          t = xv.y - a.y; d1 = fmaf(t, t, d1);
          t = xv.z - a.z; d1 = fmaf(t, t, d1);
          t = xv.w - a.w; d1 = fmaf(t, t, d1);
          t = xv.x - b.x; d2 = fmaf(t, t, d2);
          t = xv.y - b.y; d2 = fmaf(t, t, d2);
          t = xv.z - b.z; d2 = fmaf(t, t, d2);
          t = xv.w - b.w; d2 = fmaf(t, t, d2);
        }
        // the partner lane (l ^ 16) holds the other half; the same order of
        // addition in both (lower half first)
        const float o1 = __shfl_xor(d1, 16), o2 = __shfl_xor(d2, 16);
        const float D1 = (q & 1) ? o1 + d1 : d1 + o1;
        const float D2 = (q & 1) ? o2 + d2 : d2 + o2;
        constexpr float EPS = (float)(DP / 4 + 14) * U24;
        const float gm = U24 * *A.cmax * 1.01f + 1e-37f;
        auto ub = [&](float D) {
          const float r = __builtin_amdgcn_sqrtf(D >= 0x1p-96f ? D : 0x1p-96f);
          return fmaf(r, 1.0f + EPS, gm) * (1.0f + 4.0f * U24);
        };
        auto lb = [&](float D) {
          const float r = D >= 0x1p-96f ? __builtin_amdgcn_sqrtf(D) : 0.0f;
          return fmaf(r, 1.0f - EPS, -gm) * (1.0f - 4.0f * U24);
        };
        const float U1 = ub(D1), L1 = lb(D1), U2 = ub(D2), L2 = lb(D2);
        const bool win1 = act && L2 > U1, win2 = act && L1 > U2;
        // (select form: DESIGN.md section 2)
        p1 = win2 ? p2 : p1;
        kind = (win1 || win2) ? 0u : kind;
      }
    }
    // Candidate lists (kind 4), as in k_assign_mfma: the row's 16 chains
    // are spread over the four quarter lanes of its column, each holding
    // them for both row groups; every lane lists the kept keys of its own
    // chains that may be the argmin of either row, then the owner lanes
    // gather the four quarters' lists of their row.
    if (A.cand != nullptr && __ballot(kind == 2u) != 0ull) {
      // the other row group's k1, u1, B0 and kind from its owner lanes
      uint32_t k1o[2], u1o[2], b0o[2], kdo[2];
      perm_halves(__float_as_uint(k1), k1o[0], k1o[1]);
      perm_halves(__float_as_uint(u1), u1o[0], u1o[1]);
      perm_halves(__float_as_uint(B0), b0o[0], b0o[1]);
      perm_halves(kind, kdo[0], kdo[1]);
      // per row group: that row's bound state, for this lane's chains
      KeyBounds kbg[2];
      bool act[2], over[2];
#pragma unroll
      for (int pg = 0; pg < 2; ++pg) {
        act[pg] = kdo[pg] == 2u;
        kbg[pg] = ONE ? key_bounds_one(sqrtf(xx[pg]) * 1.0001f, *A.xabs * s, DP, rho)
                      : key_bounds(sqrtf(xx[pg]) * 1.0001f, *A.xabs * s, DP, rho, 1);
        const float K1 = __uint_as_float(k1o[pg]);
        over[pg] = act[pg] && (!(K1 == K1) || !(fabsf(K1) < 3.0e38f));
      }
      auto maybe = [&](float v, int pg) {  // v's centroid may be row pg's argmin (NaN: yes)
        const float K1 = __uint_as_float(k1o[pg]), U1 = __uint_as_float(u1o[pg]), BB = __uint_as_float(b0o[pg]);
        return act[pg] && !(v - K1 > 2.0f * BB + rho * (fabsf(K1) + fabsf(v))) && !(kbg[pg].lower(v) > U1);
      };
      // the owner's row collects the kept keys of the row's 16 chains (its
      // own quarter and the other three), in ascending order: each value is
      // bubbled into a sorted list of CAND_REC - 1 (np.argmin's tie-break in
      // k_rerank2; indices are distinct)
      uint32_t srt[CAND_REC - 1];
#pragma unroll
      for (int i = 0; i < CAND_REC - 1; ++i) srt[i] = 0xffffffffu;
      int nc = 0;
      auto collect = [&](uint32_t c0v, uint32_t c1v) {  // this lane's entry for row groups 0 and 1
        uint32_t h0, h1, w[4];
        swap_halves(c0v, c1v, h0, h1);
        perm_quarters(h0, w[0], w[1]);
        perm_quarters(h1, w[2], w[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = w[e] < (uint32_t)A.k;
          nc += ok;
          uint32_t x = ok ? w[e] : 0xffffffffu;
#pragma unroll
          for (int i = 0; i < CAND_REC - 1; ++i) {
            const uint32_t lo = min(srt[i], x), hi = max(srt[i], x);
            srt[i] = lo;
            x = hi;
          }
        }
      };
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int pg = 0; pg < 2; ++pg) over[pg] |= maybe(T2 ? a2[pg][c] : a3[pg][c], pg);
        collect(maybe(a1[0][c], 0) ? idx(a1[0][c], c) : 0xffffffffu, maybe(a1[1][c], 1) ? idx(a1[1][c], c) : 0xffffffffu);
        if constexpr (!T2)
          collect(maybe(a2[0][c], 0) ? idx(a2[0][c], c) : 0xffffffffu,
                  maybe(a2[1][c], 1) ? idx(a2[1][c], c) : 0xffffffffu);
      }
      uint32_t ov0, ov1, ovq[4];
      swap_halves((uint32_t)over[0], (uint32_t)over[1], ov0, ov1);
      perm_quarters(ov0, ovq[0], ovq[1]);
      perm_quarters(ov1, ovq[2], ovq[3]);
      const bool overall = (ovq[0] | ovq[1] | ovq[2] | ovq[3]) != 0u;
      const bool lead = (q & 1) == 0;
      const bool want = lead && valid && kind == 2u && !overall && nc >= 1 && nc < CAND_REC;
      const uint64_t m4 = __ballot(want);
      if (m4) {
        const int leader = __ffsll((unsigned long long)m4) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(A.cand_ctr, (uint32_t)__popcll(m4));
        base = __shfl(base, leader);
        const uint32_t slot = base + (uint32_t)__popcll(m4 & ((1ull << lane) - 1ull));
        if (want && slot < A.cand_cap) {
          uint32_t* rec = A.cand + (size_t)slot * CAND_REC;
          rec[0] = (uint32_t)nc;
#pragma unroll
          for (int i = 0; i < CAND_REC - 1; ++i) rec[1 + i] = srt[i];
          kind = 4u;
          p2 = slot;
        }
      }
    }
    const int lab = (p1 < (uint32_t)A.k) ? (int)p1 : 0;
    const bool lead = (q & 1) == 0;  // one lane of each pair (l, l ^ 16) writes
    if (wc == nullptr) {
      if (lead && valid) A.labels[row] = lab;
    } else {
      // decided rows whose label changed: written and listed; queued rows keep
      // their previous label (the resolvers compare and move them)
      const int old = (int)min((uint32_t)old_raw, (uint32_t)(A.k - 1));
      const bool changed = lead && valid && kind == 0u && lab != old;
      const uint64_t mc = __ballot(changed);
      if (mc) {
        if (changed) {
          A.labels[row] = lab;
          wc[cc + (uint32_t)__popcll(mc & ((1ull << lane) - 1ull))] =
              make_uint2((uint32_t)row, ((uint32_t)old << 16) | (uint32_t)lab);
        }
        cc += (uint32_t)__popcll(mc);
      }
    }
    const bool enq = lead && valid && (kind != 0);
    const uint64_t m = __ballot(enq);
    if (m) {
      const uint64_t m1 = __ballot(enq && (kind == 1 || kind == 4));
      const uint64_t m2 = m & ~m1;
      const uint64_t below = (1ull << lane) - 1ull;
      if (enq) {
        QEntry qe;
        qe.row = (uint32_t)row;
        qe.i1 = p1;
        qe.i2 = p2;
        qe.kind = kind;
        const uint32_t pos = (kind == 1 || kind == 4) ? qn + (uint32_t)__popcll(m1 & below)
                                                      : A.seg - 1u - (qf + (uint32_t)__popcll(m2 & below));
        wq[pos] = qe;
      }
      qn += (uint32_t)__popcll(m1);
      qf += (uint32_t)__popcll(m2);
    }
  }
  if (lane == 0) {
    A.qcount[2 * gw] = qn;
    A.qcount[2 * gw + 1] = qf;
    if (A.chg_cnt != nullptr) A.chg_cnt[gw] = cc;
  }
}

#ifndef KM_WIDE_FW
#define KM_WIDE_FW 64
#endif
static constexpr int WIDE_KC = 256, WIDE_FW = KM_WIDE_FW, WIDE_WAVES = 8;
static constexpr int WIDE_MAX_DP = 2048;  // k_fullscan stages 2 x 8 rows in LDS
static constexpr size_t WIDE_BUF = 2 * (size_t)(WIDE_KC / 32) * (WIDE_FW / 16) * 1024 + WIDE_KC * 4;

__global__ __launch_bounds__(WIDE_WAVES * 64, 2) void k_assign_wide(MfmaArgs A, int dp) {
  if (*A.gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  constexpr int NSW = WIDE_FW / 16;  // K-steps per feature piece
  constexpr int NBW = WIDE_KC / 32;  // MFMA blocks per centroid chunk
  constexpr int HIMG = NBW * NSW * 1024;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int kp = A.kp;
  const int64_t n = A.n;
  const int b = ceil_log2(kp);
  const uint32_t maskq = (1u << (b - 2)) - 1u;
  const float s = mfma_scale(*A.xabs, *A.cabs);
  const float cm = *A.cmax * s;
  const float pm = (*A.cabs * s) * (*A.xabs * s) * 1.0001f;
  const float rho = __builtin_ldexpf(1.0f, b - 2 - 23) * 1.01f;  // key truncation (relative)
  const int nkc = (kp + WIDE_KC - 1) / WIDE_KC;
  const int nfc = (dp + WIDE_FW - 1) / WIDE_FW;
  const int npc = nkc * nfc;  // pieces per tile group
  const int64_t ntiles = (n + 31) / 32;
  const int64_t nwt = (ntiles + WIDE_WAVES - 1) / WIDE_WAVES;

  // piece pc = ch * nfc + fc into buffer bf: fragment (blk, t) at (blk NSW + t)
  // KiB of each image, one 1 KiB LDS-DMA per wave-instruction
  auto stage_async = [&](int pc, int bf) {
    const int ch = pc / nfc, fc = pc - ch * nfc;
    const int nb = min(WIDE_KC, kp - ch * WIDE_KC) / 32;
    const int ns = min(WIDE_FW, dp - fc * WIDE_FW) / 16;
    char* dHi = smem + (size_t)bf * WIDE_BUF;
    for (int q = wave; q < NBW * NSW; q += WIDE_WAVES) {
      const int blk = q / NSW, t = q - blk * NSW;
      if (blk >= nb || t >= ns) continue;
      const size_t src = ((size_t)(ch * WIDE_KC + blk * 32 + r) * dp + fc * WIDE_FW + 16 * t + 8 * h) * 2;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(A.Chi) + src,
                                       (__attribute__((address_space(3))) void*)(dHi + (size_t)q * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(A.Clo) + src,
                                       (__attribute__((address_space(3))) void*)(dHi + HIMG + (size_t)q * 1024), 16,
                                       0, 0);
    }
    if (fc == 0 && wave == WIDE_WAVES - 1) {  // ||c||^2 s^2 of the chunk: nb * 128 bytes
      const char* gc = reinterpret_cast<const char*>(A.cn2s + (size_t)ch * WIDE_KC);
      if (lane * 16 < nb * 128)
        __builtin_amdgcn_global_load_lds(gc + lane * 16, (__attribute__((address_space(3))) void*)(dHi + 2 * HIMG),
                                         16, 0, 0);
    }
  };

  const uint32_t gw = blockIdx.x * WIDE_WAVES + wave;
  QEntry* wq = A.queue + (size_t)gw * A.seg;
  uint32_t qn = 0, qf = 0;
  int cbuf = 0;
  if ((int64_t)blockIdx.x < nwt) stage_async(0, 0);

  // every wave of the workgroup runs the same trip counts (barriers inside);
  // a tile past the end computes on row n - 1 and is dropped at the end
  for (int64_t wt = blockIdx.x; wt < nwt; wt += gridDim.x) {
    const int64_t tile = wt * WIDE_WAVES + wave;
    const int64_t row = tile * 32 + r;
    const bool valid = row < n;
    const float* xr = A.X + (valid ? row : (n - 1)) * dp + 8 * h;
    float a1[4], a2[4], a3[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a1[c] = a2[c] = a3[c] = FLT_MAX;
    float xx = 0.0f;
    // this row's slice of the next piece's features (lane (r, h): 8 per K-step)
    float4 xv[NSW][2];
    auto load_x = [&](int fc) {
      const int ns = min(WIDE_FW, dp - fc * WIDE_FW) / 16;
#pragma unroll
      for (int t = 0; t < NSW; ++t) {
        if (t >= ns) continue;
        xv[t][0] = *reinterpret_cast<const float4*>(xr + fc * WIDE_FW + 16 * t);
        xv[t][1] = *reinterpret_cast<const float4*>(xr + fc * WIDE_FW + 16 * t + 4);
      }
    };
    load_x(0);
    f32x16 acc[NBW];
    for (int pc = 0; pc < npc; ++pc) {
      const int ch = pc / nfc, fc = pc - ch * nfc;
      const int nb = min(WIDE_KC, kp - ch * WIDE_KC) / 32;  // even: kp is a multiple of 64
      const int ns = min(WIDE_FW, dp - fc * WIDE_FW) / 16;
      // this piece's DMA (and the row slice) landed; the other buffer is free
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const char* laneHi = smem + (size_t)cbuf * WIDE_BUF + lane * 16;
      const char* laneLo = laneHi + HIMG;
      const float* laneCn = reinterpret_cast<const float*>(smem + (size_t)cbuf * WIDE_BUF + 2 * HIMG) + 4 * h;
      if (pc + 1 < npc)
        stage_async(pc + 1, cbuf ^ 1);
      else if (wt + gridDim.x < nwt)
        stage_async(0, cbuf ^ 1);  // the next tile group starts over at piece 0
      cbuf ^= 1;
      // B operand: lane (r, h) holds features [16t + 8h, 16t + 8h + 8) of the piece
      f16x8 bh[NSW], bl[NSW];
#pragma unroll
      for (int t = 0; t < NSW; ++t) {
        const float e8[8] = {xv[t][0].x, xv[t][0].y, xv[t][0].z, xv[t][0].w,
                             xv[t][1].x, xv[t][1].y, xv[t][1].z, xv[t][1].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xs = (t < ns) ? e8[e] * s : 0.0f;
          const _Float16 hi = (_Float16)xs;
          bh[t][e] = hi;
          bl[t][e] = (_Float16)(xs - (float)hi);
          if (ch == 0) xx = fmaf(xs, xs, xx);
        }
      }
      if (pc + 1 < npc) load_x(fc + 1 < nfc ? fc + 1 : 0);  // one piece ahead
      if (fc == 0) {
#pragma unroll
        for (int blk = 0; blk < NBW; ++blk)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const float4 cv = *reinterpret_cast<const float4*>(laneCn + blk * 32 + 8 * g4);
            acc[blk][4 * g4 + 0] = cv.x;
            acc[blk][4 * g4 + 1] = cv.y;
            acc[blk][4 * g4 + 2] = cv.z;
            acc[blk][4 * g4 + 3] = cv.w;
          }
      }
#pragma unroll
      for (int t = 0; t < NSW; ++t) {
        if (t >= ns) continue;
#pragma unroll
        for (int blk = 0; blk < NBW; ++blk) {
          if (blk >= nb) continue;
          const size_t off = (size_t)(blk * NSW + t) * 1024;
          const f16x8 fh = *reinterpret_cast<const f16x8*>(laneHi + off);
          const f16x8 fl = *reinterpret_cast<const f16x8*>(laneLo + off);
          acc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh, bl[t], acc[blk], 0, 0, 0);
          acc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fl, bh[t], acc[blk], 0, 0, 0);
          acc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh, bh[t], acc[blk], 0, 0, 0);
        }
      }
      if (fc + 1 < nfc) continue;
      // register reg of block blk holds centroid j = 32 (NBW ch + blk) + 4h +
      // (reg & 3) + 8 (reg >> 2); chain reg & 3 keeps j >> 2 in the key
#pragma unroll
      for (int blk = 0; blk < NBW; ++blk) {
        if (blk >= nb) continue;
        const uint32_t jq = (uint32_t)((ch * WIDE_KC) >> 2) + 8u * (uint32_t)blk + (uint32_t)h;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const float key = __uint_as_float((__float_as_uint(acc[blk][reg]) & ~maskq) | (jq | (uint32_t)(2 * (reg >> 2))));
          top3_insert(a1[reg & 3], a2[reg & 3], a3[reg & 3], key);
        }
      }
    }
    xx += __shfl_xor(xx, 32);
    if (tile >= ntiles) continue;

    // exact merge of the 4 chains and the two lane halves (as k_assign_mfma)
    float k1 = FLT_MAX, k2 = FLT_MAX, k3 = FLT_MAX;
    uint32_t p1 = 0, p2 = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      top3p_insert(k1, k2, k3, p1, p2, a1[c], ((__float_as_uint(a1[c]) & maskq) << 2) | (uint32_t)c);
      top3p_insert(k1, k2, k3, p1, p2, a2[c], ((__float_as_uint(a2[c]) & maskq) << 2) | (uint32_t)c);
      top3p_insert(k1, k2, k3, p1, p2, a3[c], 0u);
    }
    {
      const float q1 = __shfl_xor(k1, 32), q2 = __shfl_xor(k2, 32), q3 = __shfl_xor(k3, 32);
      const uint32_t r1 = __shfl_xor(p1, 32), r2 = __shfl_xor(p2, 32);
      top3p_insert(k1, k2, k3, p1, p2, q1, r1);
      top3p_insert(k1, k2, k3, p1, p2, q2, r2);
      top3p_insert(k1, k2, k3, p1, p2, q3, 0u);
    }
    const float xn = sqrtf(xx) * 1.0001f;
    const float B0 = screen_b0(xn, cm, pm, dp);
    const float thr3 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k3));
    const float thr2 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k2));
    uint32_t kind = 0;
    if (!(k3 - k1 > thr3))
      kind = 2;
    else if (!(k2 - k1 > thr2))
      kind = 1;
    if (__ballot(kind != 0u) != 0ull && kind != 0u) {
      const KeyBounds kb = key_bounds(xn, *A.xabs * s, dp, rho);
      const float u1 = kb.upper(k1);
      if (u1 < kb.lower(k2))
        kind = 0u;
      else if (kind == 2u && kb.lower(k3) > u1)
        kind = 1u;
    }
    const int lab = (p1 < (uint32_t)A.k) ? (int)p1 : 0;
    if (h == 0 && valid) A.labels[row] = lab;
    const bool enq = (h == 0) && valid && (kind != 0);
    const uint64_t m = __ballot(enq);
    if (m) {
      const uint64_t m1 = __ballot(enq && kind == 1);
      const uint64_t m2 = m & ~m1;
      const uint64_t below = (1ull << lane) - 1ull;
      if (enq) {
        QEntry q;
        q.row = (uint32_t)row;
        q.i1 = p1;
        q.i2 = p2;
        q.kind = kind;
        const uint32_t pos = (kind == 1 || kind == 4) ? qn + (uint32_t)__popcll(m1 & below)
                                                      : A.seg - 1u - (qf + (uint32_t)__popcll(m2 & below));
        wq[pos] = q;
      }
      qn += (uint32_t)__popcll(m1);
      qf += (uint32_t)__popcll(m2);
    }
  }
  if (lane == 0) {
    A.qcount[2 * gw] = qn;
    A.qcount[2 * gw + 1] = qf;
  }
}

static int mfma_waves_env() {
  static const int e = diag_env("KM_MFMA_WAVES", KM_NARROW_WAVES);  // experiment knob: 8, 12 or 16
  static const int v = (e == 8 || e == 16) ? e : 12;
  return v;
}

static int mfma_kc(const Geometry& g, int* waves) {
  const size_t per = (size_t)g.dp * 4 + 4;
  static const int wide_waves = diag_env("KM_MFMA_WAVES_X", KM_WIDE_WAVES);  // experiment knob for 64 < dp < 192
  *waves = (g.dp >= 192) ? 4 : (g.dp <= 64 ? mfma_waves_env() : (wide_waves == 4 || wide_waves == 12 ? wide_waves : 8));
  if ((size_t)g.kp * per <= MFMA_LDS_LARGE) return g.kp;
  return (int)((MFMA_LDS_LARGE / 2 / per) / 64 * 64);  // two chunk buffers
}

// at most 2 workgroups x 8 waves per CU, each wave's segment rounded up to
// whole tiles: n + 32 * (waves) * 2 entries bound every layout
size_t queue_capacity(int64_t n, int n_cu) { return (size_t)n + (size_t)32 * 16 * n_cu * 2 + 1024; }
size_t qcount_words(int n_cu) { return (size_t)2 * 16 * n_cu + 16; }

bool mfma_path_ok(const Geometry& g) {
  if (g.dp > 256)  // k_assign_wide
    return g.dp % 16 == 0 && g.dp <= WIDE_MAX_DP && g.kp >= 64 && g.kp % 64 == 0 && g.kp <= (1 << 20);
  switch (g.dp) {
    case 16: case 32: case 48: case 64: case 96: case 128: case 192: case 256:
      return g.kp >= 64 && g.kp % 64 == 0 && g.kp <= (1 << 20);
    default:
      return false;
  }
}

hipError_t launch_prep_split(const float* C32, const Geometry& g, const float* cn2, const float* xabs,
                             const float* cabs, _Float16* Chi, _Float16* Clo, float* cn2s, const int* gate, hipStream_t s) {
  hipLaunchKernelGGL(k_prep_split, dim3(g.kp), dim3(64), 0, s, C32, g.kp, g.dp, cn2, xabs, cabs, Chi, Clo, cn2s,
                     g.k, gate);
  return hipGetLastError();
}

static int mfma_top2(int ns) {
  static const int e = diag_env("KM_TOP2", -1);  // -1: by d (key-update-bound shapes), 0/1: force
  return e >= 0 ? e : (ns <= 2 ? 1 : 0);
}

// the 16x16x32 screen (k_assign_mfma16) where dp is a multiple of 32;
// KM_MFMA16=0 builds the 32x32x16 one everywhere (A/B arm, make alt)
#ifndef KM_MFMA16
#define KM_MFMA16 1
#endif
template <int NS>
static bool launch_mfma16_ns(int waves, int blocks, size_t lds, hipStream_t s, const MfmaArgs& a) {
  static const int on = diag_env("KM_MFMA16", KM_MFMA16);
  if constexpr (NS % 2 != 0 || NS > 8) {
    return false;
  } else {
    if (!on) return false;
    const bool t2 = mfma_top2(NS);
    if (a.one) {
      // one fp16 MFMA per product: the 12- / 8-wave instances
      if (waves == 12)
        hipLaunchKernelGGL((k_assign_mfma16<NS, 12, false, true>), dim3(blocks), dim3(768), lds, s, a);
      else if (waves == 16 && NS <= 4)
        hipLaunchKernelGGL((k_assign_mfma16<NS, 16, false, true>), dim3(blocks), dim3(1024), lds, s, a);
      else
        hipLaunchKernelGGL((k_assign_mfma16<NS, 8, false, true>), dim3(blocks), dim3(512), lds, s, a);
      return true;
    }
    if (waves == 16 && NS <= 4) {
      if (t2)
        hipLaunchKernelGGL((k_assign_mfma16<NS, 16, true>), dim3(blocks), dim3(1024), lds, s, a);
      else
        hipLaunchKernelGGL((k_assign_mfma16<NS, 16>), dim3(blocks), dim3(1024), lds, s, a);
    } else if (waves == 12) {
      if (t2)
        hipLaunchKernelGGL((k_assign_mfma16<NS, 12, true>), dim3(blocks), dim3(768), lds, s, a);
      else
        hipLaunchKernelGGL((k_assign_mfma16<NS, 12>), dim3(blocks), dim3(768), lds, s, a);
    } else if (waves == 4) {
      if (t2)
        hipLaunchKernelGGL((k_assign_mfma16<NS, 4, true>), dim3(blocks), dim3(256), lds, s, a);
      else
        hipLaunchKernelGGL((k_assign_mfma16<NS, 4>), dim3(blocks), dim3(256), lds, s, a);
    } else {
      if (t2)
        hipLaunchKernelGGL((k_assign_mfma16<NS, 8, true>), dim3(blocks), dim3(512), lds, s, a);
      else
        hipLaunchKernelGGL((k_assign_mfma16<NS, 8>), dim3(blocks), dim3(512), lds, s, a);
    }
    return true;
  }
}

template <int NS>
static void launch_mfma_ns(int waves, int blocks, size_t lds, hipStream_t s, const MfmaArgs& a) {
  if (launch_mfma16_ns<NS>(waves, blocks, lds, s, a)) return;
  if constexpr (NS <= 4) {
    if (mfma_top2(NS)) {
      if (waves == 4)
        hipLaunchKernelGGL((k_assign_mfma<NS, 4, true>), dim3(blocks), dim3(256), lds, s, a);
      else if (waves == 16)
        hipLaunchKernelGGL((k_assign_mfma<NS, 16, true>), dim3(blocks), dim3(1024), lds, s, a);
      else if (waves == 12)
        hipLaunchKernelGGL((k_assign_mfma<NS, 12, true>), dim3(blocks), dim3(768), lds, s, a);
      else
        hipLaunchKernelGGL((k_assign_mfma<NS, 8, true>), dim3(blocks), dim3(512), lds, s, a);
      return;
    }
  }
  if constexpr (NS >= 12) {
    hipLaunchKernelGGL((k_assign_mfma<NS, 4>), dim3(blocks), dim3(256), lds, s, a);
  } else {
    if (waves == 4)
      hipLaunchKernelGGL((k_assign_mfma<NS, 4>), dim3(blocks), dim3(256), lds, s, a);
    else if (waves == 16) {
      if constexpr (NS <= 4)
        hipLaunchKernelGGL((k_assign_mfma<NS, 16>), dim3(blocks), dim3(1024), lds, s, a);
      else  // no 16-wave instance past dp 64 (spills): the 8-wave one, never a silent no-launch
        hipLaunchKernelGGL((k_assign_mfma<NS, 8>), dim3(blocks), dim3(512), lds, s, a);
    } else if (waves == 12)
      hipLaunchKernelGGL((k_assign_mfma<NS, 12>), dim3(blocks), dim3(768), lds, s, a);
    else
      hipLaunchKernelGGL((k_assign_mfma<NS, 8>), dim3(blocks), dim3(512), lds, s, a);
  }
}

hipError_t launch_assign_mfma(const float* X, const Geometry& g, const _Float16* Chi, const _Float16* Clo,
                              const float* cn2s, const float* cmax, const float* xabs, const float* cabs,
                              int32_t* labels, QEntry* queue, uint32_t* qcount, int n_cu, QLayout* ql,
                              const int* gate, hipStream_t s, uint32_t* cand, uint32_t* cand_ctr,
                              uint32_t cand_cap, int one, const float* C32, uint2* chg, uint32_t* chg_cnt) {
  ql->seg = 0;
  ql->nwaves = 0;
  if (g.n == 0) return hipSuccess;
  if (g.dp > 256) {
    const int64_t nwt = ((g.n + 31) / 32 + WIDE_WAVES - 1) / WIDE_WAVES;
    const int nb = (int)(nwt < n_cu ? nwt : n_cu);  // one workgroup per CU (2 x 65 KiB of LDS)
    const uint32_t seg = (uint32_t)(((nwt + nb - 1) / nb) * 32);
    ql->seg = seg;
    ql->nwaves = (uint32_t)(nb * WIDE_WAVES);
    MfmaArgs a{X, g.n, g.k, g.kp, WIDE_KC, seg, Chi, Clo, cn2s, cmax, xabs, cabs, labels, queue, qcount, gate,
               nullptr, nullptr, 0};
    hipLaunchKernelGGL(k_assign_wide, dim3(nb), dim3(WIDE_WAVES * 64), 2 * WIDE_BUF, s, a, g.dp);
    return hipGetLastError();
  }
  int waves = 8;
  const int KC = mfma_kc(g, &waves);
  if (KC < 64) return hipErrorInvalidValue;
  const size_t bufsz = (2 * (size_t)KC * g.dp * 2 + (size_t)KC * 4 + 15) / 16 * 16;
  const size_t lds = (KC < g.kp) ? 2 * bufsz : 2 * (size_t)KC * g.dp * 2 + (size_t)KC * 4;
  const int64_t ntiles = (g.n + 31) / 32;
  const int64_t nwt = (ntiles + waves - 1) / waves;
  int per_cu = (int)(MFMA_LDS_LARGE / lds);
  const int max_per_cu = (waves == 8 && g.dp <= 64) ? 2 : 1;
  if (per_cu > max_per_cu) per_cu = max_per_cu;
  if (per_cu < 1) per_cu = 1;
  int64_t blocks = (int64_t)n_cu * per_cu;
  if (blocks > nwt) blocks = nwt;
  const int nb = (int)blocks;
  const uint32_t seg = (uint32_t)(((nwt + nb - 1) / nb) * 32);
  ql->seg = seg;
  ql->nwaves = (uint32_t)(nb * waves);
  static const int use_cand = diag_env("KM_CAND", 1);  // candidate lists instead of full scans
  if (cand != nullptr && use_cand) {
    const hipError_t e = hipMemsetAsync(cand_ctr, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
  }
  const bool mfma16 = g.dp % 32 == 0 && g.dp <= 128 && KM_MFMA16;
  if (chg != nullptr && !mfma16) return hipErrorInvalidValue;  // delta statistics: k_assign_mfma16 only
  MfmaArgs a{X, g.n, g.k, g.kp, KC, seg, Chi, Clo, cn2s, cmax, xabs, cabs, labels, queue, qcount, gate,
             use_cand ? cand : nullptr, cand_ctr, cand_cap, (one && g.dp % 32 == 0 && g.dp <= 256) ? 1 : 0, C32,
             chg, chg_cnt};
  switch (g.dp / 16) {
    case 1: launch_mfma_ns<1>(waves, nb, lds, s, a); break;
    case 2: launch_mfma_ns<2>(waves, nb, lds, s, a); break;
    case 3: launch_mfma_ns<3>(waves, nb, lds, s, a); break;
    case 4: launch_mfma_ns<4>(waves, nb, lds, s, a); break;
    case 6: launch_mfma_ns<6>(waves, nb, lds, s, a); break;
    case 8: launch_mfma_ns<8>(waves, nb, lds, s, a); break;
    case 12: launch_mfma_ns<12>(waves, nb, lds, s, a); break;
    case 16: launch_mfma_ns<16>(waves, nb, lds, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// abs max of the data (fp16 scaling of the MFMA screen), accumulated over loads
__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ X, int64_t nf, float* __restrict__ out) {
  float m = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = fabsf(X[i]);
    m = (v > m || v != v) ? v : m;  // NaN wins (scale falls back to 1)
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float t = __shfl_xor(m, o);
    m = (t > m || t != t) ? t : m;
  }
  if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)out, __float_as_uint(m));
}

hipError_t launch_absmax(const float* X, int64_t nfloats, float* out, hipStream_t s) {
  if (nfloats <= 0) return hipSuccess;
  int64_t blocks = (nfloats + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_absmax, dim3((unsigned)blocks), dim3(256), 0, s, X, nfloats, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused assign + partial statistics (c3 class: kp*dp <= 16384).
//
// One workgroup of 4 waves per CU (1 per SIMD).  The fp16 hi and lo images
// of -2*c*s live in AGPRs (A fragments, 2*NB*NS*4 registers per lane, read
// by the MFMAs directly), LDS holds ||c||^2 s^2 and this workgroup's
// float64 partial sums, transposed [f][j] so that the 32 lanes
// of one ds_add_f64 (32 points, one feature) hit banks j mod 32.  Each wave
// walks 32-point tiles: fp16x3 MFMA scores, four chains of top-2 keys
// (score | j>>2), merged to the top-3 values and the best two indices, the
// rigorous screening bound, label + ambiguous-point queue, and for every
// decided point its exact fp32 row added to the table.  Ambiguous points are
// added by the resolver kernels (with their counts).
// The table is flushed with one float64 atomic per non-zero entry.
// ---------------------------------------------------------------------------

// min / max as v_med3 (no NaN-canonicalising v_max in front, unlike fminf)
__device__ __forceinline__ float kmin(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, -FLT_MAX); }
__device__ __forceinline__ float kmax(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, FLT_MAX); }

// Merge two sorted key triples (K1<=K2<=K3 with indices P1,P2 of the first
// two; likewise Q, R): the smallest three values and the indices of the
// smallest two.  Ties keep the K side (deterministic in both lane halves).
__device__ __forceinline__ void merge3(float& K1, float& K2, float& K3, uint32_t& P1, uint32_t& P2, float Q1,
                                       float Q2, float Q3, uint32_t R1, uint32_t R2) {
  const bool tk = K1 <= Q1;
  const float sa = tk ? K2 : K1;  // candidates for the second
  const float sb = tk ? Q1 : Q2;
  const uint32_t ia = tk ? P2 : P1;
  const uint32_t ib = tk ? R1 : R2;
  const float n3 = kmin(kmin(K3, Q3), kmin(kmax(K1, Q2), kmax(K2, Q1)));
  const float n1 = tk ? K1 : Q1;
  const uint32_t q1 = tk ? P1 : R1;
  const bool ta = sa <= sb;
  K2 = ta ? sa : sb;
  P2 = ta ? ia : ib;
  K1 = n1;
  P1 = q1;
  K3 = n3;
}

struct FusedArgs {
  const float* X;
  const float* xnorm;  // per-row upper bound of ||x|| (unscaled)
  int64_t n;
  int k, d;
  uint32_t seg;
  const uint4* ChiF;   // fragment-linear hi image [NB][NS][64] x 16 B
  const uint4* CloF;   // fragment-linear lo image
  const float* cn2s;   // ||c||^2 s^2 [kp], pads 1e30
  const float* bnd;    // B0 = bnd[0] * ||x|| + bnd[1]
  const float* xabs;
  const float* cabs;
  int32_t* labels;
  QEntry* queue;
  uint32_t* qcount;
  double* stats;       // [k][d+1] (sums, counts)
  const int* gate;     // nonzero: a stopped batch, the launch is a no-op
  const double* C64P;  // SSE variant: float64 centroids padded [kp][dp] (L2-resident)
  double* sse;         // SSE variant: the SSE slot stats[k (d+1)]
};

constexpr int ceil_log2_c(int v) { return v <= 1 ? 0 : 1 + ceil_log2_c((v + 1) / 2); }


// SSE (compute_sse, kmeans_spark.py:224-237): every decided row's float64
// residual to its pre-update centroid (C64P, gathered from L2 by label) is
// summed in the same pass; queued rows get theirs from the resolvers
template <int NS, int NB, bool STATS, bool REF = true, bool SSE = false>
__global__ __launch_bounds__(256, 1) void k_fused(FusedArgs A) {
  if (*A.gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  constexpr int DP = 16 * NS;
  constexpr int KP = 32 * NB;
  constexpr int WAVES = 4;
  constexpr int B = ceil_log2_c(KP);
  static_assert(B >= 3 && B - 2 <= 12, "index bits");
  static_assert(NB >= 2, "pipelined blocks");
  constexpr uint32_t maskq = (1u << (B - 2)) - 1u;
  constexpr int TS = KP;  // sum table row stride (KP + 2, which moves the lane halves to opposite bank halves: no gain)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sCn = reinterpret_cast<float*>(smem);                  // ||c||^2 s^2 [KP]
  double* tab = reinterpret_cast<double*>(smem + KP * 4);        // [DP + 1][TS]

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  for (int i = threadIdx.x; i < KP; i += WAVES * 64) sCn[i] = A.cn2s[i];
  if constexpr (STATS)
    for (int i = threadIdx.x; i < (DP + 1) * TS; i += WAVES * 64) tab[i] = 0.0;
  f16x8 Ahi[NB][NS], Alo[NB][NS];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      Ahi[b][t] = __builtin_bit_cast(f16x8, A.ChiF[(b * NS + t) * 64 + lane]);
      Alo[b][t] = __builtin_bit_cast(f16x8, A.CloF[(b * NS + t) * 64 + lane]);
    }
  // consume the image loads here: otherwise the loop's AGPR touches inherit
  // them as outstanding and the waitcnt pass drains vmcnt to 0 in every loop
  // iteration -- including the next tile's prefetch (one exposed HBM round
  // trip per two tiles)
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int t = 0; t < NS; ++t) asm volatile("" : "+a"(Ahi[b][t]), "+a"(Alo[b][t]));
  __syncthreads();

  const float s = mfma_scale(*A.xabs, *A.cabs);
  const float alpha = A.bnd[0], beta = A.bnd[1];
  const float rho = __builtin_ldexpf(1.0f, B - 2 - 23) * 1.01f;
  const int64_t n = A.n;
  const int64_t ntiles = (n + 31) / 32;
  const uint32_t gw = blockIdx.x * WAVES + wave;
  QEntry* wq = A.queue + (size_t)gw * A.seg;
  uint32_t qn = 0, qf = 0;
  const int64_t tstride = (int64_t)gridDim.x * WAVES;
  const float4* cnl = reinterpret_cast<const float4*>(sCn + 4 * h);  // + 8 blk + 2 g4

  auto load_tile = [&](int64_t tile, float4 (&xq)[NS][2], float& xnq) {
    const int64_t row = tile * 32 + r;
    const int64_t rr = row < n ? row : (n - 1);
    const float* xr = A.X + rr * DP + 8 * h;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      xq[t][0] = *reinterpret_cast<const float4*>(xr + 16 * t);
      xq[t][1] = *reinterpret_cast<const float4*>(xr + 16 * t + 4);
    }
    xnq = A.xnorm[rr];
  };

  double ss_acc = 0.0;  // SSE variant: this lane's residual sum
  auto process_tile = [&](int64_t tile, const float4 (&xc)[NS][2], float xn) {
    const int64_t row = tile * 32 + r;
    const bool valid = row < n;
    // B operand: lane (r, h) holds features [16t + 8h, +8) of point r,
    // split xs = hi + lo (fp16, RN)
    f16x8 bh[NS], bl[NS];
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const float xv[8] = {xc[t][0].x, xc[t][0].y, xc[t][0].z, xc[t][0].w,
                           xc[t][1].x, xc[t][1].y, xc[t][1].z, xc[t][1].w};
      // hi = RN_f16(xs) (v_cvt_pk_f16_f32), lo = RN_f16(xs - hi) with one
      // v_fma_mix per element (the compiler's own choice is cvt back to f32,
      // v_pk_fma, cvt_pk: 2 VALU per element instead of 1; same bits,
      // scripts/probes/split_mix.hip)
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const float xs0 = xv[e] * s, xs1 = xv[e + 1] * s;
        const f16x2 hp = {(_Float16)xs0, (_Float16)xs1};
        const f16x2 lo = split_lo(hp, xs0, xs1);
        bh[t][e] = hp[0];
        bh[t][e + 1] = hp[1];
        bl[t][e] = lo[0];
        bl[t][e + 1] = lo[1];
      }
    }
    float a1[4], a2[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a1[c] = a2[c] = FLT_MAX;
    // the images stay in AGPRs (MFMA A operands read them there); scores
    // land in VGPRs (built with -amdgpu-mfma-vgpr-form)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int t = 0; t < NS; ++t) asm volatile("" : "+a"(Ahi[b][t]), "+a"(Alo[b][t]));
    auto cn_init = [&](int blk) {
      f32x16 acc;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 cv = cnl[8 * blk + 2 * g4];
        acc[4 * g4 + 0] = cv.x;
        acc[4 * g4 + 1] = cv.y;
        acc[4 * g4 + 2] = cv.z;
        acc[4 * g4 + 3] = cv.w;
      }
      return acc;
    };
    auto mfma_block = [&](f32x16 acc, int blk) {
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ahi[blk][t], bl[t], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(Alo[blk][t], bh[t], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ahi[blk][t], bh[t], acc, 0, 0, 0);
      }
      return acc;
    };
    // register reg holds centroid j = 32 blk + 4h + (reg & 3) + 8 (reg >> 2);
    // chain reg & 3 keeps the top two keys (score | j >> 2); registers reg and
    // reg + 4 (same chain) are folded in together
    auto keys_block = [&](const f32x16& acc, int blk) {
      const uint32_t jq = (uint32_t)(8 * blk + h);
      // two keys of one chain per step: new best = min3(best, ka, kb), new
      // second = min(second, med3(best, ka, kb)) -- the same top two as one
      // key at a time, 5 VALU per 2 scores instead of 6 (c3: -2% kernel time)
#pragma unroll
      for (int q = 0; q < 16; q += 8)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int ra = q + c, rb = q + c + 4;
          const float ka = __uint_as_float((__float_as_uint(acc[ra]) & ~maskq) | (jq | (uint32_t)(2 * (ra >> 2))));
          const float kb = __uint_as_float((__float_as_uint(acc[rb]) & ~maskq) | (jq | (uint32_t)(2 * (rb >> 2))));
          const float t = __builtin_amdgcn_fmed3f(a1[c], ka, kb);
          a1[c] = __builtin_fminf(__builtin_fminf(a1[c], ka), kb);
          a2[c] = __builtin_fminf(a2[c], t);
        }
    };
    // software pipeline: block blk's MFMAs overlap block blk-1's key
    // updates (started two MFMAs in, once blk-1's scores have landed); the
    // accumulator init of block blk+1 is read from LDS meanwhile
    f32x16 accs[2];
    f32x16 cinit = cn_init(1);
    accs[0] = mfma_block(cn_init(0), 0);
#pragma unroll
    for (int blk = 1; blk < NB; ++blk) {
      const f32x16 cin = cinit;
      if (blk + 1 < NB) cinit = cn_init(blk + 1);
      accs[blk & 1] = mfma_block(cin, blk);
      keys_block(accs[(blk - 1) & 1], blk - 1);
      // MFMA, next block's init reads, MFMA, then (VALU x m, MFMA) pairs
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
#pragma unroll
      for (int i = 0; i < 3 * NS - 2; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x2, 64 / (3 * NS - 2) + 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    keys_block(accs[(NB - 1) & 1], NB - 1);

    // top-3 values and best two full indices: chains merged pairwise, then
    // the two lane halves.  A chain keeps its best two; keys it dropped are
    // only known to be >= its second, which therefore stands in for its
    // third (k3 bounds every candidate other than p1, p2 unless p1 and p2
    // share a chain: checked below).
    auto pidx = [&](float key, int c) { return ((__float_as_uint(key) & maskq) << 2) | (uint32_t)c; };
    float k1 = a1[0], k2 = a2[0], k3 = a2[0];
    uint32_t p1 = pidx(a1[0], 0), p2 = pidx(a2[0], 0);
    {
      float m1 = a1[2], m2 = a2[2], m3 = a2[2];
      uint32_t q1 = pidx(a1[2], 2), q2 = pidx(a2[2], 2);
      merge3(k1, k2, k3, p1, p2, a1[1], a2[1], a2[1], pidx(a1[1], 1), pidx(a2[1], 1));
      merge3(m1, m2, m3, q1, q2, a1[3], a2[3], a2[3], pidx(a1[3], 3), pidx(a2[3], 3));
      merge3(k1, k2, k3, p1, p2, m1, m2, m3, q1, q2);
    }
    {
      uint32_t K1, Q1, K2, Q2, K3, Q3, P1, R1, P2, R2;
      perm_halves(__float_as_uint(k1), K1, Q1);
      perm_halves(__float_as_uint(k2), K2, Q2);
      perm_halves(__float_as_uint(k3), K3, Q3);
      perm_halves(p1, P1, R1);
      perm_halves(p2, P2, R2);
      k1 = __uint_as_float(K1);
      k2 = __uint_as_float(K2);
      k3 = __uint_as_float(K3);
      p1 = P1;
      p2 = P2;
      merge3(k1, k2, k3, p1, p2, __uint_as_float(Q1), __uint_as_float(Q2), __uint_as_float(Q3), R1, R2);
    }
    // p1, p2 in one chain (same j & 3 and lane half): that chain's dropped
    // keys are only known to be >= k2, so no re-rank certificate (full scan)
    const bool same_chain = ((p1 ^ p2) & 7u) == 0u;
    const float B0 = fmaf(alpha, xn, beta);
    const float thr2 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k2));
    const float thr3 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k3));
    uint32_t kind = 0;
    if (!(k2 - k1 > thr2)) kind = (same_chain || !(k3 - k1 > thr3)) ? 2u : 1u;
    // per-key bounds where the global test failed (wave-uniform branch)
    // (REF = false: left out when the global test already settles nearly all
    // rows, the runtime's choice from the last iteration's queue fraction)
    float u1 = 0.0f;
    KeyBounds kb;
    const bool refine = REF && __ballot(kind != 0u) != 0ull;
    if (refine) {
      kb = key_bounds(xn * s, *A.xabs * s, DP, rho);
      if (kind != 0u) {
        u1 = kb.upper(k1);
        if (u1 < kb.lower(k2))
          kind = 0u;  // every other centroid (key >= k2) is provably worse
        else if (kind == 2u && !same_chain && kb.lower(k3) > u1)
          kind = 1u;  // the rest (key >= k3) is worse than i1: the answer is i1 or i2
      }
    }
    // p1, p2 in one chain but every other chain's best separated from k1: the
    // answer lies in that chain (j & 7 == p1 & 7), scanned exactly (kind 3,
    // k/8 centroids) instead of all k.  Rare: behind a wave-uniform branch.
    if (__ballot(kind == 2u && same_chain) != 0ull) {
      const uint32_t cs = p1 & 7u;
      float o = FLT_MAX;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t v0, v1;  // chain c of lane half 0 (id c) and of half 1 (id 4 + c)
        perm_halves(__float_as_uint(a1[c]), v0, v1);
        if ((uint32_t)c != cs) o = kmin(o, __uint_as_float(v0));
        if ((uint32_t)(4 + c) != cs) o = kmin(o, __uint_as_float(v1));
      }
      const float thr3x = 2.0f * B0 + rho * (fabsf(k1) + fabsf(o));
      if (kind == 2u && same_chain && (o - k1 > thr3x || (REF && kb.lower(o) > u1))) kind = 3u;
    }
    const int lab = (p1 < (uint32_t)A.k) ? (int)p1 : 0;
    if (h == 0 && valid) A.labels[row] = lab;
    const bool enq = (h == 0) && valid && (kind != 0);
    const uint64_t m = __ballot(enq);
    if (m) {
      // re-rank entries from the front, full and chain scans from the back
      const uint64_t m1 = __ballot(enq && kind == 1);
      const uint64_t m2 = m & ~m1;
      const uint64_t below = (1ull << lane) - 1ull;
      if (enq) {
        QEntry q;
        q.row = (uint32_t)row;
        q.i1 = p1;
        q.i2 = p2;
        q.kind = kind;
        const uint32_t pos = (kind == 1) ? qn + (uint32_t)__popcll(m1 & below)
                                         : A.seg - 1u - (qf + (uint32_t)__popcll(m2 & below));
        wq[pos] = q;
      }
      qn += (uint32_t)__popcll(m1);
      qf += (uint32_t)__popcll(m2);
    }
    if constexpr (STATS) {
      if (valid && kind == 0) {
        double* tp = tab + (size_t)(8 * h) * TS + lab;
#pragma unroll
        for (int t = 0; t < NS; ++t) {
          const float4 v0 = xc[t][0], v1 = xc[t][1];
          const float xe[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) atomicAdd(tp + (size_t)(16 * t + e) * TS, (double)xe[e]);
        }
        if (h == 0) atomicAdd(tab + (size_t)DP * TS + lab, 1.0);  // count row
        if constexpr (SSE) {
          // this lane's 8 NS features of the row against the float64
          // centroid (padded features are 0 - 0)
          const double* cr = A.C64P + (size_t)lab * DP + 8 * h;
#pragma unroll
          for (int t = 0; t < NS; ++t) {
            const double4 ca = *reinterpret_cast<const double4*>(cr + 16 * t);
            const double4 cb = *reinterpret_cast<const double4*>(cr + 16 * t + 4);
            const float4 v0 = xc[t][0], v1 = xc[t][1];
            const double r0 = (double)v0.x - ca.x, r1 = (double)v0.y - ca.y;
            const double r2 = (double)v0.z - ca.z, r3 = (double)v0.w - ca.w;
            const double r4 = (double)v1.x - cb.x, r5 = (double)v1.y - cb.y;
            const double r6 = (double)v1.z - cb.z, r7 = (double)v1.w - cb.w;
            ss_acc = fma(r0, r0, ss_acc);
            ss_acc = fma(r1, r1, ss_acc);
            ss_acc = fma(r2, r2, ss_acc);
            ss_acc = fma(r3, r3, ss_acc);
            ss_acc = fma(r4, r4, ss_acc);
            ss_acc = fma(r5, r5, ss_acc);
            ss_acc = fma(r6, r6, ss_acc);
            ss_acc = fma(r7, r7, ss_acc);
          }
        }
      }
    }
  };

  // tiles of this wave, two register buffers: the next tile's rows are in
  // flight while this one is processed
  // (loads are unconditional -- load_tile clamps past-the-end rows to row
  // n - 1 -- so every path reaching a wait has the same loads in flight and
  // the waitcnt pass can wait for the current tile only, not vmcnt(0))
  float4 xb0[NS][2], xb1[NS][2];
  float xn0 = 0.0f, xn1 = 0.0f;
  load_tile(gw, xb0, xn0);
  for (int64_t tile = gw; tile < ntiles; tile += 2 * tstride) {
    const int64_t t1 = tile + tstride;
    load_tile(t1, xb1, xn1);
    process_tile(tile, xb0, xn0);
    if (t1 >= ntiles) break;
    load_tile(t1 + tstride, xb0, xn0);
    process_tile(t1, xb1, xn1);
  }
  if (lane == 0) {
    A.qcount[2 * gw] = qn;
    A.qcount[2 * gw + 1] = qf;
  }
  if constexpr (SSE) {
    ss_acc = wave_sum(ss_acc);
    if (lane == 0 && ss_acc != 0.0) atomicAdd(A.sse, ss_acc);
  }
  if constexpr (STATS) {
    __syncthreads();
    const int d1 = A.d + 1;
    // row-major walk of the global [k][d+1] buffer: a wave's atomics cover
    // contiguous bytes (scattered float64 atomics run ~17x slower)
    for (int i = threadIdx.x; i < (DP + 1) * KP; i += WAVES * 64) {
      const int j = i / (DP + 1);
      const int f = i - j * (DP + 1);
      const double v = tab[(size_t)f * TS + j];
      if (v != 0.0 && (f < A.d || f == DP) && j < A.k) atomicAdd(A.stats + (size_t)j * d1 + (f == DP ? A.d : f), v);
    }
  }
}

// ---------------------------------------------------------------------------
// k_fused16: k_fused on v_mfma_f32_16x16x32_f16 ("The
// 16x16x32 shape").  Same output tile per wave -- 32 rows x KP centroids per tile,
// fp16x3 scores, images in AGPRs, rows double-buffered in registers -- with
// 16x16 accumulators: a block of 32 centroids is two 16-centroid halves (cb)
// times two 16-row groups (pg), 12 NS2 MFMAs of 16 cycles (k_fused: 3 NS of
// 32).  Lane l, q = l >> 4:
//   A operand: centroid 32 b + 16 cb + (l & 15), features 32 s + 8 q .. + 8
//              (image piece (2 b + cb) NS2 + s, k_frag_images16);
//   B operand: row 16 pg + (l & 15), the same features;
//   register i of accumulator (cb, pg): centroid j = 32 b + 16 cb + 4 q + i.
// Chains are (j & 3, q): 16 per row (k_fused: 8); keys carry j >> 2.  After
// the blocks the two row groups are reduce-scattered over the lane halves
// (lanes 0-31 keep group 0, 32-63 group 1) and merged over quarter pairs, so
// lanes l and l ^ 16 hold the top-3 and best two of row (l & 15) + 16 (l >> 5).
// The bound is screen_b0's with the 16x16x32 accumulation model (chain_err).
// ---------------------------------------------------------------------------
template <int NS2, int NB, bool STATS, bool REF = true, bool SSE = false>
__global__ __launch_bounds__(256, 1) void k_fused16(FusedArgs A) {
  if (*A.gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  constexpr int DP = 32 * NS2;
  constexpr int KP = 32 * NB;
  constexpr int WAVES = 4;
  constexpr int B = ceil_log2_c(KP);
  static_assert(B >= 3 && B - 2 <= 12, "index bits");
  static_assert(NB >= 2, "pipelined blocks");
  constexpr uint32_t maskq = (1u << (B - 2)) - 1u;
  constexpr int TS = KP;
  constexpr int NMF = 12 * NS2;  // MFMAs per block
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sCn = reinterpret_cast<float*>(smem);            // ||c||^2 s^2 [KP]
  double* tab = reinterpret_cast<double*>(smem + KP * 4);  // [DP + 1][TS]

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c16 = lane & 15;
  const int q = lane >> 4;
  const int prow = c16 + 16 * (lane >> 5);  // the tile row this lane owns after the merge
  for (int i = threadIdx.x; i < KP; i += WAVES * 64) sCn[i] = A.cn2s[i];
  if constexpr (STATS)
    for (int i = threadIdx.x; i < (DP + 1) * TS; i += WAVES * 64) tab[i] = 0.0;
  f16x8 Ahi[NB][2][NS2], Alo[NB][2][NS2];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int t = 0; t < NS2; ++t) {
        Ahi[b][cb][t] = __builtin_bit_cast(f16x8, A.ChiF[((2 * b + cb) * NS2 + t) * 64 + lane]);
        Alo[b][cb][t] = __builtin_bit_cast(f16x8, A.CloF[((2 * b + cb) * NS2 + t) * 64 + lane]);
      }
  // consume the image loads before the loop (see k_fused)
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int t = 0; t < NS2; ++t) asm volatile("" : "+a"(Ahi[b][cb][t]), "+a"(Alo[b][cb][t]));
  __syncthreads();

  const float s = mfma_scale(*A.xabs, *A.cabs);
  const float alpha = A.bnd[0], beta = A.bnd[1];
  const float rho = __builtin_ldexpf(1.0f, B - 2 - 23) * 1.01f;
  const int64_t n = A.n;
  const int64_t ntiles = (n + 31) / 32;
  const uint32_t gw = blockIdx.x * WAVES + wave;
  QEntry* wq = A.queue + (size_t)gw * A.seg;
  uint32_t qn = 0, qf = 0;
  const int64_t tstride = (int64_t)gridDim.x * WAVES;
  const float4* cnl = reinterpret_cast<const float4*>(sCn + 4 * q);  // + 8 blk + 4 cb

  auto load_tile = [&](int64_t tile, float4 (&xq)[2][NS2][2], float& xnq) {
#pragma unroll
    for (int pg = 0; pg < 2; ++pg) {
      const int64_t row = tile * 32 + 16 * pg + c16;
      const int64_t rr = row < n ? row : (n - 1);
      const float* xr = A.X + rr * DP + 8 * q;
#pragma unroll
      for (int t = 0; t < NS2; ++t) {
        xq[pg][t][0] = *reinterpret_cast<const float4*>(xr + 32 * t);
        xq[pg][t][1] = *reinterpret_cast<const float4*>(xr + 32 * t + 4);
      }
    }
    const int64_t orow = tile * 32 + prow;
    xnq = A.xnorm[orow < n ? orow : (n - 1)];
  };

  double ss_acc = 0.0;  // SSE variant: this lane's residual sum
  auto process_tile = [&](int64_t tile, const float4 (&xc)[2][NS2][2], float xn) {
    const int64_t row = tile * 32 + prow;
    const bool valid = row < n;
    // B operands: xs = hi + lo (fp16, RN), as in k_fused
    f16x8 bh[2][NS2], bl[2][NS2];
#pragma unroll
    for (int pg = 0; pg < 2; ++pg)
#pragma unroll
      for (int t = 0; t < NS2; ++t) {
        const float xv[8] = {xc[pg][t][0].x, xc[pg][t][0].y, xc[pg][t][0].z, xc[pg][t][0].w,
                             xc[pg][t][1].x, xc[pg][t][1].y, xc[pg][t][1].z, xc[pg][t][1].w};
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const float xs0 = xv[e] * s, xs1 = xv[e + 1] * s;
          const f16x2 hp = {(_Float16)xs0, (_Float16)xs1};
          bh[pg][t][e] = hp[0];
          bh[pg][t][e + 1] = hp[1];
          const f16x2 lo = split_lo(hp, xs0, xs1);
          bl[pg][t][e] = lo[0];
          bl[pg][t][e + 1] = lo[1];
        }
      }
    float a1[2][4], a2[2][4];
#pragma unroll
    for (int pg = 0; pg < 2; ++pg)
#pragma unroll
      for (int c = 0; c < 4; ++c) a1[pg][c] = a2[pg][c] = FLT_MAX;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int t = 0; t < NS2; ++t) asm volatile("" : "+a"(Ahi[b][cb][t]), "+a"(Alo[b][cb][t]));
    struct Acc {
      f32x4 v[2][2];  // [cb][pg]
    };
    auto cn_init = [&](int blk, int cb) {
      const float4 cv = cnl[8 * blk + 4 * cb];
      f32x4 r = {cv.x, cv.y, cv.z, cv.w};
      return r;
    };
    auto mfma_block = [&](const f32x4 (&ini)[2], int blk) {
      Acc a;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int pg = 0; pg < 2; ++pg) a.v[cb][pg] = ini[cb];
#pragma unroll
      for (int t = 0; t < NS2; ++t) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int pg = 0; pg < 2; ++pg)
            a.v[cb][pg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ahi[blk][cb][t], bl[pg][t], a.v[cb][pg], 0, 0, 0);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int pg = 0; pg < 2; ++pg)
            a.v[cb][pg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Alo[blk][cb][t], bh[pg][t], a.v[cb][pg], 0, 0, 0);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int pg = 0; pg < 2; ++pg)
            a.v[cb][pg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ahi[blk][cb][t], bh[pg][t], a.v[cb][pg], 0, 0, 0);
      }
      return a;
    };
    // chain (c, q) of row group pg keeps its top two keys; the two halves cb
    // of a block are folded in together (5 VALU per 2 scores, as k_fused)
    auto keys_block = [&](const Acc& a, int blk) {
      const uint32_t j0 = (uint32_t)(8 * blk + q), j1 = j0 + 4u;  // j >> 2 of halves 0 and 1
#pragma unroll
      for (int pg = 0; pg < 2; ++pg)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float ka = __uint_as_float((__float_as_uint(a.v[0][pg][c]) & ~maskq) | j0);
          const float kb = __uint_as_float((__float_as_uint(a.v[1][pg][c]) & ~maskq) | j1);
          const float t = __builtin_amdgcn_fmed3f(a1[pg][c], ka, kb);
          a1[pg][c] = __builtin_fminf(__builtin_fminf(a1[pg][c], ka), kb);
          a2[pg][c] = __builtin_fminf(a2[pg][c], t);
        }
    };
    // software pipeline as in k_fused: block blk's MFMAs overlap block blk-1's
    // key updates; block blk+1's accumulator init is read from LDS meanwhile
    Acc accs[2];
    f32x4 nxt[2] = {cn_init(1, 0), cn_init(1, 1)};
    {
      const f32x4 ini[2] = {cn_init(0, 0), cn_init(0, 1)};
      accs[0] = mfma_block(ini, 0);
    }
#pragma unroll
    for (int blk = 1; blk < NB; ++blk) {
      const f32x4 cin[2] = {nxt[0], nxt[1]};
      if (blk + 1 < NB) {
        nxt[0] = cn_init(blk + 1, 0);
        nxt[1] = cn_init(blk + 1, 1);
      }
      accs[blk & 1] = mfma_block(cin, blk);
      keys_block(accs[(blk - 1) & 1], blk - 1);
      // MFMA, next block's init reads, MFMA, then (VALU x m, MFMA) pairs
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
#pragma unroll
      for (int i = 0; i < NMF - 2; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x2, 48 / (NMF - 2) + 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    keys_block(accs[(NB - 1) & 1], NB - 1);

    // per row group: the four chains of this lane merged (as k_fused)
    auto pidx = [&](float key, int c) { return ((__float_as_uint(key) & maskq) << 2) | (uint32_t)c; };
    float g1[2], g2[2], g3[2];
    uint32_t gp1[2], gp2[2];
#pragma unroll
    for (int pg = 0; pg < 2; ++pg) {
      float k1 = a1[pg][0], k2 = a2[pg][0], k3 = a2[pg][0];
      uint32_t p1 = pidx(a1[pg][0], 0), p2 = pidx(a2[pg][0], 0);
      float m1 = a1[pg][2], m2 = a2[pg][2], m3 = a2[pg][2];
      uint32_t q1 = pidx(a1[pg][2], 2), q2 = pidx(a2[pg][2], 2);
      merge3(k1, k2, k3, p1, p2, a1[pg][1], a2[pg][1], a2[pg][1], pidx(a1[pg][1], 1), pidx(a2[pg][1], 1));
      merge3(m1, m2, m3, q1, q2, a1[pg][3], a2[pg][3], a2[pg][3], pidx(a1[pg][3], 3), pidx(a2[pg][3], 3));
      merge3(k1, k2, k3, p1, p2, m1, m2, m3, q1, q2);
      g1[pg] = k1;
      g2[pg] = k2;
      g3[pg] = k3;
      gp1[pg] = p1;
      gp2[pg] = p2;
    }
    // reduce-scatter over the lane halves: permlane32_swap(group 0, group 1)
    // gives lanes 0-31 group 0 of lanes l and l + 32, lanes 32-63 group 1 of
    // lanes l - 32 and l (the lower lane's side first in both)
    auto swap_groups = [](uint32_t v0, uint32_t v1, uint32_t& lo, uint32_t& hi) { swap_halves(v0, v1, lo, hi); };
    float k1, k2, k3;
    uint32_t p1, p2;
    {
      uint32_t K1, Q1, K2, Q2, K3, Q3, P1, R1, P2, R2;
      swap_groups(__float_as_uint(g1[0]), __float_as_uint(g1[1]), K1, Q1);
      swap_groups(__float_as_uint(g2[0]), __float_as_uint(g2[1]), K2, Q2);
      swap_groups(__float_as_uint(g3[0]), __float_as_uint(g3[1]), K3, Q3);
      swap_groups(gp1[0], gp1[1], P1, R1);
      swap_groups(gp2[0], gp2[1], P2, R2);
      k1 = __uint_as_float(K1);
      k2 = __uint_as_float(K2);
      k3 = __uint_as_float(K3);
      p1 = P1;
      p2 = P2;
      merge3(k1, k2, k3, p1, p2, __uint_as_float(Q1), __uint_as_float(Q2), __uint_as_float(Q3), R1, R2);
    }
    {
      uint32_t K1, Q1, K2, Q2, K3, Q3, P1, R1, P2, R2;
      perm_quarters(__float_as_uint(k1), K1, Q1);
      perm_quarters(__float_as_uint(k2), K2, Q2);
      perm_quarters(__float_as_uint(k3), K3, Q3);
      perm_quarters(p1, P1, R1);
      perm_quarters(p2, P2, R2);
      k1 = __uint_as_float(K1);
      k2 = __uint_as_float(K2);
      k3 = __uint_as_float(K3);
      p1 = P1;
      p2 = P2;
      merge3(k1, k2, k3, p1, p2, __uint_as_float(Q1), __uint_as_float(Q2), __uint_as_float(Q3), R1, R2);
    }
    // p1, p2 in one chain (j & 15): no re-rank certificate (see k_fused)
    const bool same_chain = ((p1 ^ p2) & 15u) == 0u;
    const float B0 = fmaf(alpha, xn, beta);
    const float thr2 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k2));
    const float thr3 = 2.0f * B0 + rho * (fabsf(k1) + fabsf(k3));
    uint32_t kind = 0;
    if (!(k2 - k1 > thr2)) kind = (same_chain || !(k3 - k1 > thr3)) ? 2u : 1u;
    float u1 = 0.0f;
    KeyBounds kb;
    const bool refine = REF && __ballot(kind != 0u) != 0ull;
    if (refine) {
      kb = key_bounds(xn * s, *A.xabs * s, DP, rho, 1);
      if (kind != 0u) {
        u1 = kb.upper(k1);
        if (u1 < kb.lower(k2))
          kind = 0u;
        else if (kind == 2u && !same_chain && kb.lower(k3) > u1)
          kind = 1u;
      }
    }
    // p1, p2 in one chain, every other chain's best separated from k1: the
    // answer lies in chain p1 & 15, a subset of the resolver's kind-3 scan
    // (j & 7 == p1 & 7)
    if (__ballot(kind == 2u && same_chain) != 0ull) {
      const uint32_t cs = p1 & 15u;
      float o = FLT_MAX;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t h0, h1, v0, v1, v2, v3;  // chain (c, quarter 0..3) of this lane's row group
        swap_groups(__float_as_uint(a1[0][c]), __float_as_uint(a1[1][c]), h0, h1);
        perm_quarters(h0, v0, v1);
        perm_quarters(h1, v2, v3);
        if ((uint32_t)c != cs) o = kmin(o, __uint_as_float(v0));
        if ((uint32_t)(4 + c) != cs) o = kmin(o, __uint_as_float(v1));
        if ((uint32_t)(8 + c) != cs) o = kmin(o, __uint_as_float(v2));
        if ((uint32_t)(12 + c) != cs) o = kmin(o, __uint_as_float(v3));
      }
      const float thr3x = 2.0f * B0 + rho * (fabsf(k1) + fabsf(o));
      if (kind == 2u && same_chain && (o - k1 > thr3x || (REF && kb.lower(o) > u1))) kind = 3u;
    }
    const int lab = (p1 < (uint32_t)A.k) ? (int)p1 : 0;
    const bool lead = (q & 1) == 0;  // one lane of each pair (l, l ^ 16) writes
    if (lead && valid) A.labels[row] = lab;
    const bool enq = lead && valid && (kind != 0);
    const uint64_t m = __ballot(enq);
    if (m) {
      const uint64_t m1 = __ballot(enq && kind == 1);
      const uint64_t m2 = m & ~m1;
      const uint64_t below = (1ull << lane) - 1ull;
      if (enq) {
        QEntry qe;
        qe.row = (uint32_t)row;
        qe.i1 = p1;
        qe.i2 = p2;
        qe.kind = kind;
        const uint32_t pos = (kind == 1) ? qn + (uint32_t)__popcll(m1 & below)
                                         : A.seg - 1u - (qf + (uint32_t)__popcll(m2 & below));
        wq[pos] = qe;
      }
      qn += (uint32_t)__popcll(m1);
      qf += (uint32_t)__popcll(m2);
    }
    if constexpr (STATS) {
      // every lane holds features 32 t + 8 q .. + 8 of both row groups: the
      // label of each decided row from its owner lanes (l & 31 and l | 32)
      const uint32_t own = (valid && kind == 0) ? (uint32_t)lab : 0xffffffffu;
      uint32_t li[2];
      perm_halves(own, li[0], li[1]);
#pragma unroll
      for (int pg = 0; pg < 2; ++pg) {
        if (li[pg] != 0xffffffffu) {
          double* tp = tab + (size_t)(8 * q) * TS + li[pg];
#pragma unroll
          for (int t = 0; t < NS2; ++t) {
            const float4 v0 = xc[pg][t][0], v1 = xc[pg][t][1];
            const float xe[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) atomicAdd(tp + (size_t)(32 * t + e) * TS, (double)xe[e]);
          }
          if (q == 0) atomicAdd(tab + (size_t)DP * TS + li[pg], 1.0);  // count row
          if constexpr (SSE) {
            const double* cr = A.C64P + (size_t)li[pg] * DP + 8 * q;
#pragma unroll
            for (int t = 0; t < NS2; ++t) {
              const double4 ca = *reinterpret_cast<const double4*>(cr + 32 * t);
              const double4 cb = *reinterpret_cast<const double4*>(cr + 32 * t + 4);
              const float4 v0 = xc[pg][t][0], v1 = xc[pg][t][1];
              const double r0 = (double)v0.x - ca.x, r1 = (double)v0.y - ca.y;
              const double r2 = (double)v0.z - ca.z, r3 = (double)v0.w - ca.w;
              const double r4 = (double)v1.x - cb.x, r5 = (double)v1.y - cb.y;
              const double r6 = (double)v1.z - cb.z, r7 = (double)v1.w - cb.w;
              ss_acc = fma(r0, r0, ss_acc);
              ss_acc = fma(r1, r1, ss_acc);
              ss_acc = fma(r2, r2, ss_acc);
              ss_acc = fma(r3, r3, ss_acc);
              ss_acc = fma(r4, r4, ss_acc);
              ss_acc = fma(r5, r5, ss_acc);
              ss_acc = fma(r6, r6, ss_acc);
              ss_acc = fma(r7, r7, ss_acc);
            }
          }
        }
      }
    }
  };

  float4 xb0[2][NS2][2], xb1[2][NS2][2];
  float xn0 = 0.0f, xn1 = 0.0f;
  load_tile(gw, xb0, xn0);
  for (int64_t tile = gw; tile < ntiles; tile += 2 * tstride) {
    const int64_t t1 = tile + tstride;
    load_tile(t1, xb1, xn1);
    process_tile(tile, xb0, xn0);
    if (t1 >= ntiles) break;
    load_tile(t1 + tstride, xb0, xn0);
    process_tile(t1, xb1, xn1);
  }
  if (lane == 0) {
    A.qcount[2 * gw] = qn;
    A.qcount[2 * gw + 1] = qf;
  }
  if constexpr (SSE) {
    ss_acc = wave_sum(ss_acc);
    if (lane == 0 && ss_acc != 0.0) atomicAdd(A.sse, ss_acc);
  }
  if constexpr (STATS) {
    __syncthreads();
    const int d1 = A.d + 1;
    for (int i = threadIdx.x; i < (DP + 1) * KP; i += WAVES * 64) {
      const int j = i / (DP + 1);
      const int f = i - j * (DP + 1);
      const double v = tab[(size_t)f * TS + j];
      if (v != 0.0 && (f < A.d || f == DP) && j < A.k) atomicAdd(A.stats + (size_t)j * d1 + (f == DP ? A.d : f), v);
    }
  }
}

// The diagnostic build's experimental kernels -- the fast screen k_fused1 /
// k_prep_bal -- live in km_diag.inc, compiled only by `make diag` (DESIGN.md
// section 4).
#ifdef KM_DIAG
#include "km_diag.inc"
#endif

// fragment-linear copies of the hi / lo images: piece (b, t), lane l holds
// 8 halves of row 32 b + (l & 31), features 16 t + 8 (l >> 5) .. + 8
__global__ __launch_bounds__(256) void k_frag_images(const _Float16* __restrict__ Chi, const _Float16* __restrict__ Clo,
                                                     int kp, int dp, uint4* __restrict__ ChiF,
                                                     uint4* __restrict__ CloF, const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  const int ns = dp / 16;
  const int total = (kp / 32) * ns * 64;
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= total) return;
  const int l = id & 63;
  const int bt = id >> 6;
  const int b = bt / ns, t = bt - b * ns;
  const size_t src = (size_t)(b * 32 + (l & 31)) * dp + 16 * t + 8 * (l >> 5);
  ChiF[id] = *reinterpret_cast<const uint4*>(Chi + src);
  CloF[id] = *reinterpret_cast<const uint4*>(Clo + src);
}

// the same for k_fused16: piece (h, t) (h = 2 b + cb, a 16-centroid half),
// lane l holds 8 halves of row 16 h + (l & 15), features 32 t + 8 (l >> 4) .. + 8
__global__ __launch_bounds__(256) void k_frag_images16(const _Float16* __restrict__ Chi,
                                                       const _Float16* __restrict__ Clo, int kp, int dp,
                                                       uint4* __restrict__ ChiF, uint4* __restrict__ CloF,
                                                       const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  const int ns2 = dp / 32;
  const int total = (kp / 16) * ns2 * 64;
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= total) return;
  const int l = id & 63;
  const int ht = id >> 6;
  const int hb = ht / ns2, t = ht - hb * ns2;
  const size_t src = (size_t)(hb * 16 + (l & 15)) * dp + 32 * t + 8 * (l >> 4);
  ChiF[id] = *reinterpret_cast<const uint4*>(Chi + src);
  CloF[id] = *reinterpret_cast<const uint4*>(Clo + src);
}

// screening-bound constants: B0 = alpha * ||x|| + beta (see k_assign_mfma)
__global__ void k_bound_consts(const float* __restrict__ cmax, const float* __restrict__ xabs,
                               const float* __restrict__ cabs, int dp, int shape16, float* __restrict__ bnd,
                               const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  // screen_b0 is affine in xn_s = s ||x||: B0 = bnd[0] ||x|| + bnd[1]
  const float s = mfma_scale(*xabs, *cabs);
  const float cm = *cmax * s;
  const float pm = (*cabs * s) * (*xabs * s) * 1.0001f;
  bnd[0] = screen_slope(cm, dp, shape16) * s * 1.0001f;  // per unscaled ||x||
  bnd[1] = screen_icpt(cm, pm, dp, shape16) * 1.0001f;
}

// upper bound of ||x|| per row (float64 sum, rounded up): L = dp/4 lanes per
// row read float4s (coalesced), partial sums combined with xor-shuffles
template <int L>
__global__ __launch_bounds__(256) void k_row_norm(const float* __restrict__ X, int64_t n, float* __restrict__ xnorm) {
  constexpr int P = 64 / L;
  const int lane = threadIdx.x & 63;
  const int q = lane / L, m = lane % L;
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r0 = gw * P; r0 < n; r0 += nw * P) {
    const int64_t row = r0 + q;
    double sq = 0.0;
    if (q < P && row < n) {
      const float4 v = *reinterpret_cast<const float4*>(X + row * (4 * L) + 4 * m);
      sq = (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
#pragma unroll
    for (int o = 1; o < L; o <<= 1) sq += __shfl_xor(sq, o);
    if (q < P && m == 0 && row < n) xnorm[row] = (float)(sqrt(sq) * (1.0 + 1e-6)) * 1.0000001f;
  }
}

__global__ __launch_bounds__(256) void k_row_norm_any(const float* __restrict__ X, int64_t n, int dp,
                                                      float* __restrict__ xnorm) {
  // one wave per row (lanes over features): dp = 48, 96, 192
  const int lane = threadIdx.x & 63;
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t row = gw; row < n; row += nw) {
    double sq = 0.0;
    for (int f = lane; f < dp; f += 64) {
      const double v = X[row * dp + f];
      sq = fma(v, v, sq);
    }
    sq = wave_sum(sq);
    if (lane == 0) xnorm[row] = (float)(sqrt(sq) * (1.0 + 1e-6)) * 1.0000001f;
  }
}

bool fused_path_ok(const Geometry& g) {
  const int ns = g.dp / 16, nb = g.kp / 32;
  if (g.dp % 16 || g.kp % 64) return false;
  switch (ns * 100 + nb) {
    case 402: case 404: case 406: case 408:
    case 202: case 204: case 206: case 208: case 212: case 216:
    case 302: case 304: case 306: case 308:
    case 802: case 804:
      return true;
    default:
      return false;
  }
}

bool fast_path_ok(const Geometry& g) { return g.dp == 64 && g.kp == 256; }

// k_fused16 (v_mfma_f32_16x16x32_f16) for dp a multiple of 32; KM_FUSED16=0
// builds the 32x32x16 k_fused everywhere (A/B arm, make alt)
#ifndef KM_FUSED16
#define KM_FUSED16 1
#endif
bool fused16_ok(const Geometry& g) {
  static const int on = diag_env("KM_FUSED16", KM_FUSED16);
  return on && fused_path_ok(g) && g.dp % 32 == 0;
}

hipError_t launch_fused(const float* X, const float* xnorm, const Geometry& g, const _Float16* Chi,
                        const _Float16* Clo, uint4* ChiF, uint4* CloF, const float* cn2s, const float* bnd,
                        const float* xabs, const float* cabs, int32_t* labels, QEntry* queue, uint32_t* qcount,
                        double* stats, int with_stats, int mode, int n_cu, QLayout* ql, const int* gate,
                        hipStream_t s, const float* C32, const float* cmax, float* bal, const double* C64P,
                        double* sse) {
  ql->seg = 0;
  ql->nwaves = 0;
  if (g.n == 0) return hipSuccess;
  const int ns = g.dp / 16, nb = g.kp / 32;
  const int refine = (mode == KM_SCREEN_X3_REFINE) ? 1 : 0;
#ifdef KM_DIAG
  if ((mode == KM_SCREEN_FAST1 || mode == KM_SCREEN_FAST2) && fast_path_ok(g) && !(with_stats && sse)) {
    hipLaunchKernelGGL(k_prep_bal, dim3(1), dim3(512), 0, s, C32, g.k, g.kp, g.dp, xabs, cabs, cmax,
                       mode == KM_SCREEN_FAST1 ? 1 : 2, reinterpret_cast<uint16_t*>(ChiF), bal, gate);
    constexpr int WAVES = 4;
    const int64_t ntiles = (g.n + 31) / 32;
    int64_t blocks = n_cu;
    if (blocks > (ntiles + WAVES - 1) / WAVES) blocks = (ntiles + WAVES - 1) / WAVES;
    const int nbk = (int)blocks;
    const int64_t nw = (int64_t)nbk * WAVES;
    const uint32_t seg = (uint32_t)(((ntiles + nw - 1) / nw) * 32);
    ql->seg = seg;
    ql->nwaves = (uint32_t)nw;
    FusedArgs a{X, xnorm, g.n, g.k, g.d, seg, ChiF, CloF, cn2s, bnd, xabs, cabs, labels, queue, qcount, stats, gate,
                C64P, sse};
    const size_t lds = (size_t)g.kp * 4 + (with_stats ? (size_t)(g.dp + 1) * g.kp * 8 : 0);
    if (mode == KM_SCREEN_FAST1) {
      if (with_stats)
        KM_TIMED_LAUNCH((k_fused1<4, 8, 1, true, WAVES>), dim3(nbk), dim3(WAVES * 64), lds, s, a, bal, cmax);
      else
        KM_TIMED_LAUNCH((k_fused1<4, 8, 1, false, WAVES>), dim3(nbk), dim3(WAVES * 64), lds, s, a, bal, cmax);
    } else {
      if (with_stats)
        KM_TIMED_LAUNCH((k_fused1<4, 8, 2, true, WAVES>), dim3(nbk), dim3(WAVES * 64), lds, s, a, bal, cmax);
      else
        KM_TIMED_LAUNCH((k_fused1<4, 8, 2, false, WAVES>), dim3(nbk), dim3(WAVES * 64), lds, s, a, bal, cmax);
    }
    return hipGetLastError();
  }
#endif
  const bool shape16 = fused16_ok(g);
  if (shape16) {
    const int total = (g.kp / 16) * (g.dp / 32) * 64;
    hipLaunchKernelGGL(k_frag_images16, dim3((total + 255) / 256), dim3(256), 0, s, Chi, Clo, g.kp, g.dp, ChiF, CloF,
                       gate);
  } else {
    const int total = nb * ns * 64;
    hipLaunchKernelGGL(k_frag_images, dim3((total + 255) / 256), dim3(256), 0, s, Chi, Clo, g.kp, g.dp, ChiF, CloF, gate);
  }
  constexpr int WAVES = 4;
  const int64_t ntiles = (g.n + 31) / 32;
  int64_t blocks = n_cu;
  if (blocks > (ntiles + WAVES - 1) / WAVES) blocks = (ntiles + WAVES - 1) / WAVES;
  const int nbk = (int)blocks;
  const int64_t nw = (int64_t)nbk * WAVES;
  const uint32_t seg = (uint32_t)(((ntiles + nw - 1) / nw) * 32);
  ql->seg = seg;
  ql->nwaves = (uint32_t)nw;
  FusedArgs a{X, xnorm, g.n, g.k, g.d, seg, ChiF, CloF, cn2s, bnd, xabs, cabs, labels, queue, qcount, stats, gate,
                C64P, sse};
  const size_t lds = (size_t)g.kp * 4 + (with_stats ? (size_t)(g.dp + 1) * g.kp * 8 : 0);
#define KM_FUSED_CASE(NS_, NB_)                                                                        \
  case NS_ * 100 + NB_:                                                                                \
    if (with_stats && sse)                                                                             \
      KM_TIMED_LAUNCH((k_fused<NS_, NB_, true, true, true>), dim3(nbk), dim3(256), lds, s, a);   \
    else if (with_stats && !refine)                                                                    \
      KM_TIMED_LAUNCH((k_fused<NS_, NB_, true, false>), dim3(nbk), dim3(256), lds, s, a);        \
    else if (with_stats)                                                                               \
      KM_TIMED_LAUNCH((k_fused<NS_, NB_, true>), dim3(nbk), dim3(256), lds, s, a);                  \
    else                                                                                               \
      KM_TIMED_LAUNCH((k_fused<NS_, NB_, false>), dim3(nbk), dim3(256), lds, s, a);                 \
    break;
#define KM_FUSED16_CASE(NS2_, NB_)                                                                      \
  case NS2_ * 100 + NB_:                                                                                \
    if (with_stats && sse)                                                                              \
      KM_TIMED_LAUNCH((k_fused16<NS2_, NB_, true, true, true>), dim3(nbk), dim3(256), lds, s, a);    \
    else if (with_stats && !refine)                                                                     \
      KM_TIMED_LAUNCH((k_fused16<NS2_, NB_, true, false>), dim3(nbk), dim3(256), lds, s, a);         \
    else if (with_stats)                                                                                \
      KM_TIMED_LAUNCH((k_fused16<NS2_, NB_, true>), dim3(nbk), dim3(256), lds, s, a);                \
    else if (KM_F16_PREDICT == 1)                                                                       \
      KM_TIMED_LAUNCH((k_fused16<NS2_, NB_, true>), dim3(nbk), dim3(256), lds_s, s, a);              \
    else if (KM_F16_PREDICT == 2)                                                                       \
      KM_TIMED_LAUNCH((k_fused16<NS2_, NB_, false, false>), dim3(nbk), dim3(256), lds, s, a);        \
    else                                                                                                \
      KM_TIMED_LAUNCH((k_fused16<NS2_, NB_, false>), dim3(nbk), dim3(256), lds, s, a);               \
    break;
#ifndef KM_F16_PREDICT
#define KM_F16_PREDICT 0
#endif
  const size_t lds_s = (size_t)g.kp * 4 + (size_t)(g.dp + 1) * g.kp * 8;
  if (shape16) {
    switch ((g.dp / 32) * 100 + nb) {
      KM_FUSED16_CASE(2, 2) KM_FUSED16_CASE(2, 4) KM_FUSED16_CASE(2, 6) KM_FUSED16_CASE(2, 8)
      KM_FUSED16_CASE(1, 2) KM_FUSED16_CASE(1, 4) KM_FUSED16_CASE(1, 6) KM_FUSED16_CASE(1, 8) KM_FUSED16_CASE(1, 12)
      KM_FUSED16_CASE(1, 16)
      KM_FUSED16_CASE(4, 2) KM_FUSED16_CASE(4, 4)
      default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
#undef KM_FUSED16_CASE
  switch (ns * 100 + nb) {
    KM_FUSED_CASE(4, 2) KM_FUSED_CASE(4, 4) KM_FUSED_CASE(4, 6) KM_FUSED_CASE(4, 8)
    KM_FUSED_CASE(2, 2) KM_FUSED_CASE(2, 4) KM_FUSED_CASE(2, 6) KM_FUSED_CASE(2, 8) KM_FUSED_CASE(2, 12)
    KM_FUSED_CASE(2, 16)
    KM_FUSED_CASE(3, 2) KM_FUSED_CASE(3, 4) KM_FUSED_CASE(3, 6) KM_FUSED_CASE(3, 8)
    KM_FUSED_CASE(8, 2) KM_FUSED_CASE(8, 4)
    default:
      return hipErrorInvalidValue;
  }
#undef KM_FUSED_CASE
  return hipGetLastError();
}

hipError_t launch_bound_consts(const float* cmax, const float* xabs, const float* cabs, const Geometry& g, float* bnd,
                               const int* gate, hipStream_t s) {
  hipLaunchKernelGGL(k_bound_consts, dim3(1), dim3(1), 0, s, cmax, xabs, cabs, g.dp, fused16_ok(g) ? 1 : 0, bnd,
                     gate);
  return hipGetLastError();
}

hipError_t launch_row_norm(const float* X, const Geometry& g, float* xnorm, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  int64_t blocks = (g.n + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  const dim3 grid((unsigned)blocks), blk(256);
  switch (g.dp / 4) {  // dp in {16, 32, 48, 64, 96, 128, 192, 256}; L must divide 64 -> 48/96/192 use 16 lanes x more
    case 4: hipLaunchKernelGGL(k_row_norm<4>, grid, blk, 0, s, X, g.n, xnorm); break;
    case 8: hipLaunchKernelGGL(k_row_norm<8>, grid, blk, 0, s, X, g.n, xnorm); break;
    case 16: hipLaunchKernelGGL(k_row_norm<16>, grid, blk, 0, s, X, g.n, xnorm); break;
    case 32: hipLaunchKernelGGL(k_row_norm<32>, grid, blk, 0, s, X, g.n, xnorm); break;
    case 64: hipLaunchKernelGGL(k_row_norm<64>, grid, blk, 0, s, X, g.n, xnorm); break;
    default: hipLaunchKernelGGL(k_row_norm_any, grid, blk, 0, s, X, g.n, g.dp, xnorm); break;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Exact float64 resolution of the queued ambiguous points (np.argmin with
// first-minimum tie-break, kmeans_spark.py:153-156).
//   k_rerank2:   {i1, i2} re-ranked, 16 lanes per entry (4 entries per wave,
//                float4 / double2 loads, all issued before use).
//   k_fullscan:  full scan, G entries per wave, lanes over centroids, the
//                transposed float64 centroids C64T[d][k] streamed through
//                LDS in column chunks shared by the workgroup's entries.
// Walks the per-wave queue segments written by k_assign_mfma.
// ---------------------------------------------------------------------------
// Exclusive prefix over the per-segment queue counts (word `which` of each
// count pair) into LDS pre[0..nseg]; blockDim.x a multiple of 64, <= 1024.
__device__ void block_prefix(const uint32_t* __restrict__ qcount, int which, uint32_t nseg,
                             uint32_t* __restrict__ pre) {
  __shared__ uint32_t wsum[16];
  const uint32_t t = threadIdx.x;
  const uint32_t nt = blockDim.x;
  const uint32_t chunk = (nseg + nt - 1u) / nt;
  const uint32_t b0 = t * chunk;
  uint32_t v = 0;
  for (uint32_t i = 0; i < chunk; ++i)
    if (b0 + i < nseg) v += qcount[2 * (b0 + i) + which];
  const int lane = t & 63, w = t >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (int i = 0; i < w; ++i) base += wsum[i];
  uint32_t run = base + inc - v;  // exclusive prefix of this thread's chunk
  for (uint32_t i = 0; i < chunk; ++i)
    if (b0 + i < nseg) {
      pre[b0 + i] = run;
      run += qcount[2 * (b0 + i) + which];
    }
  if (t == nt - 1) {
    uint32_t tot = 0;
    for (uint32_t i = 0; i < nt / 64; ++i) tot += wsum[i];
    pre[nseg] = tot;
  }
  __syncthreads();
}

// segment holding global entry g: the last sg with pre[sg] <= g
__device__ __forceinline__ uint32_t find_segment(const uint32_t* __restrict__ pre, uint32_t nseg, uint32_t g) {
  uint32_t lo = 0, hi = nseg;  // pre[lo] <= g < pre[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= g)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// With stats != nullptr the resolved points' rows are added to the partial
// sums (the fused kernel leaves every queued point to the resolvers): into an
// LDS table [f][j] flushed at the end when it fits (tab_kp > 0), else with
// global float64 atomics.  The entries of all segments are spread over all
// waves of the grid, 8 lanes per entry (np_pw8: lane u owns NumPy's
// accumulator u, so the rounding is the reference's), 8 entries per wave.
// PF (d <= 128, with the fp32 images C32 and their largest norm *cmax): the
// candidates are first scored in fp32 (each lane its features u + 8 m, summed
// over the 8 lanes) with k_fullscan's bounds [L, U] on ||x - c||; only those
// whose L is at most the smallest U (x (1 + 8u)) are evaluated in float64,
// and a single one is the answer without float64 (every other candidate is
// farther by more than 4.8e-7 relative, far beyond NumPy's rounding)
template <bool WIDE, bool PF = false>  // WIDE: d > 256 (five pairwise halvings; 512 threads, 256 VGPRs)
__global__ __launch_bounds__(WIDE ? 512 : 1024) void k_rerank2(const float* __restrict__ X, int dp, int d, int k,
                                                  const double* __restrict__ C64, const QEntry* __restrict__ queue,
                                                  const uint32_t* __restrict__ qcount, QLayout ql,
                                                  int32_t* __restrict__ labels, double* __restrict__ stats,
                                                  int tab_kp, double* __restrict__ sse, const int* __restrict__ gate,
                                                  const uint32_t* __restrict__ cand, uint32_t cand_cap, int delta,
                                                  const float* __restrict__ sse_c32, uint2* __restrict__ chg,
                                                  const uint32_t* __restrict__ chg_cnt,
                                                  const float* __restrict__ C32, const float* __restrict__ cmax) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const float cmv = PF ? *cmax : 0.0f;
  double* tab = reinterpret_cast<double*>(smem);
  uint32_t* pre = reinterpret_cast<uint32_t*>(smem + (stats && tab_kp ? (size_t)(d + 1) * tab_kp * 8 : 0));
  uint32_t* pre1 = pre + ql.nwaves + 1;  // full / chain scan entries (their sums only)
  if (stats && tab_kp)
    for (int i = threadIdx.x; i < (d + 1) * tab_kp; i += blockDim.x) tab[i] = 0.0;
  block_prefix(qcount, 0, ql.nwaves, pre);
  if (stats && !delta) block_prefix(qcount, 1, ql.nwaves, pre1);
  const uint32_t total = pre[ql.nwaves];
  const int u = threadIdx.x & 7;
  const uint32_t ng = (gridDim.x * blockDim.x) >> 3;
  double ss_acc = 0.0;
  // the loop trip count is uniform over each 8-lane group (shuffles inside)
  for (uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 3; g < total + ((ng - total % ng) % ng);
       g += ng) {
    const bool have = g < total;
    QEntry q{0, 0, 0, 0};
    size_t cpos = 0;  // delta: this entry's slot in the change list
    if (have) {
      const uint32_t sg = find_segment(pre, ql.nwaves, g);
      q = queue[(size_t)sg * ql.seg + (g - pre[sg])];
      if (delta) cpos = (size_t)sg * ql.seg + chg_cnt[sg] + (g - pre[sg]);
    }
    // kind 4: a candidate list (k_assign_mfma), count + ascending indices
    const uint32_t* rec = (have && q.kind == 4u && cand != nullptr && q.i2 < cand_cap)
                              ? cand + (size_t)q.i2 * CAND_REC : nullptr;
    const int nc = rec ? (int)min(rec[0], (uint32_t)(CAND_REC - 1)) : 0;
    const bool ok = have && (rec ? (nc >= 1 && rec[nc] < (uint32_t)k)
                                 : (q.kind != 4u && q.i1 < (uint32_t)k && q.i2 < (uint32_t)k));
    const float* __restrict__ x = X + (size_t)q.row * dp;
    int lab = 0;
    double mnorm = 0.0;  // the chosen centroid's norm (SSE)
    // np.argmin over ascending candidates, two norms per pass (NumPy's
    // pairwise order, 8 lanes per entry); kind 1 is the pass over {i1, i2}
    int npass = rec ? (ok ? (nc + 1) / 2 : 0) : 1;
    int bi = -1;
    const int ncand = rec ? nc : 2;
    uint32_t keep = 0xFFFFu;  // candidate positions evaluated in float64
    if constexpr (PF) {
      // fp32 prefilter (see above); positions p < ncand, ascending indices
      bool fin = ok;
      float xr[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int f = u + 8 * m;
        xr[m] = (ok && f < d) ? x[f] : 0.0f;
        fin = fin && fabsf(xr[m]) <= 3.0e38f;
      }
      fin = fin && (cmv <= 3.0e38f);
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) fin = fin && __shfl_xor((int)fin, o) != 0;
      if (fin) {
        const float e = ((float)((d + 7) / 8 + 8) * 0.5f + 8.0f) * U24 * 1.1f;
        const float gam = U24 * cmv * 1.01f + 1e-37f;
        float Lp[CAND_REC - 1];
        float Us = FLT_MAX;
#pragma unroll
        for (int p = 0; p < CAND_REC - 1; ++p) {
          Lp[p] = FLT_MAX;
          if (p < ncand) {
            const int j = rec ? (int)rec[1 + p] : (p == 0 ? (int)min(q.i1, q.i2) : (int)max(q.i1, q.i2));
            const float* cj = C32 + (size_t)j * dp;
            float D = 0.0f;
#pragma unroll
            for (int m = 0; m < 16; ++m) {
              const int f = u + 8 * m;
              const float df = xr[m] - (f < d ? cj[f] : 0.0f);
              D = fmaf(df, df, D);
            }
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) D += __shfl_xor(D, o);
            const bool tiny = !(D >= 0x1p-96f);
            const float r = __builtin_amdgcn_sqrtf(tiny ? 0x1p-96f : D);
            const float U = fmaf(r, 1.0f + e, gam) * (1.0f + 4.0f * U24);
            Lp[p] = fmaf(tiny ? 0.0f : r, 1.0f - e, -gam) * (1.0f - 4.0f * U24);
            Us = fminf(Us, U);
          }
        }
        keep = 0u;
#pragma unroll
        for (int p = 0; p < CAND_REC - 1; ++p) keep |= (Lp[p] <= Us * (1.0f + 8.0f * U24)) ? (1u << p) : 0u;
        if (__popc(keep) == 1 && !(sse && !sse_c32)) {
          // one candidate left: NumPy's argmin (no float64 needed)
          const int p1 = __ffs(keep) - 1;
          bi = rec ? (int)rec[1 + p1] : (p1 == 0 ? (int)min(q.i1, q.i2) : (int)max(q.i1, q.i2));
          npass = 0;
        }
      }
    }
    for (int t = 0; t < npass; ++t) {
      int a, bb;
      if (rec) {
        a = (int)rec[1 + 2 * t];
        bb = 2 * t + 1 < nc ? (int)rec[2 + 2 * t] : a;
      } else {
        a = ok ? (int)min(q.i1, q.i2) : 0;
        bb = ok ? (int)max(q.i1, q.i2) : 0;
      }
      if constexpr (PF) {
        // positions dropped by the prefilter: skipped (a pair with one kept
        // evaluates it twice, as the odd tail does)
        const bool ka = (keep >> (2 * t)) & 1u, kb = 2 * t + 1 < ncand && ((keep >> (2 * t + 1)) & 1u);
        if (!ka && !kb) continue;
        if (!ka) a = bb;
        if (!kb) bb = a;
      }
      const double* __restrict__ ca = C64 + (size_t)a * d;
      const double* __restrict__ cb = C64 + (size_t)bb * d;
      double sa, sb;
      auto sq2 = [&](int f, double& ta, double& tb) {
        const float xf = x[f];
        ta = np_sq(ca[f], xf);
        tb = np_sq(cb[f], xf);
      };
      if constexpr (WIDE)
        np_pw8<5>(sq2, 0, d, u, sa, sb);  // d <= 2048
      else
        np_pw8<2>(sq2, 0, d, u, sa, sb);
      const double va = sqrt(sa), vb = sqrt(sb);
      // running minimum updated with selects (the
      // branchy form is miscompiled in divergent code on this toolchain)
      const bool ua = np_better(va, mnorm, bi >= 0);
      mnorm = ua ? va : mnorm;
      bi = ua ? a : bi;
      const bool ub = bb != a && np_better(vb, mnorm, true);
      mnorm = ub ? vb : mnorm;
      bi = ub ? bb : bi;
    }
    lab = bi < 0 ? 0 : bi;
    if (!have) continue;
    double rsq_bad = 0.0;
    if (!ok && u == 0) {
      // corrupt candidate (cannot happen for finite data): full scan
      double best = 0.0;
      for (int j = 0; j < k; ++j) {
        const double* __restrict__ c = C64 + (size_t)j * d;
        const double v = np_norm_d<WIDE ? 5 : 2>([&](int f) { return np_sq(c[f], x[f]); }, d);
        const bool u = np_better(v, best, j > 0);  // select form
        best = u ? v : best;
        lab = u ? j : lab;
      }
      rsq_bad = best;  // the norm (np_norm_d takes the sqrt)
    }
    if (!ok) lab = __shfl(lab, (int)(threadIdx.x & 63) & ~7);
    // delta statistics (k_s1): the queued row still holds its previous label
    const int old = delta ? (int)min((uint32_t)labels[q.row], (uint32_t)(k - 1)) : -1;
    if (u == 0) labels[q.row] = lab;
    // SSE (fused path): min_distance ** 2 with the chosen centroid's norm in
    // NumPy's order (kmeans_spark.py:231-233); with sse_c32 (k_s1's delta
    // fit) the residual to the fp32 image c' of the centroid instead, as k_s1
    // adds it for the rows it decides (the update corrects the total)
    if (sse && sse_c32) {
      double r = 0.0;
      for (int f = u; f < d; f += 8) {
        const double e = (double)x[f] - (double)sse_c32[(size_t)lab * dp + f];
        r = fma(e, e, r);
      }
      ss_acc += r;
    } else if (sse && u == 0) {
      const double mn = ok ? mnorm : rsq_bad;
      ss_acc += mn * mn;
    }
    if (delta) {
      // the row's entry behind the screen's changes in its wave segment
      // (old == lab: no move), folded with them by k_s1_delta
      if (u == 0) chg[cpos] = make_uint2(q.row, ((uint32_t)old << 16) | (uint32_t)lab);
    } else if (stats) {
      for (int f = u; f < d; f += 8) {
        if (tab_kp)
          atomicAdd(tab + (size_t)f * tab_kp + lab, (double)x[f]);
        else
          atomicAdd(stats + (size_t)lab * (d + 1) + f, (double)x[f]);
      }
      if (u == 0) {  // count
        if (tab_kp)
          atomicAdd(tab + (size_t)d * tab_kp + lab, 1.0);
        else
          atomicAdd(stats + (size_t)lab * (d + 1) + d, 1.0);
      }
    }
  }
  if (stats && !delta) {
    // rows of the entries k_fullscan resolved (launched first: their labels
    // are final) into the same table -- one global float64 atomic per table
    // entry instead of one per feature per point, which serialised on the
    // few clusters that collect most scanned points (c3 k_fullscan 0.42 -> 0.38 ms)
    const uint32_t total1 = pre1[ql.nwaves];
    const uint32_t g0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 3;
    for (uint32_t g = g0; g < total1; g += ng) {
      const uint32_t sg = find_segment(pre1, ql.nwaves, g);
      const QEntry q = queue[(size_t)sg * ql.seg + (ql.seg - 1u - (g - pre1[sg]))];
      const int lab = labels[q.row];
      const float* __restrict__ x = X + (size_t)q.row * dp;
      for (int f = u; f < d; f += 8) {
        if (tab_kp)
          atomicAdd(tab + (size_t)f * tab_kp + lab, (double)x[f]);
        else
          atomicAdd(stats + (size_t)lab * (d + 1) + f, (double)x[f]);
      }
      if (u == 0) {
        if (tab_kp)
          atomicAdd(tab + (size_t)d * tab_kp + lab, 1.0);
        else
          atomicAdd(stats + (size_t)lab * (d + 1) + d, 1.0);
      }
    }
  }
  if (stats && tab_kp) {
    __syncthreads();
    for (int i = threadIdx.x; i < (d + 1) * tab_kp; i += blockDim.x) {
      const int j = i / (d + 1);
      const int f = i - j * (d + 1);
      const double v = tab[(size_t)f * tab_kp + j];
      if (v != 0.0 && j < k) atomicAdd(stats + (size_t)j * (d + 1) + f, v);
    }
  }
  if (sse) {
    ss_acc = wave_sum(ss_acc);  // lanes u == 0 hold the entries' terms
    if ((threadIdx.x & 63) == 0 && ss_acc != 0.0) atomicAdd(sse, ss_acc);
  }
}

// Full exact scans.  A workgroup (8 waves) takes batches of 8 G queued
// points, G per wave; the transposed centroids stream through LDS in chunks
// of ch columns ([d][ch] doubles), each chunk serving all 8 G points, so
// C64T is read once per batch instead of once per point (at k = 4096,
// d = 128 it is 4 MiB).  Lane j of a wave evaluates centroid c0 + j for
// each of its G points in NumPy's order (np_norm), from the chunk (one
// conflict-free double per lane) and the point's row staged in LDS
// (broadcast reads).  Full-scan entries sit at the back of each segment.
// PF (fp32 prefilter, d <= 256 with the fp32 images C32 [kp][dp] and their
// largest norm *cmax): the scan runs in fp32 first -- D~ = sum (x - c')^2 from
// fp32 chunks of the images in LDS (packed differences and fmas), its bounds
// [L, U] on ||x - c|| as in k_s1's re-score (sum rounding (d/2 + 8) u,
// sqrt 4 u, ||c - c'|| <= u cmax) -- and a point keeps, per chunk, the
// centroids whose L is under the smallest U so far (the running minimum only
// falls, so the true argmin is kept: its L is under every U).  Those (<= 64)
// are then evaluated in float64 in NumPy's order, one per lane, and the
// usual argmin decides.  A point with a non-finite row, non-finite
// centroids or more than 64 kept centroids takes the float64 chunk pass.
template <int G, bool WIDE, bool PF = false>  // WIDE: d > 256, no LDS chunks (ch = 0)
__global__ __launch_bounds__(512) void k_fullscan(const float* __restrict__ X, int dp, int d, int k,
                                                   const double* __restrict__ C64T, const QEntry* __restrict__ queue,
                                                   const uint32_t* __restrict__ qcount, QLayout ql,
                                                   int32_t* __restrict__ labels, int ch,
                                                   double* __restrict__ stats, int use_chain, int pair_chain,
                                                   double* __restrict__ sse, const int* __restrict__ gate, int delta,
                                                   const float* __restrict__ sse_c32, uint2* __restrict__ chg,
                                                   const uint32_t* __restrict__ chg_cnt,
                                                   const float* __restrict__ C32, const float* __restrict__ cmax,
                                                   const double* __restrict__ C64r) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sCT = reinterpret_cast<double*>(smem);                                    // [d][ch]
  float* xs_all = reinterpret_cast<float*>(smem + (size_t)d * ch * 8);              // [8][G][d]
  uint32_t* pre = reinterpret_cast<uint32_t*>(smem + (size_t)d * ch * 8 + (size_t)8 * G * d * 4);
  // PF: the kept centroids [8][G][64] behind the prefix (16-B aligned)
  uint32_t* kept_all = pre + ((ql.nwaves + 1u + 3u) & ~3u);
  const float cmv = PF ? *cmax : 0.0f;
  block_prefix(qcount, 1, ql.nwaves, pre);
  const uint32_t total = pre[ql.nwaves];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float* xs = xs_all + (size_t)wave * G * d;
  const uint32_t per_batch = 8u * G;
  double ss_acc = 0.0;  // SSE (fused path): lane 0's sum of the chosen sums of squares
  for (uint32_t b0 = blockIdx.x * per_batch; b0 < total; b0 += gridDim.x * per_batch) {
    uint32_t rows[G];
    bool have[G];
    int chain[G];  // kind 3: the chain j & 7 to scan, else -1
    // the G entries' queue words, then their rows, each as one batch of
    // independent loads (past-the-end slots read the last entry, unused)
    QEntry qe[G];
    size_t cpos[G];  // delta: the entries' slots in the change list
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t e = b0 + (uint32_t)(wave * G + g);
      have[g] = e < total;
      const uint32_t ec = have[g] ? e : total - 1u;
      const uint32_t sg = find_segment(pre, ql.nwaves, ec);
      qe[g] = queue[(size_t)sg * ql.seg + (ql.seg - 1u - (ec - pre[sg]))];
      cpos[g] = delta ? (size_t)sg * ql.seg + chg_cnt[sg] + qcount[2 * sg] + (ec - pre[sg]) : 0;
    }
    float xv[G][4];  // features [0, 256); wider rows stage the rest below
#pragma unroll
    for (int g = 0; g < G; ++g) {
      rows[g] = __builtin_amdgcn_readfirstlane(qe[g].row);
      const uint32_t kind = __builtin_amdgcn_readfirstlane(qe[g].kind);
      const uint32_t i1 = __builtin_amdgcn_readfirstlane(qe[g].i1);
      chain[g] = (use_chain && have[g] && kind == 3u && i1 < (uint32_t)k) ? (int)(i1 & 7u) : -1;
      const float* x = X + (size_t)rows[g] * dp;
#pragma unroll
      for (int u = 0; u < 4; ++u) xv[g][u] = (lane + 64 * u < d) ? x[lane + 64 * u] : 0.0f;
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (lane + 64 * u < d) xs[g * d + lane + 64 * u] = xv[g][u];
    if (WIDE)
#pragma unroll
      for (int g = 0; g < G; ++g)
        for (int f = 256 + lane; f < d; f += 64) xs[g * d + f] = X[(size_t)rows[g] * dp + f];
    // np.argmin across lanes (first NaN, else smallest value, lowest index),
    // then the label and, when fused, the point's row into the sums
    auto finish = [&](int g, double bv, int bi) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const double ob = __shfl_xor(bv, o);
        const int oj = __shfl_xor(bi, o);
        bool take = false;
        if (oj >= 0) {
          if (bi < 0) {
            take = true;
          } else {
            const bool on = ob != ob, mn = bv != bv;
            take = (on && !mn) || (on == mn && (on ? oj < bi : (ob < bv || (ob == bv && oj < bi))));
          }
        }
        bv = take ? ob : bv;  // select form
        bi = take ? oj : bi;
      }
      const int lab = bi < 0 ? 0 : bi;
      // delta statistics (k_s1): the queued row still holds its previous label
      const int old = delta ? (int)min((uint32_t)labels[rows[g]], (uint32_t)(k - 1)) : -1;
      if (lane == 0) labels[rows[g]] = lab;
      if (sse && sse_c32) {  // k_s1's delta fit: the residual to c' (see k_rerank2)
        for (int f = lane; f < d; f += 64) {
          const double e = (double)xs[g * d + f] - (double)sse_c32[(size_t)lab * dp + f];
          ss_acc = fma(e, e, ss_acc);
        }
      } else if (sse && lane == 0 && bi >= 0) {
        ss_acc += bv * bv;  // min_distance ** 2 (bv: the norm)
      }
      if (delta) {
        // the row's entry behind the screen's changes and the re-rank
        // entries of its wave segment (old == lab: no move; k_s1_delta)
        if (lane == 0) chg[cpos[g]] = make_uint2(rows[g], ((uint32_t)old << 16) | (uint32_t)lab);
      } else if (stats) {
        for (int f = lane; f < d; f += 64) atomicAdd(stats + (size_t)lab * (d + 1) + f, (double)xs[g * d + f]);
        if (lane == 0) atomicAdd(stats + (size_t)lab * (d + 1) + d, 1.0);  // count
      }
    };
    // chain scans (kind 3, written only by the dp <= 256 screens: two pairwise
    // halvings): the wave evaluates members j = chain + 8 m, lanes
    // over m, straight from C64T (no barriers: done before the chunk loop)
    // k <= 256: a chain has <= 32 members, so two entries share a pass (lane
    // half e of the wave on entry p + e); the other half enters the 64-lane
    // argmin with no candidate
    if (k <= 256 && pair_chain) {
      static_assert(G % 2 == 0, "entry pairs");
#pragma unroll
      for (int p = 0; p < G; p += 2) {
        const bool a0 = have[p] && chain[p] >= 0, a1 = have[p + 1] && chain[p + 1] >= 0;
        if (!a0 && !a1) continue;
        const int e = lane >> 5;
        const int j = (e ? chain[p + 1] : chain[p]) + 8 * (lane & 31);
        double bv = 0.0;
        int bi = -1;
        if ((e ? a1 : a0) && j < k) {
          const float* xg = xs + (p + e) * d;
          bv = np_norm_d<2>([&](int f) { return np_sq(C64T[(size_t)f * k + j], xg[f]); }, d);
          bi = j;
        }
        if (a0) {
          finish(p, e == 0 ? bv : 0.0, e == 0 ? bi : -1);
          have[p] = false;
        }
        if (a1) {
          finish(p + 1, e == 1 ? bv : 0.0, e == 1 ? bi : -1);
          have[p + 1] = false;
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (!have[g] || chain[g] < 0) continue;
      double bv = 0.0;
      int bi = -1;
      for (int j = chain[g] + 8 * lane; j < k; j += 8 * 64) {
        const float* xg = xs + g * d;
        const double v = np_norm_d<2>([&](int f) { return np_sq(C64T[(size_t)f * k + j], xg[f]); }, d);
        const bool u = np_better(v, bv, bi >= 0);  // select form
        bv = u ? v : bv;
        bi = u ? j : bi;
      }
      finish(g, bv, bi);
      have[g] = false;
    }
    if constexpr (PF) {
      // fp32 prefilter (see above): the wave's points with finite rows
      bool ok[G];
      bool any = false;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        bool fin = true;
        for (int f = lane; f < d; f += 64) fin = fin && (fabsf(xs[g * d + f]) <= 3.0e38f);
        ok[g] = have[g] && (cmv <= 3.0e38f) && __ballot(!fin) == 0ull;
        any |= ok[g];
      }
      if (__syncthreads_or(any)) {
        uint32_t* kept = kept_all + (size_t)wave * G * 64;
        float ust[G];
        uint32_t nk[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          ust[g] = FLT_MAX;
          nk[g] = 0u;
        }
        const int cs2 = ch + 1;  // f32x2 row stride of the chunk (bank spread of the transposed writes)
        const float e = ((float)(d / 2 + 8) * 0.5f + 8.0f) * U24 * 1.1f;
        const float gam = U24 * cmv * 1.01f + 1e-37f;
        typedef float f32x2_t __attribute__((ext_vector_type(2)));
        f32x2_t* sC = reinterpret_cast<f32x2_t*>(sCT);  // [d/2][ch + 1] feature pairs
        // chunk staging: float4 pieces of the images' rows (dp a power of
        // two: Q pieces per row), the next chunk's loads in flight in
        // registers while this one is scanned
        const int Q = dp >> 2, lq = __builtin_ctz((unsigned)Q), nf4 = ch * Q;
        const float4* C32v = reinterpret_cast<const float4*>(C32);
        float4 nv[4];
        auto fetch = [&](int c0) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int idx = threadIdx.x + t * (int)blockDim.x;
            const int jj = idx >> lq, q4 = idx & (Q - 1);
            nv[t] = (idx < nf4 && c0 + jj < k) ? C32v[(size_t)(c0 + jj) * Q + q4] : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        };
        auto put = [&]() {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int idx = threadIdx.x + t * (int)blockDim.x;
            const int jj = idx >> lq, q4 = idx & (Q - 1), p0 = 2 * q4;  // feature pairs p0, p0 + 1
            if (idx < nf4 && 2 * p0 < d) sC[p0 * cs2 + jj] = f32x2_t{nv[t].x, nv[t].y};
            if (idx < nf4 && 2 * p0 + 2 < d) sC[(p0 + 1) * cs2 + jj] = f32x2_t{nv[t].z, nv[t].w};
          }
        };
        fetch(0);
        for (int c0 = 0; c0 < k; c0 += ch) {
          __syncthreads();  // the previous chunk is scanned
          const int cw = min(ch, k - c0);
          put();
          if (c0 + ch < k) fetch(c0 + ch);
          __syncthreads();
          f32x2_t acc[G];
#pragma unroll
          for (int g = 0; g < G; ++g) acc[g] = f32x2_t{0.0f, 0.0f};
#pragma unroll 4
          for (int fp = 0; fp < (d >> 1); ++fp) {
            const f32x2_t c2 = sC[fp * cs2 + lane];
#pragma unroll
            for (int g = 0; g < G; ++g) {
              const f32x2_t x2 = reinterpret_cast<const f32x2_t*>(xs + g * d)[fp];
              const f32x2_t df = x2 - c2;
              acc[g] = __builtin_elementwise_fma(df, df, acc[g]);
            }
          }
#pragma unroll
          for (int g = 0; g < G; ++g) {
            if (!ok[g]) continue;
            const bool in = lane < cw;
            const float Dt = acc[g].x + acc[g].y;
            const bool tiny = !(Dt >= 0x1p-96f);
            const float r = __builtin_amdgcn_sqrtf(tiny ? 0x1p-96f : Dt);
            const float U = in ? fmaf(r, 1.0f + e, gam) * (1.0f + 4.0f * U24) : FLT_MAX;
            const float L = in ? fmaf(tiny ? 0.0f : r, 1.0f - e, -gam) * (1.0f - 4.0f * U24) : FLT_MAX;
            float um = U;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) um = fminf(um, __shfl_xor(um, o));
            ust[g] = fminf(ust[g], um);
            const bool keep = in && L <= ust[g] * (1.0f + 8.0f * U24);
            const uint64_t m = __ballot(keep);
            const uint32_t nm = (uint32_t)__popcll(m);
            if (nk[g] + nm <= 64u && keep)
              kept[g * 64 + nk[g] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)(c0 + lane);
            nk[g] += nm;
          }
        }
        __syncthreads();  // the kept lists are visible to every lane
        // the kept centroids in float64, NumPy's order, one per lane
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if (!ok[g] || nk[g] > 64u) continue;  // more kept: the float64 chunk pass below
          const bool act = (uint32_t)lane < nk[g];
          const int j = act ? (int)kept[g * 64 + lane] : 0;
          const float* xg = xs + g * d;
          double bv = 0.0;
          int bi = -1;
          if (act) {
            const double* cj = C64r + (size_t)j * d;  // row-major: one contiguous row per lane
            bv = np_norm_d<2>([&](int f) { return np_sq(cj[f], xg[f]); }, d);
            bi = j;
          }
          finish(g, bv, bi);
          have[g] = false;
        }
      }
    }
    double best[G];
    int bj[G];
    bool any_full = false;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      best[g] = 0.0;
      bj[g] = -1;
      any_full |= have[g];
    }
    // most batches hold chain scans only: skip the chunk pass unless some
    // wave of the workgroup still has a full scan
    if (!__syncthreads_or(any_full)) continue;
    // (reading C64T straight from L2 for short queues as well, instead of
    // staging chunks through LDS, doubled the c3 resolve time on one box:
    // 0.069 -> 0.137 ms; only the wide rows do it)
    constexpr bool direct = WIDE;
    if (direct) {
      // lane j reads C64T straight from L2, consecutive centroids on
      // consecutive lanes
      static_assert(G == 2 || G == 4, "entries per wave");
      auto direct = [&](int j, const float* xg, double& bst, int& bjj) {
        const double v = WIDE ? np_norm_d<5>([&](int f) { return np_sq(C64T[(size_t)f * k + j], xg[f]); }, d)
                              : np_norm_d<2>([&](int f) { return np_sq(C64T[(size_t)f * k + j], xg[f]); }, d);
        const bool u = np_better(v, bst, bjj >= 0);  // select form
        bst = u ? v : bst;
        bjj = u ? j : bjj;
      };
      for (int j = lane; j < k; j += 64) {
        if (have[0]) direct(j, xs, best[0], bj[0]);
        if (have[1]) direct(j, xs + d, best[1], bj[1]);
        if constexpr (G == 4) {
          if (have[2]) direct(j, xs + 2 * d, best[2], bj[2]);
          if (have[3]) direct(j, xs + 3 * d, best[3], bj[3]);
        }
      }
    }
    for (int c0 = 0; !direct && c0 < k; c0 += ch) {
      __syncthreads();  // the previous chunk is consumed (and the rows staged)
      const int cw = min(ch, k - c0);
      for (int i = threadIdx.x; i < d * ch; i += blockDim.x) {
        const int f = i / ch;
        const int jj = i - f * ch;
        sCT[i] = jj < cw ? C64T[(size_t)f * k + c0 + jj] : 0.0;
      }
      __syncthreads();
      if (lane < cw) {
        const double* ct = sCT + lane;
        // the wave's entries in pairs: each chunk value read once for two
        // points (np_pw2, NumPy's order for each); a pair with one entry
        // already resolved (chain scan) or past the end still evaluates the
        // other -- the decision is per entry, never per pair.  The running
        // minima are updated with selects, not branches: the branchy form
        //   if (have[g + 1] && np_better(vb, ...)) { best[g + 1] = vb; ... }
        // loses every update after the first chunk on this toolchain (the
        // per-chunk norms are right, the lane minima stay at chunk 0:
        // DESIGN.md section 2, "The lockstep full-scan variant"), which is
        // what made the round-2 lockstep variant return wrong labels.
#pragma unroll
        for (int g = 0; g < G; g += 2) {
          if (!have[g] && !have[g + 1]) continue;
          const float* xa = xs + g * d;
          const float* xb = xs + (g + 1) * d;
          double sa, sb;
          np_pw2<2>(
              [&](int f, double& ta, double& tb) {
                const double c = ct[(size_t)f * ch];
                ta = np_sq(c, xa[f]);
                tb = np_sq(c, xb[f]);
              },
              0, d, sa, sb);
          const double va = sqrt(sa), vb = sqrt(sb);
          const bool ua = have[g] && np_better(va, best[g], bj[g] >= 0);
          const bool ub = have[g + 1] && np_better(vb, best[g + 1], bj[g + 1] >= 0);
          best[g] = ua ? va : best[g];
          bj[g] = ua ? c0 + lane : bj[g];
          best[g + 1] = ub ? vb : best[g + 1];
          bj[g + 1] = ub ? c0 + lane : bj[g + 1];
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (have[g]) finish(g, best[g], bj[g]);
  }
  if (sse) {
    ss_acc = wave_sum(ss_acc);  // (lane 0 alone, or every lane with sse_c32)
    if (lane == 0 && ss_acc != 0.0) atomicAdd(sse, ss_acc);
  }
}

hipError_t launch_resolve(const float* X, const Geometry& g, const double* C64, const double* C64T,
                          const QEntry* queue, const uint32_t* qcount, const QLayout& ql, int32_t* labels,
                          double* stats, int n_cu, const int* gate, hipStream_t s, double* sse,
                          const uint32_t* cand, uint32_t cand_cap, int delta, const float* sse_c32, uint2* chg,
                          const uint32_t* chg_cnt, const float* C32, const float* cmax) {
  if (g.n == 0 || ql.nwaves == 0) return hipSuccess;
  if (delta && (!chg || !chg_cnt || g.k > 65535)) return hipErrorInvalidValue;
  if (delta) stats = nullptr;  // the moves go to the change list
  constexpr size_t LDS_MAX = 160 * 1024;
  const size_t pre_bytes = ((size_t)ql.nwaves + 1) * 4;
  if (pre_bytes > LDS_MAX / 4) return hipErrorInvalidValue;
  if (g.d > WIDE_MAX_DP) return hipErrorInvalidValue;
  // full / chain scans first (labels only); k_rerank2 then adds the sums of
  // both queues through its LDS table
  // entries per wave: 4 where k > 256 (half the chunk passes; c5 resolve
  // 16.6 -> 14.7 ms), else 2
  static const int fs_g = diag_env("KM_FS_G", 0);
  const int G = fs_g == 4 ? 4 : (fs_g == 2 ? 2 : (g.k > 256 ? 4 : 2));
  const int ch = g.d <= 128 ? 64 : (g.d <= 256 ? 32 : 0);  // chunk columns (<= 64 KiB of LDS); 0: direct
  // fp32 prefilter of the full scans (KM_FS_PF, default on) where the images
  // are given: + the kept lists [8][G][64] behind the 16-B aligned prefix
  static const int fs_pf = diag_env("KM_FS_PF", 1);
  const bool pf = fs_pf && ch > 0 && C32 != nullptr && cmax != nullptr && g.d % 2 == 0 &&
                  (g.dp == 32 || g.dp == 64 || g.dp == 128 || g.dp == 256) && (size_t)ch * g.dp / 4 <= 4 * 512;
  const size_t fs_lds = (size_t)g.d * ch * 8 + (size_t)8 * G * g.d * 4 +
                        (pf ? (((size_t)ql.nwaves + 4) & ~(size_t)3) * 4 + (size_t)8 * G * 64 * 4 : pre_bytes);
  if (fs_lds > LDS_MAX) return hipErrorInvalidValue;
  static const int use_chain = diag_env("KM_CHAIN", 1);
  static const int pair_chain = diag_env("KM_PAIR_CHAIN", 1);
  static const int fs_wg = diag_env("KM_FS_WG", 1);  // workgroups per CU (3: no measurable change)
  if (ch == 0)
    hipLaunchKernelGGL((k_fullscan<2, true>), dim3(n_cu * fs_wg), dim3(512), fs_lds, s, X, g.dp, g.d, g.k, C64T,
                       queue, qcount, ql, labels, ch, (double*)nullptr, use_chain, pair_chain, sse, gate, delta, sse_c32, chg,
                       chg_cnt, C32, cmax, C64);
  else if (G == 4 && pf)
    hipLaunchKernelGGL((k_fullscan<4, false, true>), dim3(n_cu * fs_wg), dim3(512), fs_lds, s, X, g.dp, g.d, g.k,
                       C64T, queue, qcount, ql, labels, ch, (double*)nullptr, use_chain, pair_chain, sse, gate, delta,
                       sse_c32, chg, chg_cnt, C32, cmax, C64);
  else if (G == 4)
    hipLaunchKernelGGL((k_fullscan<4, false>), dim3(n_cu * fs_wg), dim3(512), fs_lds, s, X, g.dp, g.d, g.k, C64T,
                       queue, qcount, ql, labels, ch, (double*)nullptr, use_chain, pair_chain, sse, gate, delta, sse_c32, chg,
                       chg_cnt, C32, cmax, C64);
  else if (pf)
    hipLaunchKernelGGL((k_fullscan<2, false, true>), dim3(n_cu * fs_wg), dim3(512), fs_lds, s, X, g.dp, g.d, g.k,
                       C64T, queue, qcount, ql, labels, ch, (double*)nullptr, use_chain, pair_chain, sse, gate, delta,
                       sse_c32, chg, chg_cnt, C32, cmax, C64);
  else
    hipLaunchKernelGGL((k_fullscan<2, false>), dim3(n_cu * fs_wg), dim3(512), fs_lds, s, X, g.dp, g.d, g.k, C64T,
                       queue, qcount, ql, labels, ch, (double*)nullptr, use_chain, pair_chain, sse, gate, delta, sse_c32, chg,
                       chg_cnt, C32, cmax, C64);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t tab_bytes = (size_t)(g.d + 1) * g.kp * 8;
  const size_t pres = (stats ? 2 : 1) * pre_bytes;
  // (delta: the moves go to the change list, stats is null)
  const int tab_kp = (stats && !delta && tab_bytes + pres <= LDS_MAX) ? g.kp : 0;
  // workgroups of the re-rank, in percent of n_cu (KM_RERANK_PCT).  Each
  // flushes its [k][d+1] table with global atomics, but fewer workgroups lose
  // more in parallelism than they save (c3 resolve 0.32-0.35 ms at 100%,
  // 0.48 at 50%, 0.80 at 25%)
  static const int rpct = diag_env("KM_RERANK_PCT", KM_RERANK_PCT);
  const int rwg = std::max(1, n_cu * std::max(1, rpct) / 100);
  // the re-rank's fp32 prefilter (KM_RR_PF, default on) where rows are <= 128 wide
  static const int rr_pf = diag_env("KM_RR_PF", 1);
  if (g.d > 256)
    hipLaunchKernelGGL(k_rerank2<true>, dim3(rwg), dim3(512), (tab_kp ? tab_bytes : 0) + pres, s, X, g.dp, g.d,
                       g.k, C64, queue, qcount, ql, labels, stats, tab_kp, sse, gate, cand, cand_cap, delta, sse_c32, chg,
                       chg_cnt, C32, cmax);
  else if (rr_pf && g.d <= 128 && C32 && cmax)
    hipLaunchKernelGGL((k_rerank2<false, true>), dim3(rwg), dim3(1024), (tab_kp ? tab_bytes : 0) + pres, s, X, g.dp,
                       g.d, g.k, C64, queue, qcount, ql, labels, stats, tab_kp, sse, gate, cand, cand_cap, delta, sse_c32,
                       chg, chg_cnt, C32, cmax);
  else
    hipLaunchKernelGGL(k_rerank2<false>, dim3(rwg), dim3(1024), (tab_kp ? tab_bytes : 0) + pres, s, X, g.dp, g.d,
                       g.k, C64, queue, qcount, ql, labels, stats, tab_kp, sse, gate, cand, cand_cap, delta, sse_c32, chg,
                       chg_cnt, C32, cmax);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Partial statistics (reduceByKey, kmeans_spark.py:169-173): per cluster
// sum of x and count, float64, into an LDS table; a workgroup owns a range of
// clusters (blockIdx.y) and a range of rows (blockIdx.x); a wave streams
// chunks of 64 contiguous rows as coalesced float4 loads (8 in flight per
// lane), labels broadcast from one coalesced load; one float64 global atomic
// per non-zero table entry at the end.
// ---------------------------------------------------------------------------
static constexpr int STATS_LDS = 156 * 1024;

// The workgroup also owns a feature range [f0, f0 + fr) (blockIdx.z):
// splitting the features instead of the clusters keeps X read once when
// k (d+1) doubles exceed LDS but k (fr+1) fit (c4: 1024 clusters x 16 features).
template <bool SSE = false>
__global__ __launch_bounds__(1024) void k_stats(const float* __restrict__ X, int64_t n, int d, int dp, int k,
                                                const int32_t* __restrict__ labels, double* __restrict__ stats,
                                                int kr, int fr, int64_t rows_per_block, const double* __restrict__ C64P,
                                                const float* __restrict__ C32, double* __restrict__ sse,
                                                const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  if constexpr (!SSE) sse = nullptr;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* tab = reinterpret_cast<double*>(smem);
  // LDS row of a cluster: fr feature slots + count.  Feature f0 + 4m + c is
  // stored at slot c*L + m (L = fr/4 lanes per row), so the 4 atomics of a
  // float4 each hit L consecutive doubles: no bank conflicts.
  const int RS = fr + 1;
  const int L = fr / 4;
  const int c0 = blockIdx.y * kr;
  const int c1 = min(k, c0 + kr);
  const int f0 = blockIdx.z * fr;
  const bool counts = blockIdx.z == 0;  // the count column reaches the global statistics from range 0 only
  const int nent = (c1 - c0) * RS;
  for (int i = threadIdx.x; i < nent; i += blockDim.x) tab[i] = 0.0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int P = 64 / L;        // rows per load instruction (L <= 64)
  const int q = lane / L;
  const int mm = lane % L;
  // L not dividing 64 (fr = 48, 96, 152, 196, ...): the lanes past the last
  // whole row idle (lane q = P would repeat row u + 1's first features)
  const bool act = q < P;
  constexpr int U = SSE ? 6 : 8;  // float4 rows in flight per lane (SSE: and as many centroid images)
  // SSE (compute_sse, kmeans_spark.py:224-237) in the same pass: each
  // (row, feature range) is summed by exactly one workgroup (the one owning
  // the row's cluster).  Per row it adds the float64 residual to the fp32
  // image c' of the pre-update centroid (C32, 16 B per 4 features gathered
  // from L2 instead of C64P's 32 B); at the flush it corrects to the float64
  // centroid c = c' + delta per cluster and feature, exactly in algebra:
  //   sum_rows (x - c)^2 = sum_rows (x - c')^2 - 2 delta (S - n c') + n delta^2
  // with S, n this workgroup's own partial sums and count (linear, so the
  // workgroups' corrections add up).  |delta| <= 2^-24 |c|, so the
  // correction's own rounding is ~2^-75 n |c|^2
  double ss = 0.0;
  for (int64_t cr = r0 + (int64_t)wave * 64; cr < r1; cr += (int64_t)nwaves * 64) {
    const int nrow = (int)min((int64_t)64, r1 - cr);
    const int labreg = lane < nrow ? labels[cr + lane] : -1;
    if ((counts || sse) && lane < nrow && labreg >= c0 && labreg < c1) atomicAdd(tab + (labreg - c0) * RS + fr, 1.0);
    const float* base = X + cr * dp + f0;
    for (int rb = 0; rb < nrow; rb += P * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = rb + u * P + q;
        v[u] = (act && rr < nrow) ? *reinterpret_cast<const float4*>(base + (size_t)rr * dp + 4 * mm)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      // the rows' labels, then (SSE) every row's centroid image gathered
      // before any is used: U L2 loads in flight instead of U dependent ones
      int labs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) labs[u] = __shfl(labreg, (rb + u * P + q) & 63);
      float4 cg[U];
      if (sse) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int rr = rb + u * P + q;
          const bool mine = act && rr < nrow && labs[u] >= c0 && labs[u] < c1;
          cg[u] = mine ? *reinterpret_cast<const float4*>(C32 + (size_t)labs[u] * dp + f0 + 4 * mm)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = rb + u * P + q;
        const int lab = labs[u];
        if (act && rr < nrow && lab >= c0 && lab < c1) {
          double* t = tab + (lab - c0) * RS + mm;
          atomicAdd(t, (double)v[u].x);
          atomicAdd(t + L, (double)v[u].y);
          atomicAdd(t + 2 * L, (double)v[u].z);
          atomicAdd(t + 3 * L, (double)v[u].w);
          if (sse) {  // padded features are 0 - 0
            const float4 c = cg[u];
            const double t0 = (double)v[u].x - (double)c.x, t1 = (double)v[u].y - (double)c.y;
            const double t2 = (double)v[u].z - (double)c.z, t3 = (double)v[u].w - (double)c.w;
            ss = fma(t0, t0, ss);
            ss = fma(t1, t1, ss);
            ss = fma(t2, t2, ss);
            ss = fma(t3, t3, ss);
          }
        }
      }
    }
  }
  __syncthreads();
  const int d1 = d + 1;
  for (int i = threadIdx.x; i < nent; i += blockDim.x) {
    const int j = i / RS;
    const int p = i - j * RS;
    const double v = tab[i];
    int f;
    if (p == fr) {
      if (!counts) continue;  // counts only from feature range 0
      f = d;
    } else {
      f = f0 + 4 * (p % L) + p / L;
      if (f >= d) continue;  // zero padding
      if (sse) {
        // delta (S - n c') and n delta^2 of this (cluster, feature); a zero
        // sum S still has a correction when n > 0
        const double n = tab[j * RS + fr];
        if (n != 0.0) {
          const double cp = (double)C32[(size_t)(c0 + j) * dp + f];
          const double dl = C64P[(size_t)(c0 + j) * dp + f] - cp;
          ss += dl * (n * dl - 2.0 * (v - n * cp));
        }
      }
    }
    if (v == 0.0) continue;
    atomicAdd(stats + (size_t)(c0 + j) * d1 + f, v);
  }
  if (sse) {
    ss = wave_sum(ss);
    if (lane == 0 && ss != 0.0) atomicAdd(sse, ss);
  }
}

// features per range: the widest (fewest blocks, longest row segments) among
// those needing the fewest cluster ranges; segments stay >= 64 bytes
static void stats_ranges(const Geometry& g, int* fr_out, int* kr_out) {
  int best_fr = g.dp, best_kr = 0, best_ncr = 1 << 30;
  if (g.dp > 256) {
    // wide rows: any multiple of 4 dividing dp, at most 256 (dp = 2000: 80)
    for (int fr = 256; fr >= 16; fr -= 4) {
      if (g.dp % fr) continue;
      int kr = (int)(STATS_LDS / ((size_t)(fr + 1) * 8));
      if (kr > g.k) kr = g.k;
      const int ncr = (g.k + kr - 1) / kr;
      if (ncr < best_ncr) {
        best_ncr = ncr;
        best_fr = fr;
        best_kr = kr;
      }
    }
    *fr_out = best_fr;
    *kr_out = best_kr;
    return;
  }
  for (int fr = g.dp; fr >= 16 && g.dp % fr == 0 && fr % 4 == 0; fr /= 2) {
    int kr = (int)(STATS_LDS / ((size_t)(fr + 1) * 8));
    if (kr > g.k) kr = g.k;
    const int ncr = (g.k + kr - 1) / kr;
    if (ncr < best_ncr) {
      best_ncr = ncr;
      best_fr = fr;
      best_kr = kr;
    }
    if (fr % 8) break;
  }
  *fr_out = best_fr;
  *kr_out = best_kr;
}

hipError_t launch_stats(const float* X, const Geometry& g, const int32_t* labels, double* stats, int n_cu,
                        const int* gate, hipStream_t s, const double* C64P, const float* C32) {
  if (g.n == 0) return hipSuccess;
  if (C64P && !C32) return hipErrorInvalidValue;
  if (g.dp > WIDE_MAX_DP || g.dp % 4) return hipErrorInvalidValue;
  int fr = 0, kr = 0;
  stats_ranges(g, &fr, &kr);
  if (kr < 1) return hipErrorInvalidValue;
  const int ranges = (g.k + kr - 1) / kr;
  const int franges = g.dp / fr;
  const size_t lds = (size_t)kr * (fr + 1) * 8;
  int per_cu = (int)((160 * 1024) / (lds + 1024));
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 2) per_cu = 2;
  int64_t bx = (int64_t)n_cu * per_cu / (ranges * franges);
  if (bx < 1) bx = 1;
  const int64_t min_rows = 4096;
  if (bx > (g.n + min_rows - 1) / min_rows) bx = (g.n + min_rows - 1) / min_rows;
  int64_t rpb = (g.n + bx - 1) / bx;
  rpb = (rpb + 63) / 64 * 64;
  if (C64P)
    hipLaunchKernelGGL((k_stats<true>), dim3((unsigned)bx, (unsigned)ranges, (unsigned)franges), dim3(1024), lds,
                       s, X, g.n, g.d, g.dp, g.k, labels, stats, kr, fr, rpb, C64P, C32,
                       stats + (size_t)g.k * (g.d + 1), gate);
  else
    hipLaunchKernelGGL((k_stats<false>), dim3((unsigned)bx, (unsigned)ranges, (unsigned)franges), dim3(1024),
                       lds, s, X, g.n, g.d, g.dp, g.k, labels, stats, kr, fr, rpb, C64P, C32, (double*)nullptr, gate);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Partial statistics for large k (k (d+1) doubles beyond LDS: c4, c5).  The
// range-tiled k_stats would re-read X once per LDS-sized cluster range (28x
// at k=4096, d=128); instead the labels are counting-sorted (histogram ->
// exclusive scan -> scatter of row ids) and each cluster's rows are summed in
// float64 by one workgroup with plain stores (no atomics): X is read once,
// as gathered whole rows.
// ---------------------------------------------------------------------------
// Wave aggregation of label atomics.  Where a few clusters hold most rows (poor
// seeds: c5_poor puts nearly all 50M rows in 3 clusters) one atomic per row
// serialises every wave on the same few words.  The wave peels the label of
// its first pending lane while that label is shared by at least two pending
// lanes (at most PEEL rounds): the lowest such lane becomes the leader and
// adds the group's size; every other lane adds 1 for itself.  All adds go out
// as ONE atomic instruction (leaders and singles together).  Returns, per
// lane, the count this lane adds (0: covered by its leader), the leader lane
// and the lane's rank within its group (lanes in lane order).  Distinct labels
// cost one ballot and stop the peeling at once.
struct Peel {
  uint32_t add;
  int leader;
  uint32_t rank;
};
template <int PEEL>
__device__ __forceinline__ Peel peel_labels(int l, bool valid) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  uint64_t pending = __ballot(valid);
  Peel p{0u, lane, 0u};
#pragma unroll
  for (int r = 0; r < PEEL; ++r) {
    if (pending == 0ull) break;
    const int first = __ffsll((unsigned long long)pending) - 1;
    const int lead = __shfl(l, first);
    const uint64_t mm = __ballot(valid && l == lead) & pending;
    if (__popcll(mm) < 2) break;  // wave-uniform
    if (lane == first) p.add = (uint32_t)__popcll(mm);
    if ((mm >> lane) & 1ull) {
      p.leader = first;
      p.rank = (uint32_t)__popcll(mm & below);
    }
    pending &= ~mm;
  }
  if ((pending >> lane) & 1ull) p.add = 1u;  // a lane of its own
  return p;
}

__global__ __launch_bounds__(1024) void k_hist(const int32_t* __restrict__ labels, int64_t n, int k,
                                               uint32_t* __restrict__ cnt, const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);
  for (int i = threadIdx.x; i < k; i += blockDim.x) hist[i] = 0u;
  __syncthreads();
  // wave-uniform trip count (every lane reaches the ballots of peel_labels)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); i0 < n; i0 += stride) {
    const int64_t i = i0 + (threadIdx.x & 63);
    const int l = i < n ? labels[i] : -1;
    const bool valid = (unsigned)l < (unsigned)k;
    const Peel p = peel_labels<4>(l, valid);
    if (p.add) atomicAdd(hist + l, p.add);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += blockDim.x)
    if (hist[i]) atomicAdd(cnt + i, hist[i]);
}

// exclusive scan of cnt[k] into off[k] and cur[k] (scatter cursors); one block
__global__ __launch_bounds__(1024) void k_scan(const uint32_t* __restrict__ cnt, int k, uint32_t* __restrict__ off,
                                               uint32_t* __restrict__ cur, const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  __shared__ uint32_t wsum[16];
  const int t = threadIdx.x;
  const int chunk = (k + 1023) / 1024;
  const int b0 = t * chunk;
  uint32_t v = 0;
  for (int i = 0; i < chunk; ++i)
    if (b0 + i < k) v += cnt[b0 + i];
  const int lane = t & 63, w = t >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t run = inc - v;
  for (int i = 0; i < w; ++i) run += wsum[i];
  for (int i = 0; i < chunk; ++i)
    if (b0 + i < k) {
      off[b0 + i] = run;
      cur[b0 + i] = run;
      run += cnt[b0 + i];
    }
}

// Scatter of row ids into label-sorted order.  A workgroup takes a contiguous
// chunk of SCAT_PER rows and aggregates before touching global memory: each
// row gets its rank among the chunk's rows of the same label from one LDS
// counter per label (returning LDS atomics, wave-aggregated by peel_labels),
// then ONE returning global cursor atomic per (chunk, label present) reserves
// that label's slots.  Where a few clusters hold most rows (c5_poor: ~3
// clusters of 50M rows) a per-row or per-wave global atomic serialises every
// wave of the chip on the same few words at the memory side.
static constexpr int SCAT_THREADS = 1024, SCAT_ROWS = 8;
static constexpr int SCAT_PER = SCAT_THREADS * SCAT_ROWS;  // rows per workgroup

__global__ __launch_bounds__(SCAT_THREADS) void k_scatter(const int32_t* __restrict__ labels, int64_t n, int k,
                                                          uint32_t* __restrict__ cur, uint32_t* __restrict__ perm,
                                                          int32_t* __restrict__ slab, const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);  // [k] chunk counts, then the chunk's base per label
  for (int i = threadIdx.x; i < k; i += SCAT_THREADS) cnt[i] = 0u;
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * SCAT_PER;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int lab[SCAT_ROWS];
  uint32_t rnk[SCAT_ROWS];
  // wave w takes rows c0 + (u * (SCAT_THREADS / 64) + w) * 64 + lane: each
  // wave-instruction reads 64 consecutive labels
#pragma unroll
  for (int u = 0; u < SCAT_ROWS; ++u) {
    const int64_t i = c0 + ((int64_t)(u * (SCAT_THREADS / 64) + wave) << 6) + lane;
    const int l = i < n ? labels[i] : -1;
    const bool valid = (unsigned)l < (unsigned)k;
    const Peel p = peel_labels<4>(l, valid);
    uint32_t base = 0u;
    if (p.add) base = atomicAdd(cnt + l, p.add);
    base = (uint32_t)__shfl((int)base, p.leader);
    lab[u] = valid ? l : -1;
    rnk[u] = base + p.rank;
  }
  __syncthreads();
  // one cursor atomic per label present in the chunk; the count becomes the
  // chunk's first slot of that label
  for (int j = threadIdx.x; j < k; j += SCAT_THREADS) {
    const uint32_t c = cnt[j];
    if (c) cnt[j] = atomicAdd(cur + j, c);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < SCAT_ROWS; ++u) {
    if (lab[u] < 0) continue;
    const int64_t i = c0 + ((int64_t)(u * (SCAT_THREADS / 64) + wave) << 6) + lane;
    const uint32_t pos = cnt[lab[u]] + rnk[u];
    perm[pos] = (uint32_t)i;
    slab[pos] = lab[u];
  }
}

// Segmented float64 sums over the label-sorted order: every wave takes an
// equal contiguous range of sorted positions; a lane group of L = dp/4 lanes
// owns one row per load (float4 per lane, 64/L rows per wave-instruction, U
// instructions in flight) and keeps a running float64 sum while its rows stay
// in one cluster, flushing it with global float64 atomics (contiguous 16 B
// per lane) when the cluster changes and at the end.  Counts come from the
// histogram.
// With C64P the SSE residuals ride along: the sorted order keeps a lane's
// centroid features constant over a run, so they are reloaded only when the
// cluster changes.
template <int L>  // lanes per row = dp / 4
__global__ __launch_bounds__(256) void k_segsum(const float* __restrict__ X, int d, int64_t n,
                                                const uint32_t* __restrict__ perm, const int32_t* __restrict__ slab,
                                                double* __restrict__ stats, const double* __restrict__ C64P,
                                                double* __restrict__ sse, const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  constexpr int P = 64 / L;  // rows per wave-instruction
  constexpr int U = 4;       // instructions in flight
  constexpr int DP = 4 * L;
  const int lane = threadIdx.x & 63;
  const int q = lane / L;
  const int m = lane % L;
  const bool act = q < P;  // dp = 48, 96, 192: the lanes past the last whole row idle
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t per = (n + nw - 1) / nw;
  const int64_t p0 = gw * per;
  const int64_t p1 = p0 + per < n ? p0 + per : n;
  const int d1 = d + 1;
  int cur = -1;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0, ss = 0.0;
  auto flush = [&]() {
    if (cur >= 0) {
      double* o = stats + (size_t)cur * d1 + 4 * m;
      if (4 * m + 0 < d) atomicAdd(o + 0, a0);
      if (4 * m + 1 < d) atomicAdd(o + 1, a1);
      if (4 * m + 2 < d) atomicAdd(o + 2, a2);
      if (4 * m + 3 < d) atomicAdd(o + 3, a3);
    }
    a0 = a1 = a2 = a3 = 0.0;
  };
  for (int64_t base = p0; act && base < p1; base += P * U) {
    float4 v[U];
    int lb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t pos = base + u * P + q;
      if (pos < p1) {
        const uint32_t row = perm[pos];
        lb[u] = slab[pos];
        v[u] = *reinterpret_cast<const float4*>(X + (size_t)row * DP + 4 * m);
      } else {
        lb[u] = -1;
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (lb[u] < 0) continue;
      if (lb[u] != cur) {
        flush();
        cur = lb[u];
        if (C64P) {
          const double2 ca = *reinterpret_cast<const double2*>(C64P + (size_t)cur * DP + 4 * m);
          const double2 cb = *reinterpret_cast<const double2*>(C64P + (size_t)cur * DP + 4 * m + 2);
          c0 = ca.x;
          c1 = ca.y;
          c2 = cb.x;
          c3 = cb.y;
        }
      }
      a0 += (double)v[u].x;
      a1 += (double)v[u].y;
      a2 += (double)v[u].z;
      a3 += (double)v[u].w;
      if (C64P) {  // padded features are 0 - 0
        const double t0 = (double)v[u].x - c0, t1 = (double)v[u].y - c1;
        const double t2 = (double)v[u].z - c2, t3 = (double)v[u].w - c3;
        ss = fma(t0, t0, ss);
        ss = fma(t1, t1, ss);
        ss = fma(t2, t2, ss);
        ss = fma(t3, t3, ss);
      }
    }
  }
  if (act) flush();
  if (C64P) {
    ss = wave_sum(ss);
    if (lane == 0 && ss != 0.0) atomicAdd(sse, ss);
  }
}

// counts of the histogram into the count column
__global__ void k_put_counts(const uint32_t* __restrict__ cnt, int k, int d, double* __restrict__ stats, const int* __restrict__ gate) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < k) stats[(size_t)j * (d + 1) + d] = (double)cnt[j];
}

size_t sorted_stats_words(int64_t n, int k) { return 2 * (size_t)n + 3 * (size_t)k + 64; }

// the range-tiled k_stats reads X once per LDS-sized cluster range; from three
// ranges on, the sort (one gathered read of X plus ~5 bytes per row of
// label/permutation traffic, and cursor atomics that contend when k is small)
// is cheaper
bool stats_needs_sort(const Geometry& g) {
  static const int min_ranges = diag_env("KM_SORT_MIN_RANGES", 3);  // A/B knob
  if (g.dp > 256) return false;  // k_segsum holds a row in one wave-instruction
  int fr = 0, kr = 0;
  stats_ranges(g, &fr, &kr);
  return kr == 0 || (g.k + kr - 1) / kr >= min_ranges;
}

hipError_t launch_stats_sorted(const float* X, const Geometry& g, const int32_t* labels, double* stats,
                               uint32_t* scratch, const double* C64P, int n_cu, const int* gate, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  if (g.dp > 256) return hipErrorInvalidValue;
  uint32_t* cnt = scratch;
  uint32_t* off = cnt + g.k;
  uint32_t* cur = off + g.k;
  uint32_t* perm = cur + g.k;
  hipError_t e = hipMemsetAsync(cnt, 0, sizeof(uint32_t) * g.k, s);
  if (e != hipSuccess) return e;
  int64_t hb = (g.n + 1023) / 1024;
  if (hb > n_cu * 2) hb = n_cu * 2;
  const size_t hist_lds = (size_t)g.k * 4;
  if (hist_lds > 64 * 1024) return hipErrorInvalidValue;  // k <= 16384
  hipLaunchKernelGGL(k_hist, dim3((unsigned)hb), dim3(1024), hist_lds, s, labels, g.n, g.k, cnt, gate);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, cnt, g.k, off, cur, gate);
  const int64_t sb = (g.n + SCAT_PER - 1) / SCAT_PER;
  if (sb > 0x7fffffff) return hipErrorInvalidValue;
  int32_t* slab = reinterpret_cast<int32_t*>(perm + g.n);
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)sb), dim3(SCAT_THREADS), (size_t)g.k * 4, s, labels, g.n, g.k, cur,
                     perm, slab, gate);
  hipLaunchKernelGGL(k_put_counts, dim3((g.k + 255) / 256), dim3(256), 0, s, cnt, g.k, g.d, stats, gate);
  // every label is in [0, k) (the assign kernels map non-finite rows to 0),
  // so all n sorted positions are written
  const int64_t nsorted = g.n;
  int64_t wb = (int64_t)n_cu * 8;
  const unsigned grid = (unsigned)wb;
  switch (g.dp / 4) {
    case 4: hipLaunchKernelGGL(k_segsum<4>, dim3(grid), dim3(256), 0, s, X, g.d, nsorted, perm, slab, stats, C64P, stats + (size_t)g.k * (g.d + 1), gate); break;
    case 8: hipLaunchKernelGGL(k_segsum<8>, dim3(grid), dim3(256), 0, s, X, g.d, nsorted, perm, slab, stats, C64P, stats + (size_t)g.k * (g.d + 1), gate); break;
    case 12: hipLaunchKernelGGL(k_segsum<12>, dim3(grid), dim3(256), 0, s, X, g.d, nsorted, perm, slab, stats, C64P, stats + (size_t)g.k * (g.d + 1), gate); break;
    case 16: hipLaunchKernelGGL(k_segsum<16>, dim3(grid), dim3(256), 0, s, X, g.d, nsorted, perm, slab, stats, C64P, stats + (size_t)g.k * (g.d + 1), gate); break;
    case 24: hipLaunchKernelGGL(k_segsum<24>, dim3(grid), dim3(256), 0, s, X, g.d, nsorted, perm, slab, stats, C64P, stats + (size_t)g.k * (g.d + 1), gate); break;
    case 32: hipLaunchKernelGGL(k_segsum<32>, dim3(grid), dim3(256), 0, s, X, g.d, nsorted, perm, slab, stats, C64P, stats + (size_t)g.k * (g.d + 1), gate); break;
    case 48: hipLaunchKernelGGL(k_segsum<48>, dim3(grid), dim3(256), 0, s, X, g.d, nsorted, perm, slab, stats, C64P, stats + (size_t)g.k * (g.d + 1), gate); break;
    case 64: hipLaunchKernelGGL(k_segsum<64>, dim3(grid), dim3(256), 0, s, X, g.d, nsorted, perm, slab, stats, C64P, stats + (size_t)g.k * (g.d + 1), gate); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Centroid update (kmeans_spark.py:176-206 + 278-294): new = sum / count,
// empties keep the old centroid (host replaces them, L191-204), per-cluster
// squared shift.  The SSE (L224-237) is the all-reduced residual slot
// stats[k (d+1)] filled by the assign / statistics passes.
// ---------------------------------------------------------------------------
// SSE correction (corr: the residuals in the SSE slot were taken to the fp32
// image c' = (float) c of each centroid -- k_s1's delta fit with compute_sse):
// per cluster sum ||x - c||^2 - sum ||x - c'||^2 = sum_f dl_f (n dl_f -
// 2 (S_f - n c'_f)), dl = c - c', exact as an identity; its rounding is
// ~2^-53 of the term, which is ~2^-24 of the cluster's share (DESIGN.md
// section 2 "Statistics and SSE").  Returns the lane's share.
__device__ __forceinline__ double sse_corr_term(double o, double S, double cnt) {
  const double cp = (double)(float)o;
  const double dl = o - cp;
  return dl * fma(cnt, dl, -2.0 * fma(-cnt, cp, S));
}

__global__ __launch_bounds__(64) void k_update(const double* __restrict__ stats, const double* __restrict__ old,
                                               int k, int d, double* __restrict__ out, double* __restrict__ work,
                                               int64_t* __restrict__ counts, const int* __restrict__ gate, int corr) {
  if (*gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  const int j = blockIdx.x;
  const int lane = threadIdx.x;
  const int d1 = d + 1;
  const double cnt = stats[(size_t)j * d1 + d];
  double sh = 0.0, nf = 0.0, cr = 0.0;
  for (int f = lane; f < d; f += 64) {
    const double S = stats[(size_t)j * d1 + f];
    const double o = old[(size_t)j * d + f];
    const double nv = (cnt > 0.0) ? S / cnt : o;
    out[(size_t)j * d + f] = nv;
    const double df = nv - o;
    sh = fma(df, df, sh);
    if (!isfinite(nv)) nf = 1.0;
    if (corr) cr += sse_corr_term(o, S, cnt);
  }
  sh = wave_sum(sh);
  nf = wave_sum(nf);
  if (corr) cr = wave_sum(cr);
  if (lane == 0) {
    work[j] = sh;
    work[k + j] = cr;
    work[2 * k + j] = nf;
    counts[j] = (int64_t)cnt;
  }
}

// Per-iteration status into *st (one history slot per iteration of a batch,
// km_update_async).  In a batch (stop_tol >= 0) the gate is raised, and the
// remaining enqueued iterations become no-ops, when the iteration converged
// (max_shift < tol, kmeans_spark.py:310), produced empty clusters (the host
// repairs them, L191-204) or non-finite centroids (L289); a gated launch only
// records that the iteration did not run.
__global__ __launch_bounds__(256) void k_finalize(const double* __restrict__ work, const int64_t* __restrict__ counts,
                                                  int k, const double* __restrict__ sse,
                                                  const uint32_t* __restrict__ qcount, uint32_t nq,
                                                  DevStatus* __restrict__ st, int* __restrict__ gate, double stop_tol, int dev_repair,
                                                  int corr) {
  if (*gate) {
    if (threadIdx.x == 0) {
      st->ran = 0;
      st->stop = 0;
    }
    return;
  }
  __shared__ double s_max[256], s_cr[256];
  __shared__ int s_emp[256], s_nf[256], s_q[256], s_qf[256];
  double mx = 0.0, cr = 0.0;
  int emp = 0, nf = 0, qa = 0, qb = 0;
  for (uint32_t w = threadIdx.x; w < nq; w += 256) {
    qa += (int)qcount[2 * w];
    qb += (int)qcount[2 * w + 1];
  }
  s_q[threadIdx.x] = qa;
  s_qf[threadIdx.x] = qb;
  for (int j = threadIdx.x; j < k; j += 256) {
    mx = fmax(mx, work[j]);
    nf |= (work[2 * k + j] != 0.0);
    emp += (counts[j] == 0);
    if (corr) cr += work[k + j];
  }
  s_max[threadIdx.x] = mx;
  s_cr[threadIdx.x] = cr;
  s_emp[threadIdx.x] = emp;
  s_nf[threadIdx.x] = nf;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      s_max[threadIdx.x] = fmax(s_max[threadIdx.x], s_max[threadIdx.x + o]);
      s_cr[threadIdx.x] += s_cr[threadIdx.x + o];
      s_emp[threadIdx.x] += s_emp[threadIdx.x + o];
      s_nf[threadIdx.x] |= s_nf[threadIdx.x + o];
      s_q[threadIdx.x] += s_q[threadIdx.x + o];
      s_qf[threadIdx.x] += s_qf[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double ms = sqrt(s_max[0]);
    st->max_shift = ms;
    st->sse = corr ? *sse + s_cr[0] : *sse;
    st->n_empty = s_emp[0];
    st->nonfinite = s_nf[0];
    st->q_full = s_qf[0];
    st->q_rerank = s_q[0];
    st->ran = 1;
    int stop = 0;
    if (stop_tol >= 0.0) {
      if (s_nf[0])
        stop = KM_STOP_NONFINITE;
      else if (s_emp[0])
        stop = dev_repair ? 0 : KM_STOP_EMPTY;  // repaired next, which then decides
      else if (ms < stop_tol)
        stop = KM_STOP_CONVERGED;
    }
    st->repaired = 0;
    st->stop = stop;
    if (stop) *gate = stop;
  }
}

// k_update + k_finalize in one workgroup for small k (c1 / c2 shapes, where
// the two launches are mostly launch gaps): same arithmetic and
// reduction order per cluster (lanes over features, wave sums), then the
// status record and the batch gate as k_finalize.  In a batch it also ends
// the iteration's other small launches: `clear` zeroes the statistics it
// consumed (the next assign accumulates into them; no memset launch), and
// with C32 it writes the small path's images of the new centroids -- the
// fp32 copy and max ||c||, exactly as k_prep_small (same per-lane fma order
// over f < dp, same wave sums) -- so the next assign needs no prep launch.
// the one-workgroup update (blockDim.x <= 1024): k_update_one, and the last
// workgroup of k_assign_small when the update is folded into the assign
// launch (COHERENT: the statistics were summed by other workgroups of the same
// launch; read at device scope)
template <bool COHERENT>
__device__ void update_one_body(double* __restrict__ stats, const double* __restrict__ old, int k, int d,
                                double* __restrict__ out, int64_t* __restrict__ counts, const double* __restrict__ sse,
                                const uint32_t* __restrict__ qcount, uint32_t nq, DevStatus* __restrict__ st,
                                int* __restrict__ gate, double stop_tol, int dev_repair, int clear,
                                float* __restrict__ C32, float* __restrict__ cmax, int dp, int kp, int corr) {
  auto ld = [](const double* p) {
    if constexpr (COHERENT)
      return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      return *p;
  };
  __shared__ double s_max[16], s_cr[16];
  __shared__ int s_emp[16], s_nf[16], s_q[16], s_qf[16];
  __shared__ unsigned int s_cm[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int d1 = d + 1;
  double mx = 0.0, crs = 0.0;
  int emp = 0, nf = 0, qa = 0, qb = 0;
  unsigned int cmb = 0u;  // max ||c|| bits (k_prep_small)
  for (int j = wave; j < k; j += nw) {
    const double cnt = ld(stats + (size_t)j * d1 + d);
    double sh = 0.0, nfl = 0.0, nn = 0.0, cr = 0.0;
    for (int f = lane; f < (C32 ? dp : d); f += 64) {
      if (f < d) {
        const double S = ld(stats + (size_t)j * d1 + f);
        const double o = old[(size_t)j * d + f];
        const double nv = (cnt > 0.0) ? S / cnt : o;
        out[(size_t)j * d + f] = nv;
        const double df = nv - o;
        sh = fma(df, df, sh);
        if (!isfinite(nv)) nfl = 1.0;
        if (corr) cr += sse_corr_term(o, S, cnt);
        if (C32) {
          nn = fma(nv, nv, nn);
          C32[(size_t)j * dp + f] = (float)nv;
        }
      } else {
        nn = fma(0.0, 0.0, nn);
        C32[(size_t)j * dp + f] = 0.0f;
      }
    }
    sh = wave_sum(sh);
    nfl = wave_sum(nfl);
    if (C32) nn = wave_sum(nn);
    if (corr) cr = wave_sum(cr);
    if (lane == 0) {
      crs += cr;
      counts[j] = (int64_t)cnt;
      mx = fmax(mx, sh);
      nf |= (nfl != 0.0);
      emp += (cnt == 0.0);
      if (C32) cmb = max(cmb, __float_as_uint(sqrtf((float)nn) * 1.0001f + 1e-30f));
    }
  }
  if (C32)  // padded rows k <= j < kp stay zero (as k_prep_small writes them)
    for (int i = threadIdx.x; i < (kp - k) * dp; i += blockDim.x) C32[(size_t)k * dp + i] = 0.0f;
  for (uint32_t w = threadIdx.x; w < nq; w += blockDim.x) {
    qa += (int)qcount[2 * w];
    qb += (int)qcount[2 * w + 1];
  }
  for (int o = 32; o >= 1; o >>= 1) {
    qa += __shfl_xor(qa, o);
    qb += __shfl_xor(qb, o);
  }
  if (lane == 0) {
    s_max[wave] = mx;
    s_cr[wave] = crs;
    s_emp[wave] = emp;
    s_nf[wave] = nf;
    s_q[wave] = qa;
    s_qf[wave] = qb;
    s_cm[wave] = cmb;
  }
  __syncthreads();
  const double sse_v = ld(sse);
  __syncthreads();  // every read of the statistics is done
  if (clear)
    for (int i = threadIdx.x; i < k * d1 + 1; i += blockDim.x) stats[i] = 0.0;
  if (threadIdx.x == 0) {
    for (int w = 1; w < nw; ++w) {
      crs += s_cr[w];
      mx = fmax(mx, s_max[w]);
      emp += s_emp[w];
      nf |= s_nf[w];
      qa += s_q[w];
      qb += s_qf[w];
      cmb = max(cmb, s_cm[w]);
    }
    if (C32) *cmax = __uint_as_float(cmb);
    const double ms = sqrt(mx);
    st->max_shift = ms;
    st->sse = corr ? sse_v + crs : sse_v;
    st->n_empty = emp;
    st->nonfinite = nf;
    st->q_full = qb;
    st->q_rerank = qa;
    st->ran = 1;
    int stop = 0;
    if (stop_tol >= 0.0) {
      if (nf)
        stop = KM_STOP_NONFINITE;
      else if (emp)
        stop = dev_repair ? 0 : KM_STOP_EMPTY;  // repaired next, which then decides
      else if (ms < stop_tol)
        stop = KM_STOP_CONVERGED;
    }
    st->repaired = 0;
    st->stop = stop;
    if (stop) *gate = stop;
  }
}

__global__ __launch_bounds__(1024) void k_update_one(double* __restrict__ stats, const double* __restrict__ old,
                                                     int k, int d, double* __restrict__ out,
                                                     int64_t* __restrict__ counts, const double* __restrict__ sse,
                                                     const uint32_t* __restrict__ qcount, uint32_t nq,
                                                     DevStatus* __restrict__ st, int* __restrict__ gate,
                                                     double stop_tol, int dev_repair, int clear, float* __restrict__ C32,
                                                     float* __restrict__ cmax, int dp, int kp, int corr) {
  if (*gate) {
    if (threadIdx.x == 0) {
      st->ran = 0;
      st->stop = 0;
    }
    return;
  }
  update_one_body<false>(stats, old, k, d, out, counts, sse, qcount, nq, st, gate, stop_tol, dev_repair, clear, C32,
                         cmax, dp, kp, corr);
}

bool update_one_ok(const Geometry& g) { return g.k <= 64 && (size_t)g.k * g.d <= 16384; }

hipError_t launch_update(double* stats, const double* C64_old, const Geometry& g, double* C64_new,
                         double* work, int64_t* counts, const uint32_t* qcount, uint32_t nq, DevStatus* status,
                         int* gate, double stop_tol, int dev_repair, hipStream_t s, int clear, float* C32,
                         float* cmax, int corr) {
  if (update_one_ok(g)) {  // at most 4 clusters per wave (c3: 2 launches, 11 vs 37 us)
    hipLaunchKernelGGL(k_update_one, dim3(1), dim3(1024), 0, s, stats, C64_old, g.k, g.d, C64_new, counts,
                       stats + (size_t)g.k * (g.d + 1), qcount, nq, status, gate, stop_tol, dev_repair, clear, C32,
                       cmax, g.dp, g.kp, corr);
    return hipGetLastError();
  }
  if (clear || C32) return hipErrorInvalidValue;  // only the one-workgroup update clears / prepares
  hipLaunchKernelGGL(k_update, dim3(g.k), dim3(64), 0, s, stats, C64_old, g.k, g.d, C64_new, work, counts, gate,
                     corr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(256), 0, s, work, counts, g.k, stats + (size_t)g.k * (g.d + 1),
                     qcount, nq, status, gate, stop_tol, dev_repair, corr);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Data moment (checks): sum_p x_p, float64.
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

hipError_t launch_sum_x(const float* X, const Geometry& g, double* out, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  int64_t blocks = (g.n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_sum_x, dim3((unsigned)blocks), dim3(256), 0, s, X, g.n, g.d, g.dp, out);
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

// Empty-cluster repair from the host (several ranks): rows[i] -> C[ids[i]]
// in one launch
__global__ void k_scatter_rows(const int64_t* __restrict__ ids, const double* __restrict__ rows, int32_t n, int d,
                               double* __restrict__ C) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n * d) return;
  const int i = (int)(t / d);
  const int f = (int)(t % d);
  C[ids[i] * d + f] = rows[t];
}

hipError_t launch_scatter_rows(const int64_t* ids, const double* rows, int32_t n, int d, double* C, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t tot = (int64_t)n * d;
  hipLaunchKernelGGL(k_scatter_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, ids, rows, n, d, C);
  return hipGetLastError();
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
