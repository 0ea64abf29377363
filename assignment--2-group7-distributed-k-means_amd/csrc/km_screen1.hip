// One-MFMA screen with in-kernel exact re-scoring (the c3 class: kp * dp <=
// 16384, dp a multiple of 32).  DESIGN.md section 2, "One-MFMA screen".
//
// Reference: kmeans_spark.py:147-159 (assign_partition: np.argmin of
// np.linalg.norm(C - x, axis=1)) and :169-173 (reduceByKey of (x, 1)).
//
// Why a new kernel: the fp16x3 screen (k_fused16) issues three f16 MFMAs per
// product and holds its 256-register images at one wave per SIMD; its tile
// body (split, merges, sums) cannot overlap the MFMAs, and the chip holds its
// clock down under the MFMA density.  Here:
//   * one v_mfma_f32_16x16x32_f16 per product: image RN16(-2 s c) (32 KB of
//     LDS at c3, read as A fragments one block pair ahead) times the row
//     RN16(s x).  Its error is large (E ~ 5 in squared distance units at c3),
//     so the screen only proposes candidates;
//   * every row whose screen cannot settle it (about 12% at c3) has its
//     candidates re-scored exactly in fp32 direct form ||x - c'||^2 from an
//     LDS copy of the fp32 centroids, with a rigorous error bound; only
//     near-ties of the candidates (1e-6 relative) go to the float64 resolvers;
//   * 16-row tiles, two waves per SIMD (512-thread workgroups), rows
//     double-buffered in registers: one wave's VALU work hides under the
//     other's MFMAs and loads;
//   * statistics: either none (predict) or DELTAS -- a row whose label did not
//     change since the last iteration adds nothing; a changed row is appended
//     to its wave's segment of a change list (row, old, new; no atomics: a
//     wave's segment holds every row it can visit, the wave writes its count
//     at the end), and k_s1_delta moves its x from the
//     old cluster's float64 sums to the new one's through an LDS table per
//     workgroup.  The runtime keeps the full sums (km_runtime.hip, "delta
//     statistics"), so the sums the update reads are the reference's
//     reduceByKey sums over every row, exactly as a fresh pass would produce
//     them up to float64 summation order.
//
// Candidate certificate (all bounds rigorous, real arithmetic on the float64
// centroids c; c' = fp32 image):
//   * chains: the output layout gives each lane 8 accumulator positions per
//     block of 32 centroids; position (cb, i) over the NB blocks is a chain
//     (32 chains per row, NB members).  Each lane keeps the chain's best two
//     keys (v_min3 / v_med3 over block pairs, 5 VALU per two keys, the block
//     id in the low mantissa bits of every key).
//   * a greedy colouring (k_s1_color) puts mutually distant centroids in one
//     chain, so that two members of a chain are rarely both close to a row.
//   * keys K~ = s^2(||c||^2 - 2 c.x) + e, |e| <= E(x) (k_s1_prep's bound).
//     m = the smallest head; every centroid whose key exceeds m + 2E (+ the
//     packing perturbation) is strictly farther than the argmin.  The heads
//     below that threshold T are the candidates; a chain whose second key is
//     below T too (a member that is neither head nor excluded) sends the row
//     to the full float64 scan.
//   * one candidate: it is the argmin.  Otherwise each candidate is
//     re-scored, D~ = fp32 sum of (x - c')^2, |D~ - D'| <= 36u D', and
//     ||x - c|| in [sqrt(D'(1-48u)) - g, sqrt(D'(1+48u)) + g], g = u cmax.
//     The winner must beat every other candidate's lower bound strictly;
//     otherwise the row is queued (kind 1: the two candidates re-ranked in
//     float64 by k_rerank2; kind 2: full float64 scan by k_fullscan).
#include <float.h>

#include "km_internal.h"

namespace km {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

constexpr float U24 = 5.9604644775390625e-08f;  // 2^-24
constexpr float U16 = 4.8828125e-04f;           // 2^-11, fp16 unit roundoff
#ifndef KM_S1_LMAX  // A/B knob: 3, 4, 5 lost or tied (profiles/r6_c3_s1_lmax_ab.json)
#define KM_S1_LMAX 8
#endif
constexpr int S1_LMAX = KM_S1_LMAX;             // candidates re-scored per row (more: the full scan)
#ifndef KM_S1_NBUF
#define KM_S1_NBUF 0  // register buffers of rows (tiles in flight + 1); 0: by row length
#endif
#ifndef KM_S1_ABL
#define KM_S1_ABL 0  // timing ablations (wrong labels): alt builds for A/B only, never the product
#endif
constexpr int ceil_log2_c(int v) { return v <= 1 ? 0 : 1 + ceil_log2_c((v + 1) / 2); }
// waves per workgroup (one workgroup per CU): three per SIMD on the c3
// geometry (dp 64, kp 256), whose kernel is latency-bound at two (DESIGN.md
// section 4), two elsewhere; KM_S1_W12=0 keeps two everywhere (A/B arm)
#ifndef KM_S1_W12
#define KM_S1_W12 1
#endif
#ifndef KM_S1_W12_C4  // the same on the c4 geometry (dp 32, kp 1024)
#define KM_S1_W12_C4 1
#endif
constexpr int s1_waves(int ns2, int nb) {
  return ((KM_S1_W12 && ns2 == 2 && nb == 8) || (KM_S1_W12_C4 && ns2 == 1 && nb == 32)) ? 12 : 8;
}

constexpr int S1_MAX_WAVES = 12;                // per CU, any geometry (change-list counts)
// rows per re-scoring batch (one per quad of a wave): 16, or 12 where twelve
// waves' rings must fit beside the image and the fp32 table
constexpr int s1_ring(int ns2, int nb) { return s1_waves(ns2, nb) == 12 ? 12 : 16; }

// the re-scoring batches run where a wave's ring (S1_RING rows of DP floats,
// 16 B of row data and 128 B of chain heads) fits beside the tables: dp <= 64
constexpr bool s1_batched(int ns2) { return ns2 <= 2; }
// tiles of 16 rows per wave step (A/B knob for 32-wide rows: two tiles per
// step lost at c4 on one box, 230 vs 159-169 ms)
#ifndef KM_S1_SERP  // serpentine sweeps of the delta fit on the (2, 8) geometry (c3 class; km_runtime next_sweep)
#define KM_S1_SERP 1
#endif
#ifndef KM_S1_TT
#define KM_S1_TT 1
#endif
constexpr int s1_tiles(int ns2) { return ns2 == 1 ? KM_S1_TT : 1; }

// k_s1's LDS: image, fp32 table (unless it goes to global), norms, slots,
// re-scoring rings; the table goes to global memory where all of it would
// not fit one workgroup's 160 KiB
constexpr size_t s1_lds_bytes(int ns2, int nb, bool table) {
  const int dp = 32 * ns2, kp = 32 * nb, nt = 32 << ceil_log2_c(nb);
  return (size_t)kp * dp * 2 + (table ? (size_t)nt * (dp + 4) * 4 : 0) + (size_t)kp * 4 + (size_t)nt * 4 +
         (s1_batched(ns2) ? (size_t)s1_waves(ns2, nb) * s1_ring(ns2, nb) * (dp * 4 + 16 + 128) : 0);
}
constexpr bool s1_table_global(int ns2, int nb) { return s1_lds_bytes(ns2, nb, true) > 160 * 1024; }


__device__ __forceinline__ uint32_t f2u(float v) { return __float_as_uint(v); }
__device__ __forceinline__ float u2f(uint32_t v) { return __uint_as_float(v); }

// minima of keys and heads without the IEEE-mode canonicalisation hipcc puts
// in front of fminf for values made by bit operations (packed keys, lane
// swaps, selects): every such value is finite here or its row is caught as
// non-finite by the certificate (`bad`: the row-norm bound is NaN / inf), and
// v_min / v_min3 order finite values exactly.  VALU results feeding VALU
// only (never an MFMA operand: DESIGN.md section 2, inline asm and MFMA)
__device__ __forceinline__ float min_raw(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float min3_raw(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// the four quarter lanes of a row (l, l ^ 16, l ^ 32, l ^ 48): min / sum
__device__ __forceinline__ float quad_min(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(f2u(v), f2u(v), false, false);
  v = min_raw(u2f(p[0]), u2f(p[1]));
  p = __builtin_amdgcn_permlane32_swap(f2u(v), f2u(v), false, false);
  return min_raw(u2f(p[0]), u2f(p[1]));
}
// the same order of additions in all four lanes ((l0 + l16) + (l32 + l48)):
// every lane of the row holds the bit-identical sum
__device__ __forceinline__ float quad_sum(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(f2u(v), f2u(v), false, false);
  v = u2f(p[0]) + u2f(p[1]);
  p = __builtin_amdgcn_permlane32_swap(f2u(v), f2u(v), false, false);
  return u2f(p[0]) + u2f(p[1]);
}
__device__ __forceinline__ int32_t quad_min_i(int32_t v) {
  auto p = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
  v = min((int32_t)p[0], (int32_t)p[1]);
  p = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
  return min((int32_t)p[0], (int32_t)p[1]);
}
// float bits -> int32 with the same order (distinct bits stay distinct, -0 < +0);
// its own inverse
__device__ __forceinline__ int32_t mono(uint32_t b) { return (int32_t)(b ^ ((uint32_t)((int32_t)b >> 31) >> 1)); }
__device__ __forceinline__ uint32_t unmono(int32_t v) { return (uint32_t)v ^ ((uint32_t)(v >> 31) >> 1); }
__device__ __forceinline__ uint32_t quad_add_u(uint32_t v) {
  auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = p[0] + p[1];
  p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return p[0] + p[1];
}

__device__ __forceinline__ float s1_scale(float xabs, float cabs) {
  // power-of-two scale: max(|x|, |c|) * s < 2^14 (km_kernels.hip mfma_scale)
  const float m = fmaxf(xabs, cabs);
  if (!(m > 0.0f) || !(m < 3.0e38f)) return 1.0f;
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.0f, 14 - e);
}

}  // namespace

// table index of chain c, member b: (c << MB) | b
struct S1Geo {
  int nb, mb, ns2;
};

// ---------------------------------------------------------------------------
// Greedy colouring of the centroids into 32 chains of nb members (one
// workgroup).  In index order, centroid j joins the non-full chain whose
// members are farthest from it (largest minimum distance; ties: lowest
// chain).  perm[(chain << mb) | member] = centroid, -1 for pads.  Only a
// cost choice: the certificate (a chain whose second key is under the
// threshold sends its row to the full scan) holds for any colouring, so a
// stale or poor one (it is recomputed once per batch) can queue rows, never
// mislabel them.
// ---------------------------------------------------------------------------
template <int DPC, int NTH>
__global__ __launch_bounds__(NTH) void k_s1_color(const float* __restrict__ C32, int k, int dp, int nb, int mb,
                                                  int32_t* __restrict__ perm, const int* __restrict__ gate) {
  if (*gate) return;
  __shared__ unsigned int cmin[32];
  __shared__ int cnt[32];
  __shared__ int cls[NTH];
  const int t = threadIdx.x;
  float cv[DPC];
#pragma unroll
  for (int f = 0; f < DPC; ++f) cv[f] = (t < k && f < dp) ? C32[(size_t)t * dp + f] : 0.0f;
  if (t < 32) cnt[t] = 0;
  cls[t] = -1;
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    if (t < 32) cmin[t] = 0x7F800000u;  // +inf
    __syncthreads();
    if (t < j) {
      float s = 0.0f;
#pragma unroll
      for (int f = 0; f < DPC; ++f) {
        const float df = cv[f] - C32[(size_t)j * dp + f];
        s = fmaf(df, df, s);
      }
      atomicMin(&cmin[cls[t]], __float_as_uint(s));
    }
    __syncthreads();
    if (t < 64) {
      // (eligible, distance bits, lowest chain) maximum over the 32 chains
      uint64_t key = 0;
      if (t < 32 && cnt[t] < nb) key = ((uint64_t)(cmin[t] + 1u) << 8) | (uint64_t)(31 - t);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t other = __shfl_xor(key, o);
        key = other > key ? other : key;
      }
      if (t == 0) {
        const int c = 31 - (int)(key & 255u);
        const int m = cnt[c];
        cls[j] = c;
        cnt[c] = m + 1;
        perm[(c << mb) | m] = j;
      }
    }
    __syncthreads();
  }
  // pads: members cnt[c] .. (1 << mb) - 1 of every chain
  for (int i = t; i < (32 << mb); i += blockDim.x) {
    const int c = i >> mb, m = i & ((1 << mb) - 1);
    if (m >= cnt[c]) perm[i] = -1;
  }
}

// ---------------------------------------------------------------------------
// Per-iteration images of the current centroids in the colouring's order.
// Blocks 0 .. (32 << mb) - 1: table index ti = (chain << mb) | member:
//   cft[ti][f]  fp32 centroid (row stride dp + 4: the LDS copy's bank spread)
//   cn2o[p]     s^2 ||c||^2 (float64 norm, rounded once; pads 1e30) at the
//               MFMA output position p = 32 member + 16 (chain >> 4) + (chain & 15)
//   img         fragment-linear A operands RN16(-2 s c') of v_mfma_f32_16x16x32_f16:
//               fragment (member, cb, t), lane l = 16 q + M holds centroid
//               chain 16 cb + M, features fq q + 8 t .. + 8 (fq = dp / 4)
// Last block: bound constants.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_s1_prep(const double* __restrict__ C64, const float* __restrict__ C32, int k,
                                                int d, int dp, S1Geo sg, const int32_t* __restrict__ perm,
                                                const float* __restrict__ cmax, const float* __restrict__ xabs,
                                                const float* __restrict__ cabs, float* __restrict__ cft,
                                                float* __restrict__ cn2o, uint4* __restrict__ img,
                                                float* __restrict__ cst,
                                                const int* __restrict__ gate) {
  if (*gate) return;
  const int b = blockIdx.x, th = threadIdx.x;
  const int nt = 32 << sg.mb;
  const float s = s1_scale(*xabs, *cabs);
  const int cs = dp + 4;
  if (b < nt) {
    const int chain = b >> sg.mb, member = b & ((1 << sg.mb) - 1);
    const int j = member < sg.nb ? perm[b] : -1;
    for (int f = th; f < cs; f += 64) cft[(size_t)b * cs + f] = (j >= 0 && f < d) ? C32[(size_t)j * dp + f] : 0.0f;
    if (member >= sg.nb) return;
    const int cb = chain >> 4, M = chain & 15;
    if (th == 0) {
      double nn = 0.0;
      if (j >= 0)
        for (int f = 0; f < d; ++f) nn = fma(C64[(size_t)j * d + f], C64[(size_t)j * d + f], nn);
      cn2o[32 * member + 16 * cb + M] = j >= 0 ? (float)(nn * (double)s * (double)s) : 1e30f;
    }
    const int fq = dp / 4;
    if (th < 4 * sg.ns2) {
      const int q = th / sg.ns2, t = th - q * sg.ns2;
      f16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int f = fq * q + 8 * t + e;
        v[e] = (j >= 0 && f < d) ? (_Float16)(-2.0f * s * C32[(size_t)j * dp + f]) : (_Float16)0.0f;
      }
      img[((size_t)(member * 2 + cb) * sg.ns2 + t) * 64 + 16 * q + M] = __builtin_bit_cast(uint4, v);
    }
    return;
  }
  if (th == 0) {
    // screen error bound E = e1 ||x|| + e0 in scaled units (||x|| unscaled),
    // see the header and DESIGN.md "One-MFMA screen": image and row rounding
    // (fp16, the image of the fp32 c' whose own rounding adds u), the fp32
    // rounding of s^2 ||c||^2, the 16x16x32 accumulation model (per MFMA 4
    // roundings of a partial sum and 28 u of the largest product; ns2 MFMAs
    // per key), fp16 underflow; times 1.25
    const float cm = *cmax, ca = *cabs * (1.0f + U24), xa = *xabs;
    const float s2 = s * s, sq = sqrtf((float)dp) * 1.0001f, nm = (float)sg.ns2;
    const float e1 = 1.25f * (2.0f * s2 * cm * (2.0f * U16 + U16 * U16 + 2.0f * U24) +
                              nm * 4.0f * U24 * 2.0f * s2 * cm * (1.0f + 2.0f * U16) +
                              ldexpf(1.0f, -25) * s * sq * (1.0f + U16));
    const float e0 = 1.25f * (U24 * s2 * cm * cm + nm * (4.0f * U24 * s2 * cm * cm +
                                                          28.0f * U24 * 2.0f * s2 * ca * xa * (1.0f + U16) * (1.0f + U16)) +
                              ldexpf(1.0f, -24) * s * sq * cm);
    cst[0] = s;
    cst[1] = e1 * 1.0001f;
    cst[2] = e0 * 1.0001f + 1e-30f;
    cst[3] = U24 * cm * 1.01f + 1e-37f;  // g: ||c - c'|| <= u ||c||
  }
}

struct S1Args {
  const float* X;
  const float* xnorm;  // per-row upper bound of ||x|| (unscaled)
  int64_t n;
  int k, d;
  uint32_t seg;
  const uint4* img;
  const float* cn2o;
  const float* cft;
  const int32_t* perm;
  const float* cst;
  int32_t* labels;
  QEntry* queue;
  uint32_t* qcount;
  uint2* chg;          // DELTA: changed rows {row, old << 16 | new}, [wave][seg]
  uint32_t* chg_cnt;   // DELTA: entries per wave segment
  double* sse;         // SSE (MODE 1): every decided row's residual to the fp32 image c' of its centroid
  const int* gate;
};

// MODE 0: labels only (predict; every decided row's label written, queued
// rows' by the resolvers).  MODE 1: delta statistics (the previous labels are
// read; only changed labels are written and moved in the sums; queued rows
// keep their previous label for the resolvers to compare).
// SSE (MODE 1 only, compute_sse with delta statistics): every row the kernel
// decides adds sum_f (x_f - c'_f)^2 in float64 (fp32 x and c' are exact in
// float64) for c' = the fp32 image of its centroid, from the table it
// re-scores with; the resolvers add the queued rows' the same way
// (launch_resolve sse_c32), and the update turns the total into
// sum ||x - c||^2 with one exact per-cluster correction from the full sums
// (k_update, sse_corr; DESIGN.md section 2 "Statistics and SSE").
template <int NS2, int NB, int MODE, bool REV = false, bool SSE = false>
__global__ __launch_bounds__(s1_waves(NS2, NB) * 64, s1_waves(NS2, NB) / 4) void k_s1(S1Args A) {
  if (*A.gate) return;  // a stopped batch (km_update_async): the rest of it is a no-op
  constexpr int S1_WAVES = s1_waves(NS2, NB);
  constexpr int S1_RING = s1_ring(NS2, NB);
  constexpr int DP = 32 * NS2;
  constexpr int FQ = 8 * NS2;  // features per quarter lane
  constexpr int KP = 32 * NB;
  constexpr int MB = ceil_log2_c(NB);
  constexpr int NT = 32 << MB;      // table entries
  constexpr int CS = DP + 4;        // LDS row stride of the fp32 centroids (floats)
  constexpr uint32_t SLOTM = (uint32_t)NT - 1u;
  constexpr uint32_t KMASK = ~SLOTM;
  // key packing perturbation: the low 5 + MB mantissa bits replaced
  constexpr float RHO = (float)SLOTM * 1.1920928955078125e-07f * 1.0001f;
  // the fp32 table stays in global memory (L2) where it does not fit LDS
  // beside the image (s1_lds_bytes)
  constexpr bool BATCH = s1_batched(NS2);
  constexpr bool TG = s1_table_global(NS2, NB);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint4* sImg = reinterpret_cast<const uint4*>(smem);    // [NB][2][NS2][64] A fragments
  float* sCf = reinterpret_cast<float*>(smem + KP * DP * 2);  // [NT][CS] (not with TG)
  float* sCn = sCf + (TG ? 0 : NT * CS);                      // [KP] output order
  int32_t* sPerm = reinterpret_cast<int32_t*>(sCn + KP);      // [NT]
  // per wave: the re-scoring ring, rows' x [S1_RING][DP], {row, old | cnt
  // << 16, s0 | s1 << 16, second head} and the 32 chain heads [4 lanes][8]
  float* sRx = reinterpret_cast<float*>(sPerm + NT);                   // [S1_WAVES][S1_RING][DP]
  uint4* sRm = reinterpret_cast<uint4*>(sRx + S1_WAVES * S1_RING * DP);  // [S1_WAVES][S1_RING]
  float4* sRh = reinterpret_cast<float4*>(sRm + S1_WAVES * S1_RING);     // [S1_WAVES][S1_RING][4][2]

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c16 = lane & 15;
  const int q = lane >> 4;
  {
    uint4* di = reinterpret_cast<uint4*>(smem);
    for (int i = threadIdx.x; i < KP * DP / 8; i += S1_WAVES * 64) di[i] = A.img[i];
    if constexpr (!TG) {
      const float4* src = reinterpret_cast<const float4*>(A.cft);
      float4* dst = reinterpret_cast<float4*>(sCf);
      for (int i = threadIdx.x; i < NT * CS / 4; i += S1_WAVES * 64) dst[i] = src[i];
    }
    for (int i = threadIdx.x; i < KP; i += S1_WAVES * 64) sCn[i] = A.cn2o[i];
    for (int i = threadIdx.x; i < NT; i += S1_WAVES * 64) sPerm[i] = A.perm[i];
  }
  __syncthreads();

  const float s = A.cst[0], e1 = A.cst[1], e0 = A.cst[2], gam = A.cst[3];
  // rows fit 32 bits (km_load_begin: n < 2^32 - 1): 32-bit row and tile arithmetic
  const uint32_t n = (uint32_t)A.n;
  const uint32_t ntiles = (n + 15u) / 16u;
  const uint32_t gw = blockIdx.x * S1_WAVES + wave;
  const uint32_t nw = gridDim.x * S1_WAVES;
  QEntry* wq = A.queue + (size_t)gw * A.seg;
  uint2* wc = A.chg + (size_t)gw * A.seg;
  uint32_t qn = 0, qf = 0, cc = 0;
  double ssa = 0.0;  // SSE: this lane's share of its decided rows' residuals
  // SSE: the lane's features of a decided row against table slot `slot`
  auto resid = [&](bool act, uint32_t slot, const float4* xv) {
    if constexpr (SSE) {
      const uint32_t sl = act ? slot : 0u;
      const float4* cp = TG ? reinterpret_cast<const float4*>(A.cft + sl * CS + FQ * q)
                            : reinterpret_cast<const float4*>(sCf + sl * CS + FQ * q);
      double r = 0.0;
#pragma unroll
      for (int u = 0; u < FQ / 4; ++u) {
        const float4 c = cp[u];
        const float4 x = xv[u];
        const double e0 = (double)x.x - (double)c.x, e1 = (double)x.y - (double)c.y;
        const double e2 = (double)x.z - (double)c.z, e3 = (double)x.w - (double)c.w;
        r = fma(e0, e0, r);
        r = fma(e1, e1, r);
        r = fma(e2, e2, r);
        r = fma(e3, e3, r);
      }
      ssa += act ? r : 0.0;
    } else {
      (void)act;
      (void)slot;
      (void)xv;
    }
  };
  // chain id bits of this lane's 8 accumulator positions (cb, i): chain 16 cb + 4 q + i
  const uint32_t qbits = (uint32_t)(4 * q) << MB;

  struct Buf {
    float4 x[FQ / 4];
    float xn;
    int32_t old;
  };
  // serpentine sweep (REV: its own instance, since a run-time select in the
  // row arithmetic cost the issue-bound c3 kernel 1.5%): step tiles mapped
  // last-first; tiles past the end stay past the end
  auto tmap = [&](uint32_t t) { return (REV && t < ntiles) ? ntiles - 1u - t : t; };
  auto load = [&](uint32_t tile, Buf& B) {
    const uint32_t row = tmap(tile) * 16u + (uint32_t)c16;
    const uint32_t rr = row < n ? row : (n - 1u);
    const float4* xr = reinterpret_cast<const float4*>(A.X + (size_t)rr * DP + FQ * q);
#pragma unroll
    for (int u = 0; u < FQ / 4; ++u) B.x[u] = xr[u];
    B.xn = A.xnorm[rr];
    if constexpr (MODE == 1) B.old = A.labels[rr];
  };

  // fp32 re-score of candidates (slots sl[0..cnt-1], ascending key order)
  // from the fp32 table: the winner by the smallest upper bound, decided when
  // every other candidate's lower bound is above it; a near tie of exactly
  // two candidates goes to the float64 pair re-rank (kind 1), anything else
  // to the full scan (kind 2).  Bounds of ||x - c|| (unscaled):
  // |Dt - D'| <= (FQ + 4) u D' <= 36 u D' (D' = ||x - c'||^2, FQ <= 32), so
  // sqrt(D') is within 18.1 u of sqrt(Dt); v_sqrt_f32 (within 2 ulp = 4 u
  // taken here) gives r, sqrt(D') = r (1 +- 23 u), widened to 32 u; then
  // ||x - c|| = sqrt(D') +- g, the fma and product: 4 u.  Below 2^-96 the
  // hardware sqrt loses accuracy: U takes sqrt(2^-96) (an over-estimate), L
  // takes 0 (an under-estimate)
  auto decide = [&](bool act0, uint32_t cnt, const uint32_t* sl, const float4* xv, int32_t& lab1, int32_t& lab2,
                    uint32_t& kind, uint32_t& ws) {
    auto partial = [&](uint32_t slot) {
      const float4* cp = TG ? reinterpret_cast<const float4*>(A.cft + slot * CS + FQ * q)
                            : reinterpret_cast<const float4*>(sCf + slot * CS + FQ * q);
      // two packed chains (v_pk_add_f32 / v_pk_fma_f32 on feature pairs):
      // each square and difference rounded once, FQ / 2 + 1 roundings per
      // chain -- inside the re-score bound's (FQ + 4) u
      f32x2 acc = {0.0f, 0.0f};
#pragma unroll
      for (int u = 0; u < FQ / 4; ++u) {
        const float4 c = cp[u];
        const float4 x = xv[u];
        const f32x2 d0 = f32x2{x.x, x.y} - f32x2{c.x, c.y};
        const f32x2 d1 = f32x2{x.z, x.w} - f32x2{c.z, c.w};
        acc = __builtin_elementwise_fma(d0, d0, acc);
        acc = __builtin_elementwise_fma(d1, d1, acc);
      }
      return acc.x + acc.y;
    };
    // winner (smallest upper bound U1, its lower bound L1, slot s1) and the
    // smallest lower bound of the others (Lo, slot s2), select form
    // throughout (branchy running minima are
    // miscompiled in divergent code on this toolchain)
    uint32_t s1 = sl[0], s2 = sl[0];
    float U1 = FLT_MAX, L1 = FLT_MAX, Lo = FLT_MAX;
    auto take = [&](bool act, float Dt, uint32_t slot) {
      const bool tiny = !(Dt >= 0x1p-96f);
      const float r = __builtin_amdgcn_sqrtf(tiny ? 0x1p-96f : Dt);
      const float U = fmaf(r, 1.0f + 32.0f * U24, gam) * (1.0f + 4.0f * U24);
      const float L = fmaf(tiny ? 0.0f : r, 1.0f - 32.0f * U24, -gam) * (1.0f - 4.0f * U24);
      const bool w = act && U < U1;              // new winner
      const float Lc = w ? L1 : L;               // the displaced winner, or this one, joins the others
      const uint32_t sc = w ? s1 : slot;
      const bool lo = act && Lc < Lo;
      Lo = lo ? Lc : Lo;
      s2 = lo ? sc : s2;
      U1 = w ? U : U1;
      L1 = w ? L : L1;
      s1 = w ? slot : s1;
    };
    // the first two (every row here has them) in one round: both tables'
    // reads in flight together; inactive lanes read slot 0 and ignore it
    {
      const uint32_t sa = act0 ? sl[0] : 0u, sb = act0 ? sl[1] : 0u;
      const float pa = partial(sa), pb = partial(sb);
      take(act0, quad_sum(pa), sa);
      take(act0, quad_sum(pb), sb);
    }
#pragma unroll
    for (int r = 2; r < S1_LMAX; ++r) {
      const bool act = act0 && (uint32_t)r < cnt;
      if (__ballot(act) == 0ull) break;
      const uint32_t slot = act ? sl[r] : 0u;
      take(act, quad_sum(partial(slot)), slot);
    }
    const int32_t l1 = sPerm[s1], l2 = sPerm[s2];
    uint32_t kd = 2u;
    if (l1 >= 0) {
      if (Lo > U1)
        kd = 0u;
      else if (cnt == 2u && l2 >= 0)
        kd = 1u;
    }
    if (act0) {
      lab1 = l1;
      lab2 = l2;
      kind = kd;
      ws = s1;  // the winner's table slot (SSE residual)
    }
  };
  // a row's outcome (every lane of its quad calls with the same values):
  // decided (kind 0) -> its label (MODE 1: only a changed one, appended to
  // the wave's change list); kind 1 / 2 -> the queue, pair re-ranks from the
  // front of the wave's segment, full scans from the back (k_fused16's
  // layout, read by launch_resolve)
  auto emit = [&](bool act, uint32_t row, uint32_t kind, int32_t lab1, int32_t lab2, int32_t old) {
    const bool decided = act && kind == 0u;
    if constexpr (MODE == 0) {
      (void)old;
      if (decided && q == 0) A.labels[row] = lab1;
    } else {
      const bool changed = decided && lab1 != old && q == 0;  // one lane per row
      const uint64_t mc = __ballot(changed);
      if (mc) {
        if (changed) {
          A.labels[row] = lab1;
          wc[cc + (uint32_t)__popcll(mc & ((1ull << lane) - 1ull))] =
              make_uint2(row, ((uint32_t)old << 16) | (uint32_t)lab1);
        }
        cc += (uint32_t)__popcll(mc);
      }
    }
    const bool enq = act && kind != 0u && q == 0;
    const uint64_t mq = __ballot(enq);
    if (mq) {
      const uint64_t m1 = __ballot(enq && kind == 1u);
      const uint64_t m2 = mq & ~m1;
      const uint64_t below = (1ull << lane) - 1ull;
      if (enq) {
        QEntry qe;
        qe.row = row;
        qe.i1 = kind == 1u ? (uint32_t)lab1 : 0u;
        qe.i2 = kind == 1u ? (uint32_t)lab2 : 0u;
        qe.kind = kind;
        const uint32_t pos = (kind == 1u) ? qn + (uint32_t)__popcll(m1 & below)
                                          : A.seg - 1u - (qf + (uint32_t)__popcll(m2 & below));
        wq[pos] = qe;
      }
      qn += (uint32_t)__popcll(m1);
      qf += (uint32_t)__popcll(m2);
    }
  };
  // the first nb rows of the wave's ring, one per quad: re-scored, emitted
  uint32_t rc = 0;  // rows in the ring (< S1_RING between tiles)
  auto rescore = [&](uint32_t nb) {
    if constexpr (BATCH) {
      const bool act = (uint32_t)c16 < nb;
      const uint32_t slot = act ? (uint32_t)c16 : 0u;
      const uint4 mt = sRm[wave * S1_RING + slot];
      float4 xv[FQ / 4];
      const float4* xs = reinterpret_cast<const float4*>(sRx + (wave * S1_RING + slot) * DP + FQ * q);
#pragma unroll
      for (int u = 0; u < FQ / 4; ++u) xv[u] = xs[u];
      const uint32_t cnt = mt.y >> 16;
      uint32_t sl[S1_LMAX];
      sl[0] = mt.z;
#pragma unroll
      for (int r = 1; r < S1_LMAX; ++r) sl[r] = 0u;
      {
        // candidates 2, 3, ...: the row's smallest heads above the first
        // (every row here has at least two)
        const float4* hp = sRh + ((wave * S1_RING + slot) * 4 + q) * 2;
        const float4 h0 = hp[0], h1 = hp[1];
        const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        float prev = u2f(mt.w);
#pragma unroll
        for (int r = 1; r < S1_LMAX; ++r) {
          if (__ballot(act && (uint32_t)r < cnt) == 0ull) break;
          float nl = FLT_MAX;
#pragma unroll
          for (int i = 0; i < 8; ++i) nl = min_raw(nl, hv[i] > prev ? hv[i] : FLT_MAX);
          prev = quad_min(nl);
          sl[r] = (uint32_t)r < cnt ? (f2u(prev) & SLOTM) : 0u;
        }
      }
      int32_t lab1 = 0, lab2 = 0;
      uint32_t kind = 2u, ws = 0u;
      decide(act, cnt, sl, xv, lab1, lab2, kind, ws);
      emit(act, mt.x, kind, lab1, lab2, (int32_t)(mt.y & 0xFFFFu));
      resid(act && kind == 0u, ws, xv);
    } else {
      (void)nb;
    }
  };

  // everything after the chains of one tile: certificate, labels, queue,
  // re-scoring ring
  auto tail = [&](uint32_t tile, const Buf& B, const float (&h)[2][4], float h2m) {
    const uint32_t row = tmap(tile) * 16u + (uint32_t)c16;
    const bool valid = row < n;
    // full slot ids in the heads, (chain << MB) | member: distinct keys, so
    // float comparisons order them totally (f32 denormals are kept, and +0
    // and -0 could only share a slot); non-finite rows are caught by `bad`
    float hk[2][4];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) hk[cb][i] = u2f(f2u(h[cb][i]) | qbits | ((uint32_t)(16 * cb + i) << MB));
    // h2m: the smallest second key of the lane's chains (an open chain: <= T)

    // the row's smallest head m, then the candidate threshold T (the
    // batched re-score finds the other candidates from the stored heads; the
    // in-tile one of dp > 64 takes the second smallest head here: the lane's
    // lowest two, med3 keeping the middle of a sorted pair and a new value,
    // merged over the quad)
    auto mn = [](float a, float b) { return __builtin_fminf(a, b); };
    auto mx = [](float a, float b) { return __builtin_fmaxf(a, b); };
    float la = FLT_MAX, lb = FLT_MAX;
    if constexpr (BATCH) {
      la = min3_raw(min3_raw(hk[0][0], hk[0][1], hk[0][2]), min3_raw(hk[0][3], hk[1][0], hk[1][1]),
                    min3_raw(hk[1][2], hk[1][3], FLT_MAX));
      la = quad_min(la);
    } else {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          lb = __builtin_amdgcn_fmed3f(la, lb, hk[cb][i]);  // (la <= lb)
          la = mn(la, hk[cb][i]);
        }
      auto p = __builtin_amdgcn_permlane16_swap(f2u(la), f2u(la), false, false);
      auto p2 = __builtin_amdgcn_permlane16_swap(f2u(lb), f2u(lb), false, false);
      float a0 = u2f(p[0]), a1 = u2f(p[1]), b0 = u2f(p2[0]), b1 = u2f(p2[1]);
      la = mn(a0, a1);
      lb = mn(mx(a0, a1), mn(b0, b1));
      p = __builtin_amdgcn_permlane32_swap(f2u(la), f2u(la), false, false);
      p2 = __builtin_amdgcn_permlane32_swap(f2u(lb), f2u(lb), false, false);
      a0 = u2f(p[0]), a1 = u2f(p[1]), b0 = u2f(p2[0]), b1 = u2f(p2[1]);
      la = mn(a0, a1);
      lb = mn(mx(a0, a1), mn(b0, b1));
    }
    const float m = la;
#if KM_S1_ABL == 1
    // timing ablation (diagnostic builds only, wrong labels): the screen core
    if (valid && q == 0) A.labels[row] = sPerm[f2u(la) & SLOTM] + (h2m < -1e30f ? 1 : 0);
    return;
#endif
    const float xn = B.xn;
    const float E = fmaf(e1, xn, e0);
    const bool bad = !(m >= -3.0e38f && m <= 3.0e38f) || !(xn <= 3.0e38f);
    constexpr float RP = RHO * (1.0f + 2.0f * RHO);
    const float R = m + RP * fabsf(m) + 2.0f * E;
    // R / (1 -+ RP) by multiplication: the reciprocals rounded away from
    // T's side by 2u, the products' roundings inside the final 4u
    constexpr float IP = (1.0f / (1.0f - RP)) * (1.0f + 2.0f * U24);
    constexpr float IM = (1.0f / (1.0f + RP)) * (1.0f - 2.0f * U24);
    float T = R * (R >= 0.0f ? IP : IM);
    T = T * (T >= 0.0f ? (1.0f + 4.0f * U24) : (1.0f - 4.0f * U24));
    // candidates: heads <= T (low 16 bits of the quad sum); a chain whose
    // second key is <= T too (high 16 bits: the row goes to the full scan)
    uint32_t cl = (h2m <= T) ? 0x10000u : 0u;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) cl += (hk[cb][i] <= T) ? 1u : 0u;
    const uint32_t cq = bad ? 0u : quad_add_u(cl);
    const uint32_t cnt = cq & 0xFFFFu;
    const bool ovf = (cq >> 16) != 0u;

    const uint32_t sm = f2u(la) & SLOTM;
    const bool ok = valid && !bad && !ovf;
    const bool needy = ok && cnt >= 2u && cnt <= (uint32_t)S1_LMAX;
    const int32_t labm = sPerm[sm];
    // one candidate: the screen decides; none / too many / an open chain /
    // non-finite input: the full scan (kind 2)
    const bool dec1 = ok && cnt == 1u && labm >= 0;
    int32_t old = 0;
    if constexpr (MODE == 1) old = (int32_t)min((uint32_t)B.old, (uint32_t)(A.k - 1));
#if KM_S1_ABL == 2
    // timing ablation (diagnostic builds only, wrong labels): no re-scoring
    emit(valid, row, dec1 || needy ? 0u : 2u, labm, 0, old);
    return;
#endif
    if constexpr (BATCH) {
      emit(valid && !needy, row, dec1 ? 0u : 2u, labm, 0, old);
      resid(dec1, sm, B.x);
      // rows with 2..LMAX candidates: into the wave's ring with their
      // smallest head and every chain head, from which the batch extracts the
      // rest; a full ring is re-scored as one batch
      const uint64_t mrow = __ballot(needy && q == 0);
      if (mrow) {
        const uint32_t nn = (uint32_t)__popcll(mrow);
        const uint32_t rk = (uint32_t)__popcll(mrow & ((1ull << c16) - 1ull));
        const uint32_t space = (uint32_t)S1_RING - rc;
        const uint4 meta = make_uint4(row, (uint32_t)old | (cnt << 16), sm, f2u(la));
        auto stash = [&](uint32_t slot) {
          float4* xs = reinterpret_cast<float4*>(sRx + (wave * S1_RING + slot) * DP + FQ * q);
#pragma unroll
          for (int u = 0; u < FQ / 4; ++u) xs[u] = B.x[u];
          if (q == 0) sRm[wave * S1_RING + slot] = meta;
          // the chain heads: the batch extracts candidates 2, 3, ... from them
          float4* hp = sRh + ((wave * S1_RING + slot) * 4 + q) * 2;
          hp[0] = make_float4(hk[0][0], hk[0][1], hk[0][2], hk[0][3]);
          hp[1] = make_float4(hk[1][0], hk[1][1], hk[1][2], hk[1][3]);
        };
        if (needy && rk < space) stash(rc + rk);
        if (nn >= space) {
          rescore((uint32_t)S1_RING);
          if (needy && rk >= space) stash(rk - space);
          rc = nn - space;
        } else {
          rc += nn;
        }
      }
    } else {
      // dp > 64: the candidates re-scored in the tile, every row of it
      uint32_t sl[S1_LMAX];
      sl[0] = sm;
      sl[1] = f2u(lb) & SLOTM;
      float prev = lb;
#pragma unroll
      for (int r = 2; r < S1_LMAX; ++r) {
        sl[r] = 0u;
        if (__ballot(needy && (uint32_t)r < cnt) == 0ull) continue;
        float nl = FLT_MAX;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) nl = min_raw(nl, hk[cb][i] > prev ? hk[cb][i] : FLT_MAX);
        prev = quad_min(nl);
        sl[r] = f2u(prev) & SLOTM;
      }
      int32_t lab1 = labm, lab2 = 0;
      uint32_t kind = dec1 ? 0u : 2u, ws = sm;
      if (__ballot(needy) != 0ull) decide(needy, cnt, sl, B.x, lab1, lab2, kind, ws);
      emit(valid, row, kind, lab1, lab2, old);
      resid(valid && kind == 0u, ws, B.x);
    }
  };

  // TT tiles of 16 rows per wave step (two where rows are 32 wide: the
  // block pairs' image reads and their latency are shared by twice the rows)
  constexpr int TT = s1_tiles(NS2);
  auto process = [&](uint32_t st, const Buf (&BB)[TT]) {
    // B operands: RN16(s x), features FQ q + 8 t .. + 8 of slice t
    f16x8 bx[TT][NS2];
#pragma unroll
    for (int u = 0; u < TT; ++u)
#pragma unroll
      for (int t = 0; t < NS2; ++t) {
        // packed: four v_pk_mul_f32 and four v_cvt_pk_f16_f32 (round to
        // nearest even) per eight features, halves in feature order
        const float4 a = BB[u].x[2 * t], c = BB[u].x[2 * t + 1];
        const f32x2 sv = {s, s};
        const f16x2 h0 = __builtin_convertvector(f32x2{a.x, a.y} * sv, f16x2);
        const f16x2 h1 = __builtin_convertvector(f32x2{a.z, a.w} * sv, f16x2);
        const f16x2 h2 = __builtin_convertvector(f32x2{c.x, c.y} * sv, f16x2);
        const f16x2 h3 = __builtin_convertvector(f32x2{c.z, c.w} * sv, f16x2);
        bx[u][t] = __builtin_shufflevector(__builtin_shufflevector(h0, h1, 0, 1, 2, 3),
                                           __builtin_shufflevector(h2, h3, 0, 1, 2, 3), 0, 1, 2, 3, 4, 5, 6, 7);
      }
    // this lane's 8 chains per tile: best key (head, member id in the low MB
    // bits); and the smallest SECOND key over the lane's chains (h2m): the
    // certificate only asks whether any chain's second key is under the
    // threshold, i.e. min over chains of min over updates of
    // med3(head, ka, kb), so one running minimum per tile replaces eight
    // per-chain ones (fewer registers, half the minimum operations)
    float h[TT][2][4], h2m[TT];
#pragma unroll
    for (int u = 0; u < TT; ++u) {
      h2m[u] = FLT_MAX;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) h[u][cb][i] = FLT_MAX;
    }
    const float4* cnl = reinterpret_cast<const float4*>(sCn + 4 * q);  // + 8 blk + 4 cb
    // a block pair's operands from LDS: A fragments (lane-linear 1 KiB
    // pieces, conflict-free) and accumulator inits
    struct Pair {
      f16x8 a[2][2][NS2];  // [block of the pair][cb][t]
      float4 c[2][2];      // [block of the pair][cb]
    };
    auto load_pair = [&](int blk, Pair& P) {
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          P.c[e][cb] = cnl[8 * (blk + e) + 4 * cb];
#pragma unroll
          for (int t = 0; t < NS2; ++t)
            P.a[e][cb][t] = __builtin_bit_cast(f16x8, sImg[(((blk + e) * 2 + cb) * NS2 + t) * 64 + lane]);
        }
    };
    // the MFMAs of a block pair (two members of every chain)
    auto mfmas = [&](const Pair& P, f32x4 (&a)[TT][2][2]) {
#pragma unroll
      for (int u = 0; u < TT; ++u)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
            a[u][e][cb] = f32x4{P.c[e][cb].x, P.c[e][cb].y, P.c[e][cb].z, P.c[e][cb].w};
#pragma unroll
      for (int t = 0; t < NS2; ++t)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int u = 0; u < TT; ++u)
              a[u][e][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(P.a[e][cb][t], bx[u][t], a[u][e][cb], 0, 0, 0);
    };
    // their keys: new head = min3(head, ka, kb), second-key minimum
    // h2m = min(h2m, med3(head, ka, kb)) over the chains
    auto keys = [&](int blk, const f32x4 (&a)[TT][2][2]) {
#pragma unroll
      for (int u = 0; u < TT; ++u) {
        float t[2][4];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float ka = u2f((f2u(a[u][0][cb][i]) & KMASK) | (uint32_t)blk);
            const float kb = u2f((f2u(a[u][1][cb][i]) & KMASK) | (uint32_t)(blk + 1));
            t[cb][i] = __builtin_amdgcn_fmed3f(h[u][cb][i], ka, kb);
            h[u][cb][i] = __builtin_fminf(__builtin_fminf(h[u][cb][i], ka), kb);
          }
        // (a chain of v_min3: two values per operation)
        float m = h2m[u];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          m = __builtin_fminf(__builtin_fminf(m, t[cb][0]), t[cb][1]);
          m = __builtin_fminf(__builtin_fminf(m, t[cb][2]), t[cb][3]);
        }
        h2m[u] = m;
      }
    };
    // keep the key state computed where it is (the compiler would otherwise
    // sink the second-key updates into the certificate's branch and hold
    // every key of the tile alive until then)
    auto pin = [&]() {
#pragma unroll
      for (int u = 0; u < TT; ++u) {
        asm volatile("" : "+v"(h2m[u]));
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(h[u][cb][i]));
      }
    };
    if constexpr (NB <= 8 && s1_waves(NS2, NB) == 12) {
      // three waves per SIMD (<= 168 registers): ONE pair of operands in
      // registers -- the MFMAs of a pair read it, then it is refilled with
      // the next pair's while this pair's keys are updated (round 6 A/B on
      // one box, profiles/r6_c3_s1_waves_ab.json: 7.81-7.84 ms against
      // 7.90-7.94 at two waves per SIMD with two operand sets, 7.89 with the
      // MFMAs of pair p beside the keys of pair p - 1, 8.04-8.11 with the
      // keys interleaved between the MFMAs by sched_group_barrier)
      Pair P;
      load_pair(0, P);
#pragma unroll
      for (int blk = 0; blk < NB; blk += 2) {
        f32x4 a[TT][2][2];
        mfmas(P, a);
        __builtin_amdgcn_sched_barrier(0);
        if (blk + 2 < NB) load_pair(blk + 2, P);
        __builtin_amdgcn_sched_barrier(0);
        keys(blk, a);
        pin();
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (NB <= 8) {
      // one block pair in flight plus the next one's operands: the partner
      // wave on the SIMD fills the MFMA pipe while this one updates its keys
      Pair pr[2];
      load_pair(0, pr[0]);
#pragma unroll
      for (int blk = 0; blk < NB; blk += 2) {
        const Pair& P = pr[(blk >> 1) & 1];
        if (blk + 2 < NB) load_pair(blk + 2, pr[((blk >> 1) + 1) & 1]);
        f32x4 a[TT][2][2];
        mfmas(P, a);
        keys(blk, a);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      // many members (NB a multiple of 4): two pairs per trip of a loop, the
      // member id a run-time value
      static_assert(NB % 4 == 0, "NB > 8 must be a multiple of 4");
      Pair pr[2];
      load_pair(0, pr[0]);
#pragma unroll 1
      for (int blk = 0; blk < NB; blk += 4) {
        f32x4 a[TT][2][2];
        load_pair(blk + 2, pr[1]);
        mfmas(pr[0], a);
        keys(blk, a);
        __builtin_amdgcn_sched_barrier(0);
        if (blk + 4 < NB) load_pair(blk + 4, pr[0]);
        mfmas(pr[1], a);
        keys(blk + 2, a);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int u = 0; u < TT; ++u) tail(st * TT + (uint32_t)u, BB[u], h[u], h2m[u]);
  };

  // this wave's steps gw, gw + nw, ... of TT tiles each; NBUF register
  // buffers of rows: NBUF - 1 steps' loads in flight while one is processed
  // (loads past the end read row n - 1 and are never used)
  constexpr int NBUF = KM_S1_NBUF > 0 ? KM_S1_NBUF : (NS2 == 1 && NB > 8 && S1_WAVES == 8 ? 3 : 2);
  const uint32_t nst = (ntiles + (uint32_t)TT - 1u) / (uint32_t)TT;
  Buf b[NBUF][TT];
  auto load_step = [&](uint32_t st, Buf (&BB)[TT]) {
#pragma unroll
    for (int u = 0; u < TT; ++u) load(st * TT + (uint32_t)u, BB[u]);
  };
#pragma unroll
  for (int u = 0; u + 1 < NBUF; ++u) load_step(gw + (uint32_t)u * nw, b[u]);
  // (st + 2 NBUF nw stays below 2^32: ntiles < 2^28, nw < 2^16)
  for (uint32_t st = gw; st < nst; st += (uint32_t)NBUF * nw) {
    bool done = false;
#pragma unroll
    for (int u = 0; u < NBUF; ++u) {
      if (!done) {
        load_step(st + (uint32_t)(u + NBUF - 1) * nw, b[(u + NBUF - 1) % NBUF]);
        process(st + (uint32_t)u * nw, b[u]);
        done = st + (uint32_t)(u + 1) * nw >= nst;
      }
    }
    if (done) break;
  }
  if (rc) rescore(rc);
  if (lane == 0) {
    A.qcount[2 * gw] = qn;
    A.qcount[2 * gw + 1] = qf;
    if constexpr (MODE == 1) A.chg_cnt[gw] = cc;
  }
  if constexpr (SSE) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) ssa += __shfl_xor(ssa, o);
    if (lane == 0 && ssa != 0.0) atomicAdd(A.sse, ssa);
  }
}

// Delta statistics (km_runtime.hip): mode 1 folds an iteration's all-reduced
// deltas into the full sums and hands them to the update (full += stats;
// stats = full); mode 2 folds them and clears the deltas for the next
// iteration (full += stats; stats = 0: the update reads full, no memset);
// mode 0 keeps an iteration's full statistics (full = stats), the base of
// the next deltas.  The SSE slot rides along (0 in delta mode).
__global__ __launch_bounds__(256) void k_s1_apply(double* __restrict__ stats, double* __restrict__ full, int64_t len,
                                                  int mode, const int* __restrict__ gate) {
  if (*gate) return;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  double v = stats[i];
  // (the SSE slot, the last entry, is this iteration's residual sum, never
  // carried: it is replaced, not added)
  if (mode >= 1 && i != len - 1) v = full[i] + v;
  full[i] = v;
  stats[i] = mode == 2 ? 0.0 : v;
}

// A change list into the delta statistics.  The list is nw wave segments
// of seg entries {row, old << 16 | new}: segment w holds cnt[w] entries of
// the screen and, with qcount (delta resolvers, launch_resolve), qcount[2w] +
// qcount[2w+1] entries of the resolvers behind them (old == new: the row kept
// its label, skipped without reading it).  The clusters are split into
// `nr` ranges of kr, each small enough for an LDS float64 table [kr][d+1];
// workgroup b aggregates range b % nr over slice b / nr of the concatenated
// list (at least S1D_MIN entries, so a short list wakes few workgroups): each
// wave takes 64 entries at a time (one per lane, its segment by a binary
// search of the LDS prefix), keeps those with an end in its range (ballot),
// and moves their rows 8 at a time (lanes over features, the x loads of the
// 8 issued together) with LDS float64 atomics; the table's non-zero entries
// then go to the statistics with global atomics.  An entry is read by every
// range's workgroups (8 B each) but its row only by the workgroups of its two
// clusters, so no float64 atomic reaches global memory per changed row: the
// c4 and c5 classes, whose [k][d+1] table exceeds LDS, fold millions of
// changed rows (poor seeds, first iterations) at the cost of reading them.
#ifndef KM_S1D_MIN
#define KM_S1D_MIN 256
#endif
constexpr uint32_t S1D_MIN = KM_S1D_MIN;
constexpr int S1D_ROWS = 8;
__global__ __launch_bounds__(1024) void k_s1_delta(const float* __restrict__ X, int dp, int d, int k,
                                                   const uint2* __restrict__ chg, const uint32_t* __restrict__ cnt,
                                                   const uint32_t* __restrict__ qcount, int nw, uint32_t seg, int kr,
                                                   int nr, double* __restrict__ stats,
                                                   const int* __restrict__ gate) {
  if (*gate) return;
  extern __shared__ double smem_d[];  // [kr][d + 1], then pre[nw + 1] and 16 wave sums
  const int d1 = d + 1;
  double* tab = smem_d;
  uint32_t* pre = reinterpret_cast<uint32_t*>(smem_d + (size_t)kr * d1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  {
    // exclusive prefix of the segment totals over the whole workgroup: thread
    // t owns segments [t c, (t + 1) c), a wave scan, then the waves' sums
    // (one pass of independent loads instead of a dependent loop on wave 0)
    uint32_t* wsum = pre + nw + 1;  // [16]
    auto total = [&](int w) {
      uint32_t v = cnt[w];
      if (qcount) v += qcount[2 * w] + qcount[2 * w + 1];
      return min(v, seg);
    };
    const int nt = (int)blockDim.x, t = (int)threadIdx.x;
    const int c = (nw + nt - 1) / nt, b0 = t * c;
    uint32_t v = 0;
    for (int i = 0; i < c; ++i)
      if (b0 + i < nw) v += total(b0 + i);
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o);
      inc += lane >= o ? u : 0u;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < wave; ++i) base += wsum[i];
    uint32_t run = base + inc - v;
    for (int i = 0; i < c; ++i)
      if (b0 + i < nw) {
        pre[b0 + i] = run;
        run += total(b0 + i);
      }
    if (t == nt - 1) pre[nw] = run;
  }
  __syncthreads();
  const int r = (int)(blockIdx.x % (uint32_t)nr);
  const uint32_t ns = gridDim.x / (uint32_t)nr, sl = blockIdx.x / (uint32_t)nr;
  const uint32_t nc = pre[nw];
  // a slice is at least S1D_MIN entries and 1/16 of the table: every busy
  // workgroup flushes its whole table with global atomics, so a short list
  // spread over all workgroups would contend on the same addresses
  const uint32_t lo = (uint32_t)r * (uint32_t)kr;
  const uint32_t span = min((uint32_t)kr, (uint32_t)k - lo);
  const uint32_t per = max(max(S1D_MIN, (uint32_t)kr * (uint32_t)d1 / 16u), (nc + ns - 1u) / ns);
  const uint32_t e0 = sl * per;
  if (sl >= ns || e0 >= nc) return;
  const uint32_t e1 = min(nc, e0 + per);
  for (int i = threadIdx.x; i < (int)span * d1; i += blockDim.x) tab[i] = 0.0;
  __syncthreads();
  // entry e of the concatenation: segment w = the last with pre[w] <= e; a
  // lane's entries only grow, so after one binary search its segment is
  // found by walking forward (a step or two per window)
  int sgl = 0;
  {
    const uint32_t e = min(e0 + (uint32_t)wave * 64u + (uint32_t)lane, nc - 1u);
    int h = nw - 1;
    while (sgl < h) {
      const int mid = (sgl + h + 1) >> 1;
      if (pre[mid] <= e) sgl = mid; else h = mid - 1;
    }
  }
  auto at = [&](uint32_t e) {
    while (sgl + 1 < nw && pre[sgl + 1] <= e) ++sgl;
    return chg[(size_t)sgl * seg + (e - pre[sgl])];
  };
  for (uint32_t base = e0 + (uint32_t)wave * 64u; base < e1; base += (uint32_t)nwv * 64u) {
    const uint32_t e = base + (uint32_t)lane;
    const uint2 c = e < e1 ? at(e) : make_uint2(0u, 0u);
    const uint32_t o = c.y >> 16, nn = c.y & 0xFFFFu;
    const bool mine = e < e1 && o != nn && (o - lo < span || nn - lo < span);
    uint64_t m = __ballot(mine);
    while (m) {
      // up to 8 of the wave's entries in range (uniform: m is scalar)
      uint32_t row[S1D_ROWS], oy[S1D_ROWS];
      int na = 0;
#pragma unroll
      for (int j = 0; j < S1D_ROWS; ++j) {
        row[j] = 0u;
        oy[j] = 0u;  // old = new = 0: no move
        if (m) {
          const int src = __builtin_ctzll(m);
          m &= m - 1ull;
          row[j] = (uint32_t)__builtin_amdgcn_readlane((int)c.x, src);
          oy[j] = (uint32_t)__builtin_amdgcn_readlane((int)c.y, src);
          ++na;
        }
      }
      for (int f0 = 0; f0 < d; f0 += 64) {
        const int f = f0 + lane;
        float x[S1D_ROWS];
#pragma unroll
        for (int j = 0; j < S1D_ROWS; ++j) x[j] = (j < na && f < d) ? X[(size_t)row[j] * dp + f] : 0.0f;
        if (f < d)
#pragma unroll
          for (int j = 0; j < S1D_ROWS; ++j) {
            const uint32_t jo = oy[j] >> 16, jn = oy[j] & 0xFFFFu;
            if (j >= na) continue;
            if (jo - lo < span) atomicAdd(tab + (size_t)(jo - lo) * d1 + f, -(double)x[j]);
            if (jn - lo < span) atomicAdd(tab + (size_t)(jn - lo) * d1 + f, (double)x[j]);
          }
      }
      if (lane < na) {
        // the counts: lane j takes entry j's two ends
        uint32_t jy = 0u;
#pragma unroll
        for (int j = 0; j < S1D_ROWS; ++j) jy = lane == j ? oy[j] : jy;
        const uint32_t jo = jy >> 16, jn = jy & 0xFFFFu;
        if (jo - lo < span) atomicAdd(tab + (size_t)(jo - lo) * d1 + d, -1.0);
        if (jn - lo < span) atomicAdd(tab + (size_t)(jn - lo) * d1 + d, 1.0);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (int)span * d1; i += blockDim.x) {
    const double v = tab[i];
    if (v != 0.0) atomicAdd(stats + (size_t)lo * d1 + i, v);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// k_s1's grid: workgroups (one per CU at most, 8 waves each) and the rows
// of one wave's queue / change-list segment
static int s1_geo_waves(const Geometry& g) { return s1_waves(g.dp / 32, g.kp / 32); }
static int64_t s1_grid(const Geometry& g, int n_cu, int* nbk, uint32_t* seg) {
  const int tt = s1_tiles(g.dp / 32);
  const int w = s1_geo_waves(g);
  const int64_t nst = ((g.n + 15) / 16 + tt - 1) / tt;  // wave steps of tt tiles
  int64_t blocks = n_cu;
  if (blocks > (nst + w - 1) / w) blocks = (nst + w - 1) / w;
  *nbk = (int)blocks;
  const int64_t nw = blocks * w;
  *seg = nw ? (uint32_t)(((nst + nw - 1) / nw) * 16 * tt) : 0u;
  return nw;
}

size_t s1_chg_entries(const Geometry& g, int n_cu) {
  int nbk;
  uint32_t seg;
  const int64_t nw = s1_grid(g, n_cu, &nbk, &seg);
  return (size_t)std::max<int64_t>(nw * (int64_t)seg, 1);
}

size_t s1_wave_slots(int n_cu) { return (size_t)n_cu * S1_MAX_WAVES; }

// delta statistics on every geometry with 16-bit cluster ids (k_s1_delta
// splits the clusters into ranges whose LDS tables fit)
bool s1_delta_ok(const Geometry& g, int n_cu) {
  (void)n_cu;
  return g.k <= 65535;
}

hipError_t launch_chg_delta(const float* X, const Geometry& g, const uint2* chg, const uint32_t* chg_cnt, int nw,
                            uint32_t seg, double* stats, int n_cu, const int* gate, hipStream_t s,
                            const uint32_t* qcount) {
  if (g.n == 0 || nw == 0) return hipSuccess;
  if (g.k > 65535) return hipErrorInvalidValue;
  constexpr size_t LDS = 160 * 1024;
  const size_t pre = ((size_t)nw + 1 + 16) * 4;  // + the prefix's per-wave sums
  const size_t row = (size_t)(g.d + 1) * 8;  // one cluster's table row
  if (pre > 64 * 1024 || pre + row > LDS) return hipErrorInvalidValue;
  // ranges of clusters whose [kr][d+1] table fits beside the prefix, as few
  // as possible, balanced; ~n_cu workgroups (at least one per range)
  const int kmax = (int)((LDS - pre) / row);
  const int nr = (g.k + kmax - 1) / kmax;
  const int kr = (g.k + nr - 1) / nr;
  const int ns = std::max(1, (n_cu + nr / 2) / nr);
  hipLaunchKernelGGL(k_s1_delta, dim3((unsigned)(nr * ns)), dim3(1024), (size_t)kr * row + pre, s, X, g.dp, g.d, g.k,
                     chg, chg_cnt, qcount, nw, seg, kr, nr, stats, gate);
  return hipGetLastError();
}

hipError_t launch_s1_delta(const float* X, const Geometry& g, const uint2* chg, const uint32_t* chg_cnt,
                           double* stats, int n_cu, const int* gate, hipStream_t s, const uint32_t* qcount) {
  if (g.n == 0) return hipSuccess;
  int nbk;
  uint32_t seg;
  const int64_t nw = s1_grid(g, n_cu, &nbk, &seg);
  if (!s1_delta_ok(g, n_cu)) return hipErrorInvalidValue;
  return launch_chg_delta(X, g, chg, chg_cnt, (int)nw, seg, stats, n_cu, gate, s, qcount);
}

hipError_t launch_s1_apply(double* stats, double* full, int64_t len, int mode, const int* gate, hipStream_t s) {
  if (len <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_s1_apply, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, s, stats, full, len, mode, gate);
  return hipGetLastError();
}

// geometry only (never n): every rank of a job must take the same path, or
// their delta and full statistics would be summed together
bool s1_ok(const Geometry& g) {
  if (g.dp % 32 || g.kp % 64) return false;
  switch ((g.dp / 32) * 100 + g.kp / 32) {
    case 202: case 204: case 206: case 208:
    case 102: case 104: case 106: case 108: case 112: case 116: case 132:
    case 216:
    case 402: case 404:
      return true;
    default:
      return false;
  }
}

static S1Geo s1_geo(const Geometry& g) {
  S1Geo sg;
  sg.nb = g.kp / 32;
  sg.mb = ceil_log2_c(sg.nb);
  sg.ns2 = g.dp / 32;
  return sg;
}

size_t s1_table_entries(const Geometry& g) { return (size_t)32 << s1_geo(g).mb; }

hipError_t launch_s1_color(const float* C32, const Geometry& g, int32_t* perm, const int* gate, hipStream_t s) {
  const S1Geo sg = s1_geo(g);
  if (g.k > (g.dp == 32 ? 1024 : 512)) return hipErrorInvalidValue;
  switch (g.dp) {
    case 32:
      if (g.k > 512)
        hipLaunchKernelGGL((k_s1_color<32, 1024>), dim3(1), dim3(1024), 0, s, C32, g.k, g.dp, sg.nb, sg.mb, perm, gate);
      else
        hipLaunchKernelGGL((k_s1_color<32, 512>), dim3(1), dim3(512), 0, s, C32, g.k, g.dp, sg.nb, sg.mb, perm, gate);
      break;
    case 64:
      hipLaunchKernelGGL((k_s1_color<64, 512>), dim3(1), dim3(512), 0, s, C32, g.k, g.dp, sg.nb, sg.mb, perm, gate);
      break;
    case 128:
      hipLaunchKernelGGL((k_s1_color<128, 512>), dim3(1), dim3(512), 0, s, C32, g.k, g.dp, sg.nb, sg.mb, perm, gate);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_s1_prep(const double* C64, const float* C32, const Geometry& g, const int32_t* perm,
                          const float* cmax, const float* xabs, const float* cabs, float* cft, float* cn2o,
                          uint4* img, float* cst, const int* gate, hipStream_t s) {
  const S1Geo sg = s1_geo(g);
  const int nt = 32 << sg.mb;
  hipLaunchKernelGGL(k_s1_prep, dim3(nt + 1), dim3(64), 0, s, C64, C32, g.k, g.d, g.dp, sg, perm, cmax, xabs, cabs,
                     cft, cn2o, img, cst, gate);
  return hipGetLastError();
}

hipError_t launch_s1(const float* X, const float* xnorm, const Geometry& g, const uint4* img, const float* cn2o,
                     const float* cft, const int32_t* perm, const float* cst, int32_t* labels,
                     QEntry* queue, uint32_t* qcount, uint2* chg, uint32_t* chg_cnt, int delta, int n_cu,
                     QLayout* ql, const int* gate, hipStream_t s, int rev, double* sse) {
  ql->seg = 0;
  ql->nwaves = 0;
  if (g.n == 0) return hipSuccess;
  const S1Geo sg = s1_geo(g);
  const int nt = 32 << sg.mb;
  int nbk;
  uint32_t seg;
  const int64_t nw = s1_grid(g, n_cu, &nbk, &seg);
  ql->seg = seg;
  ql->nwaves = (uint32_t)nw;
  if (sse && !delta) return hipErrorInvalidValue;  // residuals ride with delta statistics only
  S1Args a{X, xnorm, g.n, g.k, g.d, seg, img, cn2o, cft, perm, cst, labels, queue, qcount, chg, chg_cnt, sse, gate};
  const size_t lds = s1_lds_bytes(sg.ns2, sg.nb, !s1_table_global(sg.ns2, sg.nb));
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  (void)nt;
#define KM_S1_CASE(NS2_, NB_)                                                                                   \
  case NS2_ * 100 + NB_:                                                                                        \
    if (delta && sse)                                                                                           \
      KM_TIMED_LAUNCH((k_s1<NS2_, NB_, 1, false, true>), dim3(nbk), dim3(s1_waves(NS2_, NB_) * 64), lds, s, a); \
    else if (delta && rev && KM_S1_SERP && NS2_ == 2 && NB_ == 8)                                               \
      KM_TIMED_LAUNCH((k_s1<2, 8, 1, true>), dim3(nbk), dim3(s1_waves(2, 8) * 64), lds, s, a);                  \
    else if (delta)                                                                                             \
      KM_TIMED_LAUNCH((k_s1<NS2_, NB_, 1>), dim3(nbk), dim3(s1_waves(NS2_, NB_) * 64), lds, s, a);              \
    else                                                                                                        \
      KM_TIMED_LAUNCH((k_s1<NS2_, NB_, 0>), dim3(nbk), dim3(s1_waves(NS2_, NB_) * 64), lds, s, a);              \
    break;
  switch (sg.ns2 * 100 + sg.nb) {
    KM_S1_CASE(2, 2) KM_S1_CASE(2, 4) KM_S1_CASE(2, 6) KM_S1_CASE(2, 8)
    KM_S1_CASE(1, 2) KM_S1_CASE(1, 4) KM_S1_CASE(1, 6) KM_S1_CASE(1, 8) KM_S1_CASE(1, 12) KM_S1_CASE(1, 16)
    KM_S1_CASE(1, 32) KM_S1_CASE(2, 16) KM_S1_CASE(4, 2) KM_S1_CASE(4, 4)
    default:
      return hipErrorInvalidValue;
  }
#undef KM_S1_CASE
  return hipGetLastError();
}

}  // namespace km
