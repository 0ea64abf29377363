// Exact float64 distances in the reference's rounding (device helpers shared
// by km_kernels.hip and the probes under scripts/probes).
#pragma once
#include <hip/hip_runtime.h>

namespace km {

// ---------------------------------------------------------------------------
// Exact distances.  The reference ranks centroids by np.linalg.norm(C - point,
// axis=1) (kmeans_spark.py:153) and takes np.argmin (L156): per centroid
// t_f = c_f - x_f and t_f*t_f each rounded in float64 (no fma), summed by
// NumPy's pairwise_sum over the contiguous feature axis, then sqrt; the first
// index wins ties of the sqrt values.  pairwise_sum (NumPy
// _core/src/umath/loops_utils.h.src): n < 8 -> sequential from 0.0; n <= 128
// -> 8 strided accumulators r[i%8] over the first n - n%8 terms, combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), remainder added in order; n > 128 ->
// halves split at n/2 rounded down to a multiple of 8, summed recursively.
// Reproducing that order makes the float64 labels bit-identical to the
// reference's, near-ties included (tests/test_gpu_parity.py near-tie case).
// Contraction is off in np_sq and np_add, whose fmul/fadd therefore carry no
// 'contract' flag: a fused multiply-add would skip the square's rounding.
// (HIP's __dadd_rn/__dmul_rn are plain + and * defined in a header, so a
// pragma around their call sites does not reach them.)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double np_sq(double c, float x) {
#pragma clang fp contract(off)
  const double t = c - (double)x;
  return t * t;
}

__device__ __forceinline__ double np_add(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}

__device__ __forceinline__ double np_combine8(const double (&r)[8]) {
#pragma clang fp contract(off)
  return np_add(np_add(np_add(r[0], r[1]), np_add(r[2], r[3])),
                   np_add(np_add(r[4], r[5]), np_add(r[6], r[7])));
}

// pairwise block, n <= 128 terms sq(lo), ..., sq(lo + n - 1)
template <class SQ>
__device__ inline double np_pw_block(const SQ& sq, int lo, int n) {
#pragma clang fp contract(off)
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r = np_add(r, sq(lo + i));
    return r;
  }
  double r[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) r[u] = sq(lo + u);
  const int nm = n - (n & 7);
  int i = 8;
  for (; i < nm; i += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = np_add(r[u], sq(lo + i + u));
  }
  double res = np_combine8(r);
  for (; i < n; ++i) res = np_add(res, sq(lo + i));
  return res;
}

template <int DEPTH, class SQ>
__device__ inline double np_pw(const SQ& sq, int lo, int n) {
#pragma clang fp contract(off)
  if constexpr (DEPTH == 0) {
    return np_pw_block(sq, lo, n);
  } else {
    if (n <= 128) return np_pw_block(sq, lo, n);
    int n2 = n >> 1;
    n2 -= n2 & 7;
    return np_add(np_pw<DEPTH - 1>(sq, lo, n2), np_pw<DEPTH - 1>(sq, lo + n2, n - n2));
  }
}

// Two norms in lockstep (one lane): SQ2(f, ta, tb) yields the terms of both
// at feature f, so a centroid value read once serves two points; each sum
// keeps NumPy's pairwise order exactly as np_pw_block / np_pw do.
template <class SQ2>
__device__ inline void np_pw2_block(const SQ2& sq, int lo, int n, double& sa, double& sb) {
#pragma clang fp contract(off)
  if (n < 8) {
    double ra = 0.0, rb = 0.0;
    for (int i = 0; i < n; ++i) {
      double ta, tb;
      sq(lo + i, ta, tb);
      ra = np_add(ra, ta);
      rb = np_add(rb, tb);
    }
    sa = ra;
    sb = rb;
    return;
  }
  double ra[8], rb[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) sq(lo + u, ra[u], rb[u]);
  const int nm = n - (n & 7);
  int i = 8;
  for (; i < nm; i += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      double ta, tb;
      sq(lo + i + u, ta, tb);
      ra[u] = np_add(ra[u], ta);
      rb[u] = np_add(rb[u], tb);
    }
  }
  double xa = np_combine8(ra), xb = np_combine8(rb);
  for (; i < n; ++i) {
    double ta, tb;
    sq(lo + i, ta, tb);
    xa = np_add(xa, ta);
    xb = np_add(xb, tb);
  }
  sa = xa;
  sb = xb;
}

template <int DEPTH, class SQ2>
__device__ inline void np_pw2(const SQ2& sq, int lo, int n, double& sa, double& sb) {
#pragma clang fp contract(off)
  if constexpr (DEPTH == 0) {
    np_pw2_block(sq, lo, n, sa, sb);
  } else {
    if (n <= 128) {
      np_pw2_block(sq, lo, n, sa, sb);
      return;
    }
    int n2 = n >> 1;
    n2 -= n2 & 7;
    double a1, b1, a2, b2;
    np_pw2<DEPTH - 1>(sq, lo, n2, a1, b1);
    np_pw2<DEPTH - 1>(sq, lo + n2, n - n2, a2, b2);
    sa = np_add(a1, a2);
    sb = np_add(b1, b2);
  }
}

// np.linalg.norm of one centroid row: two halvings suffice for d <= 256 (a
// half of n <= 256 has at most n/2 + 8 terms), five for d <= 2048 (wide rows)
template <int DEPTH, class SQ>
__device__ inline double np_norm_d(const SQ& sq, int d) {
  return sqrt(np_pw<DEPTH>(sq, 0, d));
}
template <class SQ>
__device__ inline double np_norm(const SQ& sq, int d) {
  if (d <= 256) return sqrt(np_pw<2>(sq, 0, d));
  return sqrt(np_pw<5>(sq, 0, d));
}

// same, with the point in registers (d <= DP <= 128: one block, unrolled so
// x[] stays in VGPRs)
template <int DP>
__device__ inline double np_norm_reg(const float (&x)[DP], const double* __restrict__ c, int d) {
#pragma clang fp contract(off)
  static_assert(DP <= 128 && DP >= 8, "one pairwise block");
  double res = 0.0;
  if (d < 8) {
#pragma unroll
    for (int f = 0; f < 8; ++f)
      if (f < d) res = np_add(res, np_sq(c[f], x[f]));
  } else {
    const int nm = d - (d & 7);
    double r[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) r[f] = np_sq(c[f], x[f]);
#pragma unroll
    for (int f = 8; f < DP; ++f)
      if (f < nm) r[f & 7] = np_add(r[f & 7], np_sq(c[f], x[f]));
    res = np_combine8(r);
#pragma unroll
    for (int f = 8; f < DP; ++f)
      if (f >= nm && f < d) res = np_add(res, np_sq(c[f], x[f]));
  }
  return sqrt(res);
}

// Cooperative form: 8 consecutive lanes (u = lane & 7) evaluate one norm,
// lane u holding NumPy's accumulator r[u]; the xor-butterfly over 1, 2, 4
// forms exactly ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) (IEEE addition is
// commutative), after which every lane holds the block sum and adds the
// remainder terms itself.  SQ2 evaluates two norms (a, b) at once.
template <class SQ2>
__device__ inline void np_pw_block8(const SQ2& sq, int lo, int n, int u, double& sa, double& sb) {
#pragma clang fp contract(off)
  double ra = 0.0, rb = 0.0;
  if (n < 8) {
    for (int i = 0; i < n; ++i) {
      double ta, tb;
      sq(lo + i, ta, tb);
      ra = np_add(ra, ta);
      rb = np_add(rb, tb);
    }
    sa = ra;
    sb = rb;
    return;
  }
  sq(lo + u, ra, rb);
  const int nm = n - (n & 7);
  for (int i = 8; i < nm; i += 8) {
    double ta, tb;
    sq(lo + i + u, ta, tb);
    ra = np_add(ra, ta);
    rb = np_add(rb, tb);
  }
#pragma unroll
  for (int o = 1; o <= 4; o <<= 1) {
    ra = np_add(ra, __shfl_xor(ra, o));
    rb = np_add(rb, __shfl_xor(rb, o));
  }
  for (int i = nm; i < n; ++i) {
    double ta, tb;
    sq(lo + i, ta, tb);
    ra = np_add(ra, ta);
    rb = np_add(rb, tb);
  }
  sa = ra;
  sb = rb;
}

template <int DEPTH, class SQ2>
__device__ inline void np_pw8(const SQ2& sq, int lo, int n, int u, double& sa, double& sb) {
#pragma clang fp contract(off)
  if constexpr (DEPTH == 0) {
    np_pw_block8(sq, lo, n, u, sa, sb);
  } else {
    if (n <= 128) {
      np_pw_block8(sq, lo, n, u, sa, sb);
      return;
    }
    int n2 = n >> 1;
    n2 -= n2 & 7;
    double a1, b1, a2, b2;
    np_pw8<DEPTH - 1>(sq, lo, n2, u, a1, b1);
    np_pw8<DEPTH - 1>(sq, lo + n2, n - n2, u, a2, b2);
    sa = np_add(a1, a2);
    sb = np_add(b1, b2);
  }
}

// np.argmin update in ascending index order: the first NaN wins, else the
// first strict minimum
__device__ __forceinline__ bool np_better(double v, double best, bool have) {
  if (!have) return true;
  if (best != best) return false;
  return (v != v) || v < best;
}

// np.argmin over a pair (a < b)
__device__ __forceinline__ bool np_pick_second(double va, double vb) {
  return !(va != va) && ((vb != vb) || vb < va);
}

}  // namespace km
