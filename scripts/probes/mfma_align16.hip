// Probe: accumulation behaviour of v_mfma_f32_16x16x32_f16 on gfx950 (the
// 16x16x32 counterpart of mfma_align.hip / mfma_round.hip, which characterise
// v_mfma_f32_32x32x16_f16 for the screening bound in km_kernels.hip).
// Lane mapping (cdna_hip_programming.md section 3): lane l holds
// A[row l&15][k = 8(l>>4) + e] and B[k = 8(l>>4) + e][col l&15]; D[0][0] is lane 0, reg 0.
// Prints: (1) alignment: exact result 2^(12-m) from a cancelling pair +-2^12
// and a small product at slot s -- survived (1), dropped (0) or changed (x);
// (2) the rounding cases of mfma_round.hip with 32 products; (3) the worst
// error over random sign-mixed inputs vs u*sum|terms| and vs u*max|term|,
// and the same with the cancelling pair in different 8-slot groups.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int KK = 32;

__global__ void k(const float* a32, const float* b32, float c0, float* out) {
  const int lane = threadIdx.x, r = lane & 15, q = lane >> 4;
  f16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    const int kk = 8 * q + e;
    a[e] = (_Float16)(r == 0 ? a32[kk] : 0.0f);
    b[e] = (_Float16)(r == 0 ? b32[kk] : 0.0f);
  }
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  if (lane == 0) acc[0] = c0;
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];
}

static float *da, *db, *dout;
static float run(const float* a, const float* b, float c0) {
  float o;
  (void)hipMemcpy(da, a, 4 * KK, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, 4 * KK, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, c0, dout);
  (void)hipMemcpy(&o, dout, 4, hipMemcpyDeviceToHost);
  return o;
}

int main() {
  (void)hipMalloc(&da, 4 * KK); (void)hipMalloc(&db, 4 * KK); (void)hipMalloc(&dout, 4);
  float a[KK], b[KK];
  auto small = [&](int m, float& x, float& y) {
    const int e = 12 - m;
    const int e1 = e / 2, e2 = e - e1;
    x = ldexpf(1.0f, e1);
    y = ldexpf(1.0f, e2);
  };
  printf("m   : Cbig(C=2^12,p=-2^12 @0, small @s=1,8,16,31) | prods(+2^12 @0, -2^12 @1, small @2,9,17,31) | "
         "prods(+2^12 @0, -2^12 @24, small @1,12,25,31)\n");
  for (int m = 16; m <= 44; m += 2) {
    char line[512]; int pos = 0;
    pos += snprintf(line + pos, sizeof line - pos, "%3d :", m);
    const float ex = ldexpf(1.0f, 12 - m);
    for (int s : {1, 8, 16, 31}) {
      memset(a, 0, sizeof a); memset(b, 0, sizeof b);
      a[0] = -64; b[0] = 64;
      small(m, a[s], b[s]);
      const float o = run(a, b, 4096.0f);
      pos += snprintf(line + pos, sizeof line - pos, " %s", o == ex ? "1" : (o == 0.0f ? "0" : "x"));
    }
    pos += snprintf(line + pos, sizeof line - pos, "   |");
    for (int s : {2, 9, 17, 31}) {
      memset(a, 0, sizeof a); memset(b, 0, sizeof b);
      a[0] = 64; b[0] = 64; a[1] = -64; b[1] = 64;
      small(m, a[s], b[s]);
      const float o = run(a, b, 0.0f);
      pos += snprintf(line + pos, sizeof line - pos, " %s", o == ex ? "1" : (o == 0.0f ? "0" : "x"));
    }
    pos += snprintf(line + pos, sizeof line - pos, "   |");
    for (int s : {1, 12, 25, 31}) {
      memset(a, 0, sizeof a); memset(b, 0, sizeof b);
      a[0] = 64; b[0] = 64; a[24] = -64; b[24] = 64;
      small(m, a[s], b[s]);
      const float o = run(a, b, 0.0f);
      pos += snprintf(line + pos, sizeof line - pos, " %s", o == ex ? "1" : (o == 0.0f ? "0" : "x"));
    }
    printf("%s\n", line);
  }
  // rounding cases (mfma_round.hip with 32 products)
  for (int i = 0; i < KK; ++i) { a[i] = 1.0f; b[i] = 0.5f; }
  printf("case1 C=2^24 + 32*0.5 : got %.1f (exact %.1f, sequential %.1f)\n", run(a, b, 16777216.0f), 16777232.0,
         16777216.0);
  memset(a, 0, sizeof a); memset(b, 0, sizeof b);
  for (int i = 0; i < 3; ++i) { a[i] = 1.0f / 4096; b[i] = 1.0f / 8192; }
  float o = run(a, b, 1.0f);
  printf("case6 1 + 3*2^-25 : got 1 + %.3g ulp (exact-once 1 ulp, truncating 0)\n", (o - 1.0f) / 1.1920929e-07f);
  memset(a, 0, sizeof a); memset(b, 0, sizeof b);
  for (int i = 0; i < 3; ++i) { a[i] = -1.0f / 4096; b[i] = 1.0f / 8192; }
  o = run(a, b, 1.0f);
  printf("case7 1 - 3*2^-25 : got 1 - %.4g * 2^-24 (RNE once: 1 or 2; trunc toward 0: 2; sequential: 0)\n",
         (1.0f - o) / 5.9604645e-08f);
  // random sign-mixed inputs: terms spread over 16 binades (as mfma_align.hip), then over 4
  unsigned seed = 12345;
  auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return (seed >> 8) * (1.0 / 16777216.0); };
  for (int spread : {16, 4}) {
    double worst_sum = 0, worst_max = 0;
    for (int trial = 0; trial < 20000; ++trial) {
      double exact = 0, suma = 0, mx = 0;
      for (int i = 0; i < KK; ++i) {
        const float ea = (float)(rnd() * 2 - 1) * ldexpf(1.0f, (int)(rnd() * spread) - spread / 2);
        const float eb = (float)(rnd() * 2 - 1) * ldexpf(1.0f, (int)(rnd() * spread) - spread / 2);
        a[i] = (float)(_Float16)ea; b[i] = (float)(_Float16)eb;
        const double p = (double)a[i] * b[i];
        exact += p; suma += fabs(p); mx = fmax(mx, fabs(p));
      }
      const float c0 = (float)((rnd() * 2 - 1) * ldexp(1.0, (int)(rnd() * 20) - 6));
      exact += c0; suma += fabs(c0); mx = fmax(mx, fabs(c0));
      const double ov = run(a, b, c0);
      const double err = fabs(ov - exact);
      const double u = ldexp(1.0, -24);
      worst_sum = fmax(worst_sum, err / (u * suma));
      worst_max = fmax(worst_max, (err - u * fabs(exact)) / (u * mx));
    }
    printf("random (spread %d binades): max err/(u*sum|terms|) = %.3f ; max (err - u|exact|)/(u*max|term|) = %.3f\n",
           spread, worst_sum, worst_max);
  }
  return 0;
}
