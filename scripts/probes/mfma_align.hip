// Probe: alignment width of v_mfma_f32_32x32x16_f16's internal sum.  Exact
// result = 2^(12-m): a cancelling pair +-2^12 (in C and a product, or two
// products at slots i, j) plus a small product 2^(12-m) at slot s.  Prints,
// per m, whether the small term survived (1), was dropped (0) or changed.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const float* a16, const float* b16, float c0, float* out) {
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  f16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    const int kk = 8 * h + e;
    a[e] = (_Float16)(r == 0 ? a16[kk] : 0.0f);
    b[e] = (_Float16)(r == 0 ? b16[kk] : 0.0f);
  }
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  if (lane == 0) acc[0] = c0;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];
}

static float *da, *db, *dout;
static float run(const float* a, const float* b, float c0) {
  float o;
  (void)hipMemcpy(da, a, 64, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, c0, dout);
  (void)hipMemcpy(&o, dout, 4, hipMemcpyDeviceToHost);
  return o;
}

int main() {
  (void)hipMalloc(&da, 64); (void)hipMalloc(&db, 64); (void)hipMalloc(&dout, 4);
  float a[16], b[16];
  // small product 2^(12-m) = a*b with a = 2^-7 .. built as 2^e1 * 2^e2 within fp16 normal range
  auto small = [&](int m, float& x, float& y) {
    const int e = 12 - m;  // target exponent
    const int e1 = e / 2, e2 = e - e1;
    x = ldexpf(1.0f, e1);
    y = ldexpf(1.0f, e2);
  };
  printf("m   : Cbig(C=2^12,p=-2^12 @0, small @s=1,8,15) | prods(+2^12 @0, -2^12 @1, small @2,9,15)\n");
  for (int m = 16; m <= 44; m += 2) {
    char line[256]; int pos = 0;
    pos += snprintf(line + pos, sizeof line - pos, "%3d :", m);
    for (int s : {1, 8, 15}) {
      memset(a, 0, sizeof a); memset(b, 0, sizeof b);
      a[0] = -64; b[0] = 64;
      small(m, a[s], b[s]);
      const float o = run(a, b, 4096.0f);
      const float ex = ldexpf(1.0f, 12 - m);
      pos += snprintf(line + pos, sizeof line - pos, " %s", o == ex ? "1" : (o == 0.0f ? "0" : "x"));
    }
    pos += snprintf(line + pos, sizeof line - pos, "   |");
    for (int s : {2, 9, 15}) {
      memset(a, 0, sizeof a); memset(b, 0, sizeof b);
      a[0] = 64; b[0] = 64; a[1] = -64; b[1] = 64;
      small(m, a[s], b[s]);
      const float o = run(a, b, 0.0f);
      const float ex = ldexpf(1.0f, 12 - m);
      pos += snprintf(line + pos, sizeof line - pos, " %s", o == ex ? "1" : (o == 0.0f ? "0" : "x"));
    }
    printf("%s\n", line);
  }
  // max relative error over random sign-mixed inputs vs sum of |terms| and vs max |term|
  double worst_sum = 0, worst_max = 0;
  unsigned seed = 12345;
  auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return (seed >> 8) * (1.0 / 16777216.0); };
  for (int trial = 0; trial < 20000; ++trial) {
    double exact = 0, suma = 0, mx = 0;
    for (int i = 0; i < 16; ++i) {
      const float ea = (float)(rnd() * 2 - 1) * ldexpf(1.0f, (int)(rnd() * 16) - 8);
      const float eb = (float)(rnd() * 2 - 1) * ldexpf(1.0f, (int)(rnd() * 16) - 8);
      a[i] = (float)(_Float16)ea; b[i] = (float)(_Float16)eb;
      const double p = (double)a[i] * b[i];
      exact += p; suma += fabs(p); mx = fmax(mx, fabs(p));
    }
    const float c0 = (float)((rnd() * 2 - 1) * ldexp(1.0, (int)(rnd() * 20) - 6));
    exact += c0; suma += fabs(c0); mx = fmax(mx, fabs(c0));
    const double o = run(a, b, c0);
    const double err = fabs(o - exact);
    const double u = ldexp(1.0, -24);
    worst_sum = fmax(worst_sum, err / (u * suma));
    worst_max = fmax(worst_max, (err - u * fabs(exact)) / (u * mx));
  }
  printf("random: max err / (u*sum|terms|) = %.3f ; max (err - u|exact|)/(u*max|term|) = %.3f\n", worst_sum, worst_max);
  return 0;
}
