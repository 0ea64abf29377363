// Probe: rounding behaviour of v_mfma_f32_32x32x16_f16 accumulation on gfx950.
// D = C + sum_k A[i][k] B[k][j].  Each case fills row 0 / column 0 only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const float* a16, const float* b16, float c0, float* out) {
  // A: 32x16 (rows on lanes&31, k = 8*(lane>>5) + e); B: 16x32 same mapping on columns
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  f16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    const int kk = 8 * h + e;
    a[e] = (_Float16)(r == 0 ? a16[kk] : 0.0f);
    b[e] = (_Float16)(r == 0 ? b16[kk] : 0.0f);
  }
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  if (lane == 0) acc[0] = c0;   // D[0][0] lives in lane 0, reg 0
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];
}

static float run(const float* a, const float* b, float c0) {
  float *da, *db, *dout, o;
  hipMalloc(&da, 64); hipMalloc(&db, 64); hipMalloc(&dout, 4);
  hipMemcpy(da, a, 64, hipMemcpyHostToDevice); hipMemcpy(db, b, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, c0, dout);
  hipMemcpy(&o, dout, 4, hipMemcpyDeviceToHost);
  hipFree(da); hipFree(db); hipFree(dout);
  return o;
}

int main() {
  float a[16], b[16];
  // case 1: C = 2^24, 16 products of 0.5: sequential RNE gives 2^24, exact gives 2^24 + 8
  for (int i = 0; i < 16; ++i) { a[i] = 1.0f; b[i] = 0.5f; }
  printf("case1 C=2^24 + 16*0.5 : got %.1f  (exact %.1f, sequential %.1f)\n", run(a, b, 16777216.0f), 16777224.0, 16777216.0);
  // case 2: C = 1, two products 2^-24
  memset(a, 0, sizeof a); memset(b, 0, sizeof b);
  a[0] = a[1] = 1.0f / 4096; b[0] = b[1] = 1.0f / 4096;
  float o = run(a, b, 1.0f);
  printf("case2 1 + 2*2^-24 : got 1 + %.3g ulp(2^-23)\n", (o - 1.0f) / 1.1920929e-07f);
  // case 3: C = 0, products 2^12 and -2^12 and 2^-12*2^-12 : exact 2^-24
  memset(a, 0, sizeof a); memset(b, 0, sizeof b);
  a[0] = 4096; b[0] = 1; a[1] = -4096; b[1] = 1; a[2] = 1.0f / 4096; b[2] = 1.0f / 4096;
  printf("case3 4096-4096+2^-24 : got %.6g (exact %.6g)\n", run(a, b, 0.0f), 5.9604645e-08);
  // case 4: C = 2^24, product +1 at k=0 then -1 ... 15 products of 1: exact 2^24+15 -> RNE(2^24+15)=2^24+16
  for (int i = 0; i < 16; ++i) { a[i] = 1.0f; b[i] = 1.0f; }
  a[0] = 0; 
  printf("case4 2^24 + 15*1 : got %.1f (exact-once %.1f; sequential %.1f)\n", run(a, b, 16777216.0f), 16777232.0, 16777216.0);
  // case 5: products only, large cancellation: 2048*2048 - 2048*2048 + 1*2^-14 (C = 0)
  memset(a, 0, sizeof a); memset(b, 0, sizeof b);
  a[0] = 2048; b[0] = 2048; a[5] = -2048; b[5] = 2048; a[9] = 1; b[9] = 1.0f / 16384;
  printf("case5 2^22-2^22+2^-14 : got %.6g (exact %.6g)\n", run(a, b, 0.0f), 1.0 / 16384);
  // case 6: C = 1, product 2^-25 * 3 (three products of 2^-25 each... use 2^-12*2^-13)
  memset(a, 0, sizeof a); memset(b, 0, sizeof b);
  for (int i = 0; i < 3; ++i) { a[i] = 1.0f / 4096; b[i] = 1.0f / 8192; }
  o = run(a, b, 1.0f);
  printf("case6 1 + 3*2^-25 : got 1 + %.3g ulp (exact-once 1 ulp, truncating 0)\n", (o - 1.0f) / 1.1920929e-07f);
  // case 7: C = 1, products -2^-25 (one): RNE exact-once -> 1 (tie to even? 1-2^-25: ulp below 1 is 2^-24 -> 1-2^-25 is a tie between 1 and 1-2^-24 -> even=1)
  memset(a, 0, sizeof a); memset(b, 0, sizeof b);
  a[0] = -1.0f / 4096; b[0] = 1.0f / 8192; a[1] = -1.0f / 4096; b[1] = 1.0f / 8192; a[2] = -1.0f/4096; b[2] = 1.0f/8192;
  o = run(a, b, 1.0f);
  printf("case7 1 - 3*2^-25 : got 1 - %.4g * 2^-24 (RNE once: 1 or 2 ; trunc toward 0: 2; sequential: 0)\n", (1.0f - o) / 5.9604645e-08f);
  return 0;
}
