// Probe: cycles per v_mfma_f32_32x32x16_f16 in the fused kernel's block
// structure (dependent 12-MFMA chains), A operand in AGPRs vs VGPRs, one
// wave per SIMD.  Build with -mllvm -amdgpu-mfma-vgpr-form.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NB, bool AGPR, int CHAINS, bool INDEP = false>
__global__ __launch_bounds__(256, 1) void chain(const f16x8* img, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  f16x8 A[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int t = 0; t < 4; ++t) A[b][t] = img[(b * 4 + t) * 64 + lane];
  f16x8 bv[4];
  for (int t = 0; t < 4; ++t)
    for (int e = 0; e < 8; ++e) bv[t][e] = (_Float16)(0.001f * (lane + e + t));
  float sink = 0.0f;
  for (int it = 0; it < iters; ++it) {
    if constexpr (AGPR) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int t = 0; t < 4; ++t) asm volatile("" : "+a"(A[b][t]));
    }
#pragma unroll
    for (int b = 0; b < NB; b += CHAINS) {
      f32x16 acc[CHAINS];
#pragma unroll
      for (int c = 0; c < CHAINS; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[c][i] = INDEP ? 0.0f : sink;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rep = 0; rep < 3; ++rep)
#pragma unroll
          for (int c = 0; c < CHAINS; ++c)
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[b + c][t], bv[(t + rep) & 3], acc[c], 0, 0, 0);
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) sink = INDEP ? fmaxf(sink, acc[c][b & 15]) : sink + acc[c][0] * 1e-30f;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = sink;
}

template <int NB, bool AGPR, int CHAINS, bool INDEP = false>
static void run(const f16x8* img, float* out, int n_cu, const char* name) {
  const int iters = 400;
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  hipLaunchKernelGGL((chain<NB, AGPR, CHAINS, INDEP>), dim3(n_cu), dim3(256), 0, 0, img, out, iters);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((chain<NB, AGPR, CHAINS, INDEP>), dim3(n_cu), dim3(256), 0, 0, img, out, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  const double n_mfma = (double)iters * NB * 12;
  printf("%-28s %.3f ms  %.2f ns/MFMA  (%.1f cyc @2.1GHz)\n", name, ms, ms * 1e6 / n_mfma, ms * 1e6 / n_mfma * 2.1);
}

int main() {
  int n_cu = 0;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  f16x8* img; float* out;
  (void)hipMalloc(&img, sizeof(f16x8) * 64 * 64);
  (void)hipMemset(img, 0, sizeof(f16x8) * 64 * 64);
  (void)hipMalloc(&out, sizeof(float) * n_cu * 256);
  run<8, true, 1>(img, out, n_cu, "AGPR A, 1 chain");
  run<8, true, 2>(img, out, n_cu, "AGPR A, 2 chains");
  run<8, false, 1>(img, out, n_cu, "VGPR A, 1 chain");
  run<8, false, 2>(img, out, n_cu, "VGPR A, 2 chains");
  run<4, false, 1>(img, out, n_cu, "VGPR A (4 blk), 1 chain");
  run<8, true, 1, true>(img, out, n_cu, "AGPR A, indep blocks");
  run<8, true, 2, true>(img, out, n_cu, "AGPR A, indep, 2 chains");
  return 0;
}
