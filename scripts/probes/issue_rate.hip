// Probe: VALU issue rate and MFMA+VALU overlap vs waves per SIMD (gfx950).
// Inline-asm streams: per slot one v_mfma_f32_32x32x16_f16 (optional) + NV
// independent v_med3_f32 (16 rotating destinations).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define MED(i) "v_med3_f32 %" #i ", %" #i ", %16, %17\n"
template <int NV, int MF>
__global__ __launch_bounds__(512) void mix(float* out, int iters) {
  f16x8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = (_Float16)(threadIdx.x * 0.001f + e); b[e] = (_Float16)(e * 0.5f); }
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  float k0 = 1, k1 = 2, k2 = 3, k3 = 4, k4 = 5, k5 = 6, k6 = 7, k7 = 8, k8 = 9, k9 = 10, k10 = 11, k11 = 12,
        k12 = 13, k13 = 14, k14 = 15, k15 = 16;
  const float x = threadIdx.x * 1e-3f, y = 0.5f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if constexpr (MF) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
      if constexpr (NV >= 4)
        asm volatile(MED(0) MED(1) MED(2) MED(3)
                     : "+v"(k0), "+v"(k1), "+v"(k2), "+v"(k3), "+v"(k4), "+v"(k5), "+v"(k6), "+v"(k7), "+v"(k8),
                       "+v"(k9), "+v"(k10), "+v"(k11), "+v"(k12), "+v"(k13), "+v"(k14), "+v"(k15)
                     : "v"(x), "v"(y));
      if constexpr (NV >= 8)
        asm volatile(MED(4) MED(5) MED(6) MED(7)
                     : "+v"(k0), "+v"(k1), "+v"(k2), "+v"(k3), "+v"(k4), "+v"(k5), "+v"(k6), "+v"(k7), "+v"(k8),
                       "+v"(k9), "+v"(k10), "+v"(k11), "+v"(k12), "+v"(k13), "+v"(k14), "+v"(k15)
                     : "v"(x), "v"(y));
      if constexpr (NV >= 12)
        asm volatile(MED(8) MED(9) MED(10) MED(11)
                     : "+v"(k0), "+v"(k1), "+v"(k2), "+v"(k3), "+v"(k4), "+v"(k5), "+v"(k6), "+v"(k7), "+v"(k8),
                       "+v"(k9), "+v"(k10), "+v"(k11), "+v"(k12), "+v"(k13), "+v"(k14), "+v"(k15)
                     : "v"(x), "v"(y));
      if constexpr (NV >= 16)
        asm volatile(MED(12) MED(13) MED(14) MED(15)
                     : "+v"(k0), "+v"(k1), "+v"(k2), "+v"(k3), "+v"(k4), "+v"(k5), "+v"(k6), "+v"(k7), "+v"(k8),
                       "+v"(k9), "+v"(k10), "+v"(k11), "+v"(k12), "+v"(k13), "+v"(k14), "+v"(k15)
                     : "v"(x), "v"(y));
    }
  }
  float s = k0 + k1 + k2 + k3 + k4 + k5 + k6 + k7 + k8 + k9 + k10 + k11 + k12 + k13 + k14 + k15;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NV, int MF>
static void run(int wps, float* out, int n_cu) {
  const int iters = 4000;
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  hipLaunchKernelGGL((mix<NV, MF>), dim3(n_cu), dim3(256 * wps), 0, 0, out, iters);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((mix<NV, MF>), dim3(n_cu), dim3(256 * wps), 0, 0, out, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  const double ns_slot = ms * 1e6 / (iters * 8.0);  // SIMD time per slot (all waves of the SIMD)
  printf("waves/SIMD=%d mfma=%d NV=%2d : SIMD time per slot-round %.2f ns = %.1f cyc@2.1G (per wave-slot %.1f cyc)\n",
         wps, MF, NV, ns_slot, ns_slot * 2.1, ns_slot * 2.1 / wps);
}

int main() {
  int n_cu = 0;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out; (void)hipMalloc(&out, sizeof(float) * n_cu * 512 * 2);
  for (int w = 1; w <= 2; ++w) {
    run<0, 1>(w, out, n_cu);
    run<8, 0>(w, out, n_cu);
    run<16, 0>(w, out, n_cu);
    run<4, 1>(w, out, n_cu);
    run<8, 1>(w, out, n_cu);
    run<12, 1>(w, out, n_cu);
    run<16, 1>(w, out, n_cu);
  }
  return 0;
}
