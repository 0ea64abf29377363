// Probe: the fp16 hi/lo split of k_fused done with v_fma_mix{lo,hi}_f16
// (lo = RN_f16(xs - hi), one instruction per element) against the plain
// C++ conversion chain; prints the number of differing lo halves.
//   hipcc --offload-arch=gfx950 -O3 split_mix.hip -o /tmp/split_mix && /tmp/split_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__global__ void k_split(const float* x, int n, float s, uint32_t* ref, uint32_t* mix) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const float xs0 = x[2 * i] * s, xs1 = x[2 * i + 1] * s;
  const f16x2 hp = {(_Float16)xs0, (_Float16)xs1};
  const f16x2 lr = {(_Float16)((float)hp[0] * -1.0f + xs0), (_Float16)((float)hp[1] * -1.0f + xs1)};
  ref[i] = __builtin_bit_cast(uint32_t, lr);
  uint32_t lp;
  asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, -%1, 1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lp)
      : "v"(__builtin_bit_cast(uint32_t, hp)), "v"(xs0), "v"(xs1));
  mix[i] = lp;
}

int main() {
  const int n = 1 << 22;
  std::vector<float> h(n);
  std::mt19937 g(7);
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  std::uniform_int_distribution<int> ex(-30, 14);
  for (int i = 0; i < n; ++i) h[i] = ldexpf(u(g), ex(g));
  float *dx;
  uint32_t *dr, *dm;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dr, n * 2);
  hipMalloc(&dm, n * 2);
  hipMemcpy(dx, h.data(), n * 4, hipMemcpyHostToDevice);
  int bad = 0;
  for (float s : {1.0f, 1024.0f, 0.5f}) {
    hipLaunchKernelGGL(k_split, dim3(n / 512), dim3(256), 0, 0, dx, n, s, dr, dm);
    std::vector<uint32_t> r(n / 2), m(n / 2);
    hipMemcpy(r.data(), dr, n * 2, hipMemcpyDeviceToHost);
    hipMemcpy(m.data(), dm, n * 2, hipMemcpyDeviceToHost);
    int b = 0;
    for (int i = 0; i < n / 2; ++i) b += (r[i] != m[i]);
    printf("scale %g: %d of %d pairs differ\n", s, b, n / 2);
    bad += b;
  }
  printf(bad ? "SPLIT_MIX FAIL\n" : "SPLIT_MIX OK\n");
  return bad ? 1 : 0;
}
