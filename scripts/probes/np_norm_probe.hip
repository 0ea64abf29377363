// Probe: km_exact.h's np_norm on the GPU vs NumPy (scripts/probes/np_norm_probe.py).
// in: X float32 [n][d], C float64 [k][d] (raw files); out: sum and norm per (i, j).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../../assignment--2-group7-distributed-k-means_amd/csrc/km_exact.h"

__global__ void k_probe(const float* X, const double* C, int n, int k, int d, double* sums, double* norms) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * k) return;
  const int i = t / k, j = t % k;
  const float* x = X + (size_t)i * d;
  const double* c = C + (size_t)j * d;
  auto sq = [&](int f) { return km::np_sq(c[f], x[f]); };
  sums[t] = km::np_pw<2>(sq, 0, d);
  norms[t] = km::np_norm(sq, d);
}

int main(int argc, char** argv) {
  if (argc != 6) { fprintf(stderr, "usage: probe X.bin C.bin n k d\n"); return 2; }
  const int n = atoi(argv[3]), k = atoi(argv[4]), d = atoi(argv[5]);
  std::vector<float> X((size_t)n * d);
  std::vector<double> C((size_t)k * d), S((size_t)n * k), N((size_t)n * k);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(X.data(), 4, X.size(), f) != X.size()) return 3;
  fclose(f);
  f = fopen(argv[2], "rb");
  if (!f || fread(C.data(), 8, C.size(), f) != C.size()) return 3;
  fclose(f);
  float* dX; double *dC, *dS, *dN;
  if (hipMalloc(&dX, X.size() * 4) || hipMalloc(&dC, C.size() * 8) || hipMalloc(&dS, S.size() * 8) ||
      hipMalloc(&dN, N.size() * 8)) return 4;
  hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3((n * k + 255) / 256), dim3(256), 0, 0, dX, dC, n, k, d, dS, dN);
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  hipMemcpy(S.data(), dS, S.size() * 8, hipMemcpyDeviceToHost);
  hipMemcpy(N.data(), dN, N.size() * 8, hipMemcpyDeviceToHost);
  f = fopen("gpurun_out/probe_sums.bin", "wb");
  fwrite(S.data(), 8, S.size(), f);
  fclose(f);
  f = fopen("gpurun_out/probe_norms.bin", "wb");
  fwrite(N.data(), 8, N.size(), f);
  fclose(f);
  return 0;
}
