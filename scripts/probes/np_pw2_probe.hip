// Probe: km_exact.h's lockstep np_pw2 (two points per centroid read) on the
// GPU vs NumPy's pairwise sums (scripts/probes/np_pw2_probe.py).
// in: X float32 [n][d] (n even), C float64 [k][d]; out: sums [n][k].
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../../assignment--2-group7-distributed-k-means_amd/csrc/km_exact.h"

__global__ void k_probe(const float* X, const double* C, int n, int k, int d, double* sums) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (n / 2) * k) return;
  const int i = 2 * (t / k), j = t % k;
  const float* xa = X + (size_t)i * d;
  const float* xb = xa + d;
  const double* c = C + (size_t)j * d;
  double sa, sb;
  km::np_pw2<2>(
      [&](int f, double& ta, double& tb) {
        const double cv = c[f];
        ta = km::np_sq(cv, xa[f]);
        tb = km::np_sq(cv, xb[f]);
      },
      0, d, sa, sb);
  sums[(size_t)i * k + j] = sa;
  sums[(size_t)(i + 1) * k + j] = sb;
}

int main(int argc, char** argv) {
  if (argc != 6) { fprintf(stderr, "usage: probe X.bin C.bin n k d\n"); return 2; }
  const int n = atoi(argv[3]), k = atoi(argv[4]), d = atoi(argv[5]);
  std::vector<float> X((size_t)n * d);
  std::vector<double> C((size_t)k * d), S((size_t)n * k);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(X.data(), 4, X.size(), f) != X.size()) return 3;
  fclose(f);
  f = fopen(argv[2], "rb");
  if (!f || fread(C.data(), 8, C.size(), f) != C.size()) return 3;
  fclose(f);
  float* dX; double *dC, *dS;
  if (hipMalloc(&dX, X.size() * 4) || hipMalloc(&dC, C.size() * 8) || hipMalloc(&dS, S.size() * 8)) return 4;
  hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(((n / 2) * k + 255) / 256), dim3(256), 0, 0, dX, dC, n, k, d, dS);
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  hipMemcpy(S.data(), dS, S.size() * 8, hipMemcpyDeviceToHost);
  f = fopen("gpurun_out/pw2_sums.bin", "wb");
  fwrite(S.data(), 8, S.size(), f);
  fclose(f);
  return 0;
}
