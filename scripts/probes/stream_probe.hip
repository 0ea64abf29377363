// Probe: HBM streaming rate of k_s1's row-tile load pattern (gfx950).
// X = 100M rows x 64 floats (25.6 GB, the c3 workload).  One workgroup per
// CU of W waves, each wave walks 16-row tiles (4 KiB) with NBUF register
// buffers (NBUF - 1 tiles in flight while one is consumed), then V dependent
// VALU operations per tile on the loaded values (the screen's work stand-in).
// Patterns of the four float4 loads per lane:
//   0: k_s1 today -- lane (q = lane / 16, r = lane % 16) reads row r, bytes
//      64 q + 16 u (u = 0..3): 16 rows x 4 scattered 16-B pieces per load
//   1: row-contiguous -- lane (q, r) reads row r, bytes 64 u + 16 q: each
//      load takes 64 contiguous bytes of every row
//   2: lane-linear -- load u reads bytes 1024 u + 16 lane of the tile
//      (fully coalesced 1 KiB per instruction)
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

template <int W, int NBUF, int PAT, int V>
__global__ __launch_bounds__(W * 64) void stream(const float4* __restrict__ X, uint32_t ntiles, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, r = lane & 15;
  const uint32_t gw = blockIdx.x * W + wave, nw = gridDim.x * W;
  auto off = [&](uint32_t tile, int u) -> size_t {
    const size_t base = (size_t)tile * 256;  // float4 units: 16 rows x 16 float4
    if (PAT == 0) return base + r * 16 + q * 4 + u;
    if (PAT == 1) return base + r * 16 + u * 4 + q;
    return base + u * 64 + lane;
  };
  float4 b[NBUF][4];
  float acc = 0.0f;
  auto load = [&](uint32_t tile, float4 (&B)[4]) {
    const uint32_t t = tile < ntiles ? tile : ntiles - 1;
#pragma unroll
    for (int u = 0; u < 4; ++u) B[u] = X[off(t, u)];
  };
  auto work = [&](const float4 (&B)[4]) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[4 * u] = B[u].x;
      v[4 * u + 1] = B[u].y;
      v[4 * u + 2] = B[u].z;
      v[4 * u + 3] = B[u].w;
    }
#pragma unroll
    for (int i = 0; i < V / 16; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = fmaf(v[j], 1.0001f, 0.5f);
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += v[j];
    acc += s;
  };
#pragma unroll
  for (int u = 0; u + 1 < NBUF; ++u) load(gw + u * nw, b[u]);
  for (uint32_t st = gw; st < ntiles; st += NBUF * nw) {
    bool done = false;
#pragma unroll
    for (int u = 0; u < NBUF; ++u) {
      if (!done) {
        load(st + (u + NBUF - 1) * nw, b[(u + NBUF - 1) % NBUF]);
        work(b[u]);
        done = st + (u + 1) * nw >= ntiles;
      }
    }
    if (done) break;
  }
  out[blockIdx.x * W * 64 + threadIdx.x] = acc;
}

template <int W, int NBUF, int PAT, int V>
void run(const float4* X, uint32_t ntiles, float* out, int ncu, double bytes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float best = 1e30f, tot = 0.0f;
  const int reps = 5;
  for (int i = 0; i < reps + 1; ++i) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((stream<W, NBUF, PAT, V>), dim3(ncu), dim3(W * 64), 0, 0, X, ntiles, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (i > 0) {
      tot += ms;
      if (ms < best) best = ms;
    }
  }
  printf("waves %2d nbuf %d pattern %d valu %4d: avg %.3f ms best %.3f ms  %.0f GB/s\n", W, NBUF, PAT, V,
         tot / reps, best, bytes / (tot / reps) / 1e6);
  fflush(stdout);
}

int main() {
  const uint32_t rows = 100000000u, ntiles = rows / 16;
  const double bytes = (double)rows * 256.0;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  float4* X;
  float* out;
  CHECK(hipMalloc(&X, (size_t)bytes));
  CHECK(hipMemset(X, 0x3c, (size_t)bytes));
  CHECK(hipMalloc(&out, sizeof(float) * p.multiProcessorCount * 16 * 64));
  const int ncu = p.multiProcessorCount;
  run<8, 2, 0, 0>(X, ntiles, out, ncu, bytes);
  run<8, 2, 1, 0>(X, ntiles, out, ncu, bytes);
  run<8, 2, 2, 0>(X, ntiles, out, ncu, bytes);
  run<12, 2, 0, 0>(X, ntiles, out, ncu, bytes);
  run<12, 2, 1, 0>(X, ntiles, out, ncu, bytes);
  run<8, 3, 0, 0>(X, ntiles, out, ncu, bytes);
  run<8, 4, 0, 0>(X, ntiles, out, ncu, bytes);
  run<16, 2, 0, 0>(X, ntiles, out, ncu, bytes);
  run<16, 3, 2, 0>(X, ntiles, out, ncu, bytes);
  // with a compute stand-in per tile (the screen spends ~1,000-2,000 cycles
  // per tile and wave)
  run<8, 2, 0, 256>(X, ntiles, out, ncu, bytes);
  run<12, 2, 0, 256>(X, ntiles, out, ncu, bytes);
  run<8, 3, 0, 256>(X, ntiles, out, ncu, bytes);
  run<8, 4, 0, 256>(X, ntiles, out, ncu, bytes);
  run<12, 3, 0, 256>(X, ntiles, out, ncu, bytes);
  run<8, 2, 1, 256>(X, ntiles, out, ncu, bytes);
  run<12, 2, 1, 256>(X, ntiles, out, ncu, bytes);
  run<8, 2, 0, 512>(X, ntiles, out, ncu, bytes);
  run<12, 2, 0, 512>(X, ntiles, out, ncu, bytes);
  run<8, 4, 0, 512>(X, ntiles, out, ncu, bytes);
  run<12, 3, 0, 512>(X, ntiles, out, ncu, bytes);
  CHECK(hipFree(X));
  CHECK(hipFree(out));
  return 0;
}
