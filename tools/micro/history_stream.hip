// Microbenchmark (not part of the library): the LDS-mode history pass's memory pattern in isolation.
// One workgroup per problem, NW waves, each wave takes entries j = wave, wave + NW, ... of a history
// that grows by one entry per "iteration" (as the solve's does), EF entries in flight per wave, rows
// of GM float4 groups per lane; per entry the four dots, one transposed wave reduction and the two
// accumulations the solve does.  Layouts: 0 = per problem an S block then a W block (the solve's),
// 1 = S_j and W_j adjacent.  Prints GB/s of history rows read.
// usage: history_stream [P] [1: non-zero rows] [x: solve layout only]
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../deep-attention-visual-odometry_amd/csrc
//        -I../../include history_stream.hip -o history_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "dava_common.hpp"

using namespace dava;
typedef float f4v __attribute__((ext_vector_type(4)));

template <int GM, int EF, int NW, int LAYOUT>
__global__ __launch_bounds__(64 * NW) void stream_kernel(const float* __restrict__ hist, int P, int Pv, int kcap,
                                                         int iters, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
  const int G = (P + 3) / 4;
  const float* base = hist + (size_t)blockIdx.x * 2 * kcap * Pv;
  f4v y[GM], g[GM], pa[GM], pb[GM];
  bool ok[GM];
#pragma unroll
  for (int m = 0; m < GM; ++m) {
    ok[m] = m < GM - 1 || lane + 64 * m < G;
    y[m] = f4v{1e-3f * lane, 1.f, 2.f, 3.f};
    g[m] = f4v{1.f, 1e-3f * m, 2.f, 1.f};
    pa[m] = pb[m] = f4v{0, 0, 0, 0};
  }
  __shared__ float red[NW * 4];
  auto srow = [&](int j) { return LAYOUT == 0 ? base + (size_t)j * Pv : base + (size_t)2 * j * Pv; };
  auto wrow = [&](int j) { return LAYOUT == 0 ? base + (size_t)(kcap + j) * Pv : base + (size_t)(2 * j + 1) * Pv; };
  for (int it = 1; it <= iters; ++it) {
    const int nh = it < kcap ? it : kcap;
    int j = wave;
    for (; j + (EF - 1) * NW < nh; j += EF * NW) {
      f4v s[EF][GM], w[EF][GM];
#pragma unroll
      for (int e = 0; e < EF; ++e)
#pragma unroll
        for (int m = 0; m < GM; ++m) {
          const int q = lane + 64 * m;
          s[e][m] = ok[m] ? *reinterpret_cast<const f4v*>(srow(j + e * NW) + 4 * q) : f4v{0, 0, 0, 0};
          w[e][m] = ok[m] ? *reinterpret_cast<const f4v*>(wrow(j + e * NW) + 4 * q) : f4v{0, 0, 0, 0};
        }
#pragma unroll
      for (int e = 0; e < EF; ++e) {
        float a = 0, b = 0, c = 0, d = 0;
#pragma unroll
        for (int m = 0; m < GM; ++m)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            a += s[e][m][t] * y[m][t]; b += w[e][m][t] * y[m][t];
            c += s[e][m][t] * g[m][t]; d += w[e][m][t] * g[m][t];
          }
        const float4 r = wave_sum4(a, b, c, d);
#pragma unroll
        for (int m = 0; m < GM; ++m) {
          pa[m] += r.x * s[e][m] + r.y * w[e][m];
          pb[m] += r.z * s[e][m] + r.w * w[e][m];
        }
      }
    }
    for (; j < nh; j += NW) {
#pragma unroll
      for (int m = 0; m < GM; ++m) {
        const int q = lane + 64 * m;
        const f4v s = ok[m] ? *reinterpret_cast<const f4v*>(srow(j) + 4 * q) : f4v{0, 0, 0, 0};
        const f4v w = ok[m] ? *reinterpret_cast<const f4v*>(wrow(j) + 4 * q) : f4v{0, 0, 0, 0};
        pa[m] += 1e-3f * s;
        pb[m] += 1e-3f * w;
      }
    }
    // the rest of an iteration: one block reduction
    if (lane == 0) red[wave * 4] = pa[0][0];
    __syncthreads();
    if (threadIdx.x == 0) { float t = 0; for (int i = 0; i < NW; ++i) t += red[4 * i]; pa[0][0] += 1e-9f * t; }
    __syncthreads();
  }
  float t = 0;
#pragma unroll
  for (int m = 0; m < GM; ++m) t += pa[m][0] + pa[m][1] + pb[m][2] + pb[m][3];
  if (t == 12345.f) out[blockIdx.x * 64 * NW + threadIdx.x] = t;  // keep the work
}

__global__ void fill_rows(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = 1e-3f * (float)((i * 2654435761u) % 1000u) - 0.5f;
}

template <int GM, int EF, int NW, int LAYOUT>
void run(const char* tag, const float* hist, int B, int P, int Pv, int kcap, int iters, float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  stream_kernel<GM, EF, NW, LAYOUT><<<B, 64 * NW>>>(hist, P, Pv, kcap, iters, out);
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) stream_kernel<GM, EF, NW, LAYOUT><<<B, 64 * NW>>>(hist, P, Pv, kcap, iters, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= reps;
  double entries = 0;
  for (int it = 1; it <= iters; ++it) entries += it < kcap ? it : kcap;
  const double bytes = entries * 2.0 * P * 4.0 * B;
  printf("%-28s B=%5d P=%5d NW=%d EF=%d layout=%d: %8.3f ms  %7.1f GB/s  (%.1f GB/s per CU)\n", tag, B, P, NW, EF,
         LAYOUT, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 256);
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 399;
  const int iters = 100, kcap = 101;
  const int Pv = (P + 3) / 4 * 4;
  const int Bmax = 4096;
  float *hist, *out;
  hipMalloc(&hist, (size_t)Bmax * 2 * kcap * Pv * 4);
  hipMemset(hist, 0, (size_t)Bmax * 2 * kcap * Pv * 4);
  if (argc > 2 && atoi(argv[2]) == 1) {  // non-zero rows (the solve's rows are never all zero)
    const size_t n = (size_t)Bmax * 2 * kcap * Pv;
    hipLaunchKernelGGL(fill_rows, dim3(4096), dim3(256), 0, 0, hist, n);
  }
  hipMalloc(&out, (size_t)Bmax * 1024 * 4);
  for (int B : {64, 256, 512, 1024, 2048}) {
    run<2, 4, 2, 0>("c2 pass (solve layout)", hist, B, P, Pv, kcap, iters, out);
    if (argc > 3) continue;  // the solve layout only
    run<2, 4, 2, 1>("c2 pass (S_j W_j adjacent)", hist, B, P, Pv, kcap, iters, out);
    run<2, 8, 2, 0>("c2 pass EF 8", hist, B, P, Pv, kcap, iters, out);
    run<2, 4, 1, 0>("c2 pass one wave", hist, B, P, Pv, kcap, iters, out);
    run<2, 4, 4, 0>("c2 pass four waves", hist, B, P, Pv, kcap, iters, out);
  }
  hipFree(hist); hipFree(out);
  return 0;
}
