// Microbenchmark (not part of the library): the LDS-mode solve's own history pass,
// dava::compact_products_fused<GM, NW> from csrc/bfgs_solve.hip, run back to back over a history that
// grows by one entry per "iteration" -- the memory pattern of tools/micro/history_stream.hip, but with
// the solve's code (buffer loads, per-entry coefficient reads, priority drop, deferred cross-wave
// combine) instead of a stand-in loop.  Next to it the stand-in loop's kernel is rebuilt here on the
// same (non-zero) rows, so the two rates compare directly.  Prints GB/s of history rows read.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I../../include
//        -I../../deep-attention-visual-odometry_amd/csrc solve_pass_stream.hip -o solve_pass_stream
#define DAVA_DEVICE_PASSES_ONLY 1  // the device passes only, not the solve kernels and host API
#include "../../deep-attention-visual-odometry_amd/csrc/bfgs_solve.hip"

#include <cstdio>
#include <cstdlib>
#include <string>

namespace micro {
using namespace dava;

// LDS image: g, gp, a_out, b_out, spare0..3 (Pv floats each), hrho, hc (kcap each), LDS history (lcap entries)
template <int GM, int NW>
__global__ __launch_bounds__(64 * NW) void solve_pass_kernel(const float* __restrict__ hist, int P, int Pv, int kcap,
                                                             int iters, int lcap, float* out) {
  extern __shared__ float lds[];
  float* g = lds;
  float* gp = g + Pv;
  float* ao = gp + Pv;
  float* bo = ao + Pv;
  float* s0 = bo + Pv;
  float* s1 = s0 + Pv;
  float* s2 = s1 + Pv;
  float* s3 = s2 + Pv;
  float* hrho = s3 + Pv;
  float* hc = hrho + kcap;
  float* LH = hc + kcap;
  const float* S = hist + (size_t)blockIdx.x * 2 * kcap * Pv;
  const float* W = S + (size_t)kcap * Pv;
  for (int i = threadIdx.x; i < Pv; i += 64 * NW) {
    g[i] = i < P ? 1e-3f * (i % 7) : 0.f;
    gp[i] = i < P ? 2e-3f * (i % 5) : 0.f;
  }
  for (int i = threadIdx.x; i < kcap; i += 64 * NW) { hrho[i] = 0.5f; hc[i] = 1.25f; }
  for (int i = threadIdx.x; i < 2 * lcap * Pv; i += 64 * NW) LH[i] = 1e-4f;
  __syncthreads();
  for (int it = 1; it <= iters; ++it) {
    const int nh = it < kcap ? it : kcap;
    compact_products_fused<GM, NW>(P, Pv, nh, S, W, LH, lcap, hrho, hc, 1.0f, g, gp, ao, bo, s0, s1, s2, s3);
    __syncthreads();
  }
  float t = 0;
  for (int i = threadIdx.x; i < Pv; i += 64 * NW) t += s0[i] + s2[i] + s1[i] + s3[i];
  if (t == 12345.f) out[blockIdx.x * 64 * NW + threadIdx.x] = t;  // keep the work
}

__global__ void fill(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = 1e-3f * (float)((i * 2654435761u) % 1000u) - 0.5f;
}

template <int GM, int NW>
void run(const char* tag, const float* hist, int B, int P, int Pv, int kcap, int iters, int lcap, float* out) {
  const int lds = (8 * Pv + 2 * kcap + 2 * lcap * Pv) * 4;
  const auto k = solve_pass_kernel<GM, NW>;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  // one warm-up launch, then `reps` launches timed one by one: the best is the ceiling (boxes and runs
  // differ by a few per cent; the mean is printed beside it)
  hipLaunchKernelGGL(k, dim3(B), dim3(64 * NW), lds, 0, hist, P, Pv, kcap, iters, lcap, out);
  const int reps = 8;
  float ms = 1e30f, mean = 0.f;
  for (int r = 0; r < reps; ++r) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(B), dim3(64 * NW), lds, 0, hist, P, Pv, kcap, iters, lcap, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float t;
    (void)hipEventElapsedTime(&t, a, b);
    ms = t < ms ? t : ms;
    mean += t / reps;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
  }
  double entries = 0;  // entries read from HBM (the first lcap come from LDS)
  for (int it = 1; it <= iters; ++it) entries += (it < kcap ? it : kcap) > lcap ? (it < kcap ? it : kcap) - lcap : 0;
  const double bytes = entries * 2.0 * Pv * 4.0 * B;
  printf("%-34s B=%5d P=%5d NW=%d lcap=%d lds=%6d: %8.3f ms  %7.1f GB/s  (%.1f GB/s per CU; best of %d, mean %.3f ms)\n",
         tag, B, P, NW, lcap, lds, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 256, reps, mean);
}
}  // namespace micro

int main(int argc, char** argv) {
  // argv[1] = P.  P <= 512: C2 rows (2 float4 groups per lane, 2 waves per problem), B = 64 / 256 / 1024.
  // P > 512: the headline's rows (C3: P = 794, 4 groups per lane, 4 waves per problem), B = 512 / 2048 / 8192
  // with the solve's 6 LDS-resident entries -- the same resident set (two workgroups per CU) and the same
  // 8 (k - 1 - 6) Pv bytes per problem-iteration the bench line's byte model charges: the rate this access
  // pattern reaches with nothing else on the CU, i.e. the measured ceiling of the headline's history phase.
  const int P = argc > 1 ? atoi(argv[1]) : 396;  // C2: 2 views x 128 points
  const int iters = 100, kcap = 99;
  const int Pv = (P + 3) / 4 * 4;
  const bool c3 = P > 512;
  const int Bmax = c3 ? 8192 : 2048;
  float *hist, *out;
  const size_t n = (size_t)Bmax * 2 * kcap * Pv;
  if (hipMalloc(&hist, n * 4) != hipSuccess || hipMalloc(&out, (size_t)Bmax * 1024 * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(micro::fill, dim3(4096), dim3(256), 0, 0, hist, n);
  if (argc > 2 && std::string(argv[2]) == "ceiling") {  // bench.py's live ceiling: the headline's rows only
    micro::run<4, 4>("C3 rows, 6 entries in LDS", hist, 8192, P, Pv, kcap, iters, 6, out);
  } else if (c3) {
    for (int B : {512, 2048, 8192}) {
      micro::run<4, 4>("C3 rows, all rows in HBM", hist, B, P, Pv, kcap, iters, 0, out);
      micro::run<4, 4>("C3 rows, 6 entries in LDS", hist, B, P, Pv, kcap, iters, 6, out);
    }
  } else {
    for (int B : {64, 256, 1024}) {
      micro::run<2, 2>("solve pass, all rows in HBM", hist, B, P, Pv, kcap, iters, 0, out);
      micro::run<2, 2>("solve pass, 6 entries in LDS", hist, B, P, Pv, kcap, iters, 6, out);
    }
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  hipFree(hist);
  hipFree(out);
  return 0;
}
