// Microbenchmark (not part of the library): the global-vector solve's history pass alone --
// dava::wide_direction<GT, 8, STAGED> from csrc/bfgs_solve.hip (C5: P = 12,381, GT = 7 float4 groups per
// thread, eight waves, one workgroup per problem) -- run back to back over a history that grows by one
// entry per "iteration", as the solve does, with nothing else on the CU.  STAGED = the solve's XL form
// (rows HBM -> LDS by global_load_lds one entry ahead; with 3 row slots 1.5 entries ahead, the LDS the
// solve's x would have to give up); otherwise the rows go to registers.  B = 1 / 16
// / 256 workgroups: one CU alone, a few, every CU.  Prints ms and GB/s of history rows read, and the time
// per entry.  The question it answers: what bounds the C5 history phase (≈ 4.6 us per 99 KB entry in
// the solve at B = 256).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I../../include
//        -I../../deep-attention-visual-odometry_amd/csrc wide_pass_stream.hip -o wide_pass_stream
#define DAVA_DEVICE_PASSES_ONLY 1  // the device passes only, not the solve kernels and host API
#include "../../deep-attention-visual-odometry_amd/csrc/bfgs_solve.hip"

#include <cstdio>
#include <cstdlib>

namespace micro {
using namespace dava;

constexpr int kNW = 8;
constexpr int kGT = 7;

// per problem in HBM: S rows, W rows (kcap x Pv each), then g, gp, s vectors (Pv each)
// layout 0: per problem [S rows | W rows | g gp s], problems `stride` floats apart;
// layout 1 (entry-major): S row j of problem b at (j B + b) Pv, W rows after all S rows, vectors after those
template <bool STAGED, int RS>
__global__ __launch_bounds__(64 * kNW, 1) void wide_kernel(float* __restrict__ ws, int P, int Pv, int kcap,
                                                           int iters, float* out, size_t stride, int layout) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* d = lds;                 // the stage: RS rows (Pv each; the solve's XL form: d and the gradient slot)
  float* hrho = lds + RS * Pv;    // kcap
  float* hc = hrho + kcap;        // kcap
  float* scratch = hc + kcap;     // 2 * NW * 32
  float *S, *W, *g;
  size_t rs = Pv;  // row stride
  if (layout == 0) {
    S = ws + (size_t)blockIdx.x * stride;
    W = S + (size_t)kcap * Pv;
    g = W + (size_t)kcap * Pv;
  } else {
    S = ws + (size_t)blockIdx.x * Pv;
    W = ws + (size_t)kcap * gridDim.x * Pv + (size_t)blockIdx.x * Pv;
    g = ws + 2 * (size_t)kcap * gridDim.x * Pv + (size_t)blockIdx.x * 3 * Pv;
    rs = (size_t)gridDim.x * Pv;
  }
  float* gp = g + Pv;
  float* s = gp + Pv;
  for (int i = threadIdx.x; i < kcap; i += 64 * kNW) { hrho[i] = 0.5f; hc[i] = 1.25f; }
  __syncthreads();
  int buf = 0;
  float acc = 0.f;
  for (int it = 1; it <= iters; ++it) {
    const int nh = it - 1 < kcap ? it - 1 : kcap - 1;
    // appends go to entry nh (rewritten every iteration once the history is full)
    acc += wide_direction<kGT, kNW, STAGED, RS>(P, Pv, nh, S, W, hrho, hc, 1.0f, g, gp, s, d, S + (size_t)nh * rs,
                                                W + (size_t)nh * rs, scratch, buf, nh, nullptr, nullptr,
                                                STAGED ? lds : nullptr, rs);
    __syncthreads();
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;  // keep the work
}

__global__ void fill(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = 1e-4f * (float)((i * 2654435761u) % 1000u) - 0.05f;
}

template <bool STAGED, int RS = 2>
void run(const char* tag, float* ws, int B, int P, int Pv, int kcap, int iters, float* out, size_t stride, int layout) {
  const int lds = (RS * Pv + 2 * kcap + 2 * kNW * 32) * 4;
  const auto k = wide_kernel<STAGED, RS>;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(k, dim3(B), dim3(64 * kNW), lds, 0, ws, P, Pv, kcap, iters, out, stride, layout);
  const int reps = 3;
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(B), dim3(64 * kNW), lds, 0, ws, P, Pv, kcap, iters, out, stride, layout);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float t;
    (void)hipEventElapsedTime(&t, a, b);
    best = t < best ? t : best;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
  }
  double entries = 0;
  for (int it = 1; it <= iters; ++it) entries += it - 1 < kcap ? it - 1 : kcap - 1;
  const double bytes = entries * 2.0 * Pv * 4.0 * B;
  printf("%-22s B=%4d P=%5d: %8.3f ms  %7.1f GB/s  (%.1f GB/s per CU in use; %.2f us per entry)\n", tag, B, P, best,
         bytes / best / 1e6, bytes / best / 1e6 / (B < 256 ? B : 256), best * 1e3 / entries);
}
}  // namespace micro

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 12381;  // C5: 16 views x 4096 points
  // argv[2]: iterations (the history's footprint: 2 (iters - 1) Pv floats per problem), default the solve's 100
  const int iters = argc > 2 ? atoi(argv[2]) : 100, kcap = iters - 1;
  const int Pv = (P + 3) / 4 * 4;
  if ((Pv / 4 + 511) / 512 != micro::kGT) {
    printf("P = %d needs %d groups per thread, this build has %d\n", P, (Pv / 4 + 511) / 512, micro::kGT);
    return 1;
  }
  const int Bmax = 256;
  float *ws, *out;
  const size_t per = 2 * (size_t)kcap * Pv + 3 * (size_t)Pv;
  const size_t pad = 3328;  // floats: 13 KB, an odd multiple of 256 B
  if (hipMalloc(&ws, Bmax * (per + pad) * 4) != hipSuccess || hipMalloc(&out, Bmax * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(micro::fill, dim3(4096), dim3(256), 0, 0, ws, Bmax * (per + pad));
  if (argc > 2) {  // footprint scan: B = 256 only
    micro::run<true, 2>("staged, problem-major", ws, 256, P, Pv, kcap, iters, out, per, 0);
    micro::run<false>("registers", ws, 256, P, Pv, kcap, iters, out, per, 0);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
  }
  for (int B : {1, 64, 256}) {
#if DAVA_MICRO_NOSYNC
    micro::run<true, 2>("staged, NO block sum", ws, B, P, Pv, kcap, iters, out, per, 0);
    continue;
#endif
    micro::run<true, 2>("staged, problem-major", ws, B, P, Pv, kcap, iters, out, per, 0);
    micro::run<true, 2>("staged, padded stride", ws, B, P, Pv, kcap, iters, out, per + pad, 0);
    micro::run<true, 2>("staged, entry-major", ws, B, P, Pv, kcap, iters, out, per, 1);
    if (B == 256) micro::run<false>("registers, entry-major", ws, B, P, Pv, kcap, iters, out, per, 1);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  hipFree(ws);
  hipFree(out);
  return 0;
}
