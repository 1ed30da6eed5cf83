// Reverse-mode (vector-Jacobian) kernels of the generic BFGS building blocks (fp32, fp64).
//
// The reference differentiates THROUGH its solve when the initial parameters
// require grad (autograd_solvers/bfgs_solver.py:85, :134 create_graph, :213-215):
// autograd then walks back through every inverse-Hessian scale and update,
// every search direction and every closure gradient.  The closure part stays
// in PyTorch (it is the caller's code); the solver's own ops get these HIP
// backward kernels, so the drop-in solver's graph has the same nodes as the
// reference's:
//   dava_bfgs_update_inverse_hessian_backward_*  VJP of bfgs_solver.py:235-303, with
//                                                InverseCurvature's custom backward
//                                                (utils/func_inverse_curvature.py:36-51)
//   dava_bfgs_initial_scale_backward_*           VJP of bfgs_solver.py:217-233
//   dava_bfgs_scale_matrix_backward_*            VJP of the k == 1 rescale (:159-167)
//   dava_bfgs_search_direction_backward_*        VJP of d = -H g (:173-176)
// Every output pointer may be NULL (that gradient is not formed).  One workgroup
// per problem; all matrices are row-major (batch, n, n).
#include "dava_common.hpp"

namespace dava {

template <typename T>
__device__ __forceinline__ T block_total(T v, T* red) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

// A v: one wave per row (coalesced along the row), result to out[i]
template <typename T, typename F>
__device__ __forceinline__ void rows_dot(int64_t n, const T* A, F&& v, T* out) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  for (int64_t i = wave; i < n; i += kWaves) {
    T acc = 0;
    for (int64_t j = lane; j < n; j += kWave) acc += A[i * n + j] * v(j);
    acc = wave_sum(acc);
    if (lane == 0) out[i] = acc;
  }
}

// A^T u: one thread per column (consecutive threads -> consecutive columns)
template <typename T, typename F>
__device__ __forceinline__ void cols_dot(int64_t n, const T* A, F&& u, T* out) {
  for (int64_t j = threadIdx.x; j < n; j += kBlock) {
    T acc = 0;
    for (int64_t i = 0; i < n; ++i) acc += u(i) * A[i * n + j];
    out[j] = acc;
  }
}

// H+ = H + (s r)(s)^T (1 + gip) - (s r)(yH)^T - (Hy)(s r)^T,  yH = y^T H, Hy = H y,
// r = 1/(s.y) (0 if s.y <= 0), gip = yH . (y r).  Given G = dL/dH+:
//   sbar_r = q G s - G yH - G^T Hy,   gipbar = (s r) . G s,   q = 1 + gip
//   yHbar = -G^T (s r) + gipbar (y r),  Hybar = -G (s r)
//   Hbar  = G + y yHbar^T + Hybar y^T
//   rbar  = gipbar (y . yH) + s . sbar_r,  go = -r r rbar   (InverseCurvature)
//   sbar  = q G^T (s r) + r sbar_r + go y
//   ybar  = H yHbar + H^T Hybar + r gipbar yH + go s
// LDS: 9 vectors of n.
template <typename T>
__global__ __launch_bounds__(kBlock) void update_backward_kernel(int64_t n, const T* __restrict__ h,
                                                                 const T* __restrict__ s, const T* __restrict__ y,
                                                                 const T* __restrict__ g, T* __restrict__ gh,
                                                                 T* __restrict__ gs, T* __restrict__ gy) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* yH = reinterpret_cast<T*>(smem);
  T* Hy = yH + n;
  T* Gs = Hy + n;
  T* GyH = Gs + n;
  T* GTsr = GyH + n;
  T* GTHy = GTsr + n;
  T* yHbar = GTHy + n;
  T* t1 = yHbar + n;
  T* t2 = t1 + n;
  __shared__ T red[kWaves];
  const int64_t b = blockIdx.x;
  const T* H = h + b * n * n;
  const T* G = g + b * n * n;
  const T* sv = s + b * n;
  const T* yv = y + b * n;
  const int tid = threadIdx.x;

  cols_dot(n, H, [&](int64_t i) { return yv[i]; }, yH);
  rows_dot(n, H, [&](int64_t j) { return yv[j]; }, Hy);
  T sy = 0;
  for (int64_t i = tid; i < n; i += kBlock) sy += sv[i] * yv[i];
  sy = block_total(sy, red);  // (barriers publish yH / Hy)
  const T r = sy <= T(0) ? T(0) : T(1) / sy;
  T gip = 0, yyh = 0;
  for (int64_t j = tid; j < n; j += kBlock) {
    gip += yH[j] * (yv[j] * r);
    yyh += yv[j] * yH[j];
  }
  gip = block_total(gip, red);
  yyh = block_total(yyh, red);
  const T q = T(1) + gip;

  rows_dot(n, G, [&](int64_t j) { return sv[j]; }, Gs);
  rows_dot(n, G, [&](int64_t j) { return yH[j]; }, GyH);
  cols_dot(n, G, [&](int64_t i) { return sv[i] * r; }, GTsr);
  cols_dot(n, G, [&](int64_t i) { return Hy[i]; }, GTHy);
  __syncthreads();
  T gipbar = 0;
  for (int64_t i = tid; i < n; i += kBlock) gipbar += (sv[i] * r) * Gs[i];
  gipbar = block_total(gipbar, red);
  for (int64_t j = tid; j < n; j += kBlock) yHbar[j] = gipbar * (yv[j] * r) - GTsr[j];
  __syncthreads();
  // Hybar_i = -r Gs_i
  rows_dot(n, H, [&](int64_t j) { return yHbar[j]; }, t1);
  cols_dot(n, H, [&](int64_t i) { return T(-1) * r * Gs[i]; }, t2);
  T rbar = 0;
  for (int64_t i = tid; i < n; i += kBlock) rbar += sv[i] * (q * Gs[i] - GyH[i] - GTHy[i]);
  rbar = block_total(rbar, red) + gipbar * yyh;  // (barriers publish t1 / t2)
  const T go = T(-1) * r * r * rbar;
  for (int64_t i = tid; i < n; i += kBlock) {
    const T sbar_r = q * Gs[i] - GyH[i] - GTHy[i];
    if (gs) gs[b * n + i] = q * GTsr[i] + r * sbar_r + go * yv[i];
    if (gy) gy[b * n + i] = t1[i] + t2[i] + r * gipbar * yH[i] + go * sv[i];
  }
  if (gh) {
    const int lane = tid & (kWave - 1), wave = tid / kWave;
    for (int64_t i = wave; i < n; i += kWaves) {
      const T yi = yv[i], hyb = T(-1) * r * Gs[i];
      for (int64_t j = lane; j < n; j += kWave) gh[b * n * n + i * n + j] = G[i * n + j] + yi * yHbar[j] + hyb * yv[j];
    }
  }
}

// gamma = clamp(num / clamp(den, 1e-5), min 1e-4), num = s.y, den = y.y
template <typename T>
__global__ __launch_bounds__(kBlock) void initial_scale_backward_kernel(int64_t n, const T* s, const T* y,
                                                                        const T* gout, T* gs, T* gy) {
  __shared__ T red[kWaves];
  const int64_t b = blockIdx.x;
  T yy = 0, sy = 0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    const T yi = y[b * n + i];
    yy += yi * yi;
    sy += s[b * n + i] * yi;
  }
  yy = block_total(yy, red);
  sy = block_total(sy, red);
  const T dc = clamp_min(yy, T(1e-5));
  const T t = sy / dc;
  const T tbar = t >= T(1e-4) ? gout[b] : T(0);  // clamp backward passes where input >= min
  const T numbar = tbar / dc;
  const T dcbar = T(-1) * tbar * sy / (dc * dc);
  const T denbar = yy >= T(1e-5) ? dcbar : T(0);
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    const T si = s[b * n + i], yi = y[b * n + i];
    if (gs) gs[b * n + i] = numbar * yi;
    if (gy) gy[b * n + i] = numbar * si + denbar * T(2) * yi;
  }
}

// H' = gamma H:  Hbar = gamma G,  gammabar = sum G o H
template <typename T>
__global__ __launch_bounds__(kBlock) void scale_matrix_backward_kernel(int64_t nn, const T* scale, const T* h,
                                                                       const T* g, T* gscale, T* gh) {
  __shared__ T red[kWaves];
  const int64_t b = blockIdx.x;
  const T gm = scale[b];
  T acc = 0;
  for (int64_t e = threadIdx.x; e < nn; e += kBlock) {
    const T ge = g[b * nn + e];
    if (gscale) acc += ge * h[b * nn + e];
    if (gh) gh[b * nn + e] = gm * ge;
  }
  if (gscale) {
    acc = block_total(acc, red);
    if (threadIdx.x == 0) gscale[b] = acc;
  }
}

// d = -H g:  gbar = -H^T dbar,  Hbar = -dbar g^T
template <typename T>
__global__ __launch_bounds__(kBlock) void search_direction_backward_kernel(int64_t n, const T* h, const T* g,
                                                                          const T* dbar, T* gh, T* gg) {
  const int64_t b = blockIdx.x;
  const T* H = h + b * n * n;
  const T* db = dbar + b * n;
  const T* gv = g + b * n;
  if (gg) cols_dot(n, H, [&](int64_t i) { return T(-1) * db[i]; }, gg + b * n);
  if (gh) {
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    for (int64_t i = wave; i < n; i += kWaves) {
      const T di = T(-1) * db[i];
      for (int64_t j = lane; j < n; j += kWave) gh[b * n * n + i * n + j] = di * gv[j];
    }
  }
}

inline int launched_ok() { return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH; }

constexpr int kUpdateBackwardVectors = 9;

template <typename T>
int update_backward(int64_t batch, int64_t n, const T* h, const T* s, const T* y, const T* g, T* gh, T* gs, T* gy,
                    void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!h || !s || !y || !g) return DAVA_ERR_INVALID_ARGUMENT;
  const size_t lds = kUpdateBackwardVectors * (size_t)n * sizeof(T);
  if (lds > 150 * 1024) return DAVA_ERR_UNSUPPORTED;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(update_backward_kernel<T>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(update_backward_kernel<T>, dim3((unsigned)batch), dim3(kBlock), lds,
                     static_cast<hipStream_t>(stream), n, h, s, y, g, gh, gs, gy);
  return launched_ok();
}

template <typename T>
int initial_scale_backward(int64_t batch, int64_t n, const T* s, const T* y, const T* gout, T* gs, T* gy,
                           void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!s || !y || !gout) return DAVA_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(initial_scale_backward_kernel<T>, dim3((unsigned)batch), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), n, s, y, gout, gs, gy);
  return launched_ok();
}

template <typename T>
int scale_matrix_backward(int64_t batch, int64_t n, const T* scale, const T* h, const T* g, T* gscale, T* gh,
                          void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!scale || !h || !g) return DAVA_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(scale_matrix_backward_kernel<T>, dim3((unsigned)batch), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), n * n, scale, h, g, gscale, gh);
  return launched_ok();
}

template <typename T>
int search_direction_backward(int64_t batch, int64_t n, const T* h, const T* g, const T* dbar, T* gh, T* gg,
                              void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!h || !g || !dbar) return DAVA_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(search_direction_backward_kernel<T>, dim3((unsigned)batch), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), n, h, g, dbar, gh, gg);
  return launched_ok();
}

}  // namespace dava

using namespace dava;

#define DAVA_GRAD_ENTRY_POINTS(SUFFIX, T)                                                                          \
  extern "C" int dava_bfgs_update_inverse_hessian_backward_##SUFFIX(int64_t batch, int64_t n, const T* h,         \
                                                                    const T* s, const T* y, const T* grad_out,    \
                                                                    T* grad_h, T* grad_s, T* grad_y,              \
                                                                    void* stream) {                               \
    return update_backward<T>(batch, n, h, s, y, grad_out, grad_h, grad_s, grad_y, stream);                      \
  }                                                                                                               \
  extern "C" int dava_bfgs_initial_scale_backward_##SUFFIX(int64_t batch, int64_t n, const T* s, const T* y,      \
                                                           const T* grad_out, T* grad_s, T* grad_y,              \
                                                           void* stream) {                                        \
    return initial_scale_backward<T>(batch, n, s, y, grad_out, grad_s, grad_y, stream);                          \
  }                                                                                                               \
  extern "C" int dava_bfgs_scale_matrix_backward_##SUFFIX(int64_t batch, int64_t n, const T* scale, const T* h,  \
                                                          const T* grad_out, T* grad_scale, T* grad_h,           \
                                                          void* stream) {                                         \
    return scale_matrix_backward<T>(batch, n, scale, h, grad_out, grad_scale, grad_h, stream);                   \
  }                                                                                                               \
  extern "C" int dava_bfgs_search_direction_backward_##SUFFIX(int64_t batch, int64_t n, const T* h, const T* g,  \
                                                              const T* grad_d, T* grad_h, T* grad_g,             \
                                                              void* stream) {                                     \
    return search_direction_backward<T>(batch, n, h, g, grad_d, grad_h, grad_g, stream);                         \
  }

DAVA_GRAD_ENTRY_POINTS(f32, float)
DAVA_GRAD_ENTRY_POINTS(f64, double)
