// Generic batched BFGS building blocks on gfx950 (fp32 and fp64).
//
// These serve the drop-in BFGSSolver when the caller's error function is an
// arbitrary Python closure (the reference's general contract,
// autograd_solvers/bfgs_solver.py:80-84): the closure and its gradient run in
// PyTorch on the GPU, everything the solver itself computes runs here.
//   dava_bfgs_update_inverse_hessian_*   bfgs_solver.py:235-303
//   dava_bfgs_initial_scale_*            bfgs_solver.py:217-233
//   dava_bfgs_scale_matrix_*             bfgs_solver.py:159-167
//   dava_bfgs_search_direction_*         bfgs_solver.py:173-176
//   dava_wolfe_{init,propose,update}_*   line_search/wolfe_conditions.py:76-237
#include "dava_common.hpp"

namespace dava {

template <typename T>
__device__ __forceinline__ T block_sum1(T v, T* red) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

// One workgroup per problem.  LDS: yH[n], Hy[n].
template <typename T>
__global__ __launch_bounds__(kBlock) void update_inverse_hessian_kernel(int64_t n, const T* __restrict__ h,
                                                                       const T* __restrict__ s,
                                                                       const T* __restrict__ y, T* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* yH = reinterpret_cast<T*>(smem);
  T* Hy = yH + n;
  __shared__ T red[kWaves];
  const int64_t b = blockIdx.x;
  const T* H = h + b * n * n;
  const T* sv = s + b * n;
  const T* yv = y + b * n;
  T* O = out + b * n * n;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  // y^T H (column sums; consecutive threads -> consecutive columns)
  for (int64_t j = tid; j < n; j += kBlock) {
    T acc = 0;
    for (int64_t i = 0; i < n; ++i) acc += yv[i] * H[i * n + j];
    yH[j] = acc;
  }
  // H y (one wave per row)
  for (int64_t i = wave; i < n; i += kWaves) {
    T acc = 0;
    for (int64_t j = lane; j < n; j += kWave) acc += H[i * n + j] * yv[j];
    acc = wave_sum(acc);
    if (lane == 0) Hy[i] = acc;
  }
  // curvature s.y -> rho (func_inverse_curvature.py:24-28)
  T sy = 0;
  for (int64_t i = tid; i < n; i += kBlock) sy += sv[i] * yv[i];
  sy = block_sum1(sy, red);
  const T rho = sy <= T(0) ? T(0) : T(1) / sy;
  T yhy = 0;  // sum_j yH_j (y_j rho)
  for (int64_t j = tid; j < n; j += kBlock) yhy += yH[j] * (yv[j] * rho);
  yhy = block_sum1(yhy, red);  // (its barriers also publish yH / Hy)
  const T c = T(1) + yhy;
  for (int64_t i = wave; i < n; i += kWaves) {
    const T sri = sv[i] * rho, hyi = Hy[i];
    for (int64_t j = lane; j < n; j += kWave) {
      const T srj = sv[j] * rho;
      T t = H[i * n + j] + (sri * sv[j]) * c;
      t = t - sri * yH[j];
      O[i * n + j] = t - hyi * srj;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void initial_scale_kernel(int64_t n, const T* s, const T* y, T* out) {
  __shared__ T red[kWaves];
  const int64_t b = blockIdx.x;
  T yy = 0, sy = 0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    const T yi = y[b * n + i];
    yy += yi * yi;
    sy += s[b * n + i] * yi;
  }
  yy = block_sum1(yy, red);
  sy = block_sum1(sy, red);
  if (threadIdx.x == 0) out[b] = clamp_min(sy / clamp_min(yy, T(1e-5)), T(1e-4));
}

template <typename T>
__global__ void scale_matrix_kernel(int64_t batch, int64_t nn, const T* scale, const T* h, T* out) {
  const int64_t total = batch * nn;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x)
    out[e] = scale[e / nn] * h[e];
}

template <typename T>
__global__ __launch_bounds__(kBlock) void search_direction_kernel(int64_t n, const T* h, const T* g, T* d) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const T* H = h + b * n * n;
  const T* gv = g + b * n;
  for (int64_t i = wave; i < n; i += kWaves) {
    T acc = 0;
    for (int64_t j = lane; j < n; j += kWave) acc += H[i * n + j] * gv[j];
    acc = wave_sum(acc);
    if (lane == 0) d[b * n + i] = T(-1) * acc;
  }
}

// ---- compact-history search direction for the generic loop (r06) ----
// The generic loop (any closure) used to keep the reference's dense (B, P, P) inverse Hessian and gather /
// scatter it with the active-problem mask every iteration (bfgs_solver.py:157-180).  This op keeps the same
// rank-2 terms as history rows instead -- the fused solve's COMPACT form, exact BFGS in product form:
//   H' v = gamma v + sum_{j < count} [c_j rho_j (s_j . v) - rho_j (w_j . v)] s_j - rho_j (s_j . v) w_j
// and one launch per iteration does, for every active problem r (history slot b = idx[r]):
//   count == 0: gamma = clamp(s.y / clamp(y.y, 1e-5), 1e-4) (bfgs_solver.py:217-233), stored in gamma[b];
//   H'y, H'g from the stored entries (pass 1: each wave reduces its entries' four dots into coefficients in
//   LDS; pass 2: column-parallel accumulation, every row read once more);
//   rho = 1/(s.y) (0 if s.y <= 0, func_inverse_curvature.py:24-28), c = 1 + rho y.H'y;
//   d = -H g with H = H' + c rho s s^T - rho s (H'y)^T - rho (H'y) s^T (the fused kernel's formula order);
//   appends entry `count` = (s, H'y, rho, c).
// Memory O(count P) per problem instead of O(P^2); bytes per iteration 2 x 8 count Pv instead of the dense
// path's ~5 x 4 P^2.  Rows: S, W (B, cap, Pv); rho, c (B, cap); g, y, s, d (n_active, P) contiguous.
template <typename T>
__device__ __forceinline__ T block_sum_n(T v, T* red) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  T t = red[0];
  for (int w = 1; w < (int)(blockDim.x / kWave); ++w) t += red[w];
  return t;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void compact_direction_kernel(int64_t P, int64_t Pv, int64_t cap, int64_t count,
                                                                  const int64_t* __restrict__ idx,
                                                                  const T* __restrict__ g, const T* __restrict__ y,
                                                                  const T* __restrict__ s, T* S, T* W, T* rho, T* cc,
                                                                  T* gamma, T* __restrict__ d) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* yl = reinterpret_cast<T*>(smem);
  T* gl = yl + Pv;
  T* coef = gl + Pv;  // 4 per entry: (a_y, b_y, a_g, b_g)
  __shared__ T red[kWaves];
  const int64_t r = blockIdx.x;
  const int64_t b = idx[r];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const T* gr = g + r * P;
  const T* yr = y + r * P;
  const T* sr = s + r * P;
  T* dr = d + r * P;
  T* Sb = S + b * cap * Pv;
  T* Wb = W + b * cap * Pv;
  for (int64_t i = tid; i < P; i += kBlock) {
    yl[i] = yr[i];
    gl[i] = gr[i];
  }
  __syncthreads();
  // pass 1: per entry, the four dots (s_j.y, s_j.g, w_j.y, w_j.g) -> coefficients, entries dealt to waves
  for (int64_t j = wave; j < count; j += kWaves) {
    const T* sj = Sb + j * Pv;
    const T* wj = Wb + j * Pv;
    T sy = 0, sg = 0, wy = 0, wg = 0;
    for (int64_t i = lane; i < P; i += kWave) {
      const T a = sj[i], w = wj[i], yi = yl[i], gi = gl[i];
      sy += a * yi; sg += a * gi; wy += w * yi; wg += w * gi;
    }
    sy = wave_sum(sy); sg = wave_sum(sg); wy = wave_sum(wy); wg = wave_sum(wg);
    if (lane == 0) {
      const T rj = rho[b * cap + j], cj = cc[b * cap + j];
      coef[4 * j + 0] = cj * rj * sy - rj * wy;
      coef[4 * j + 1] = -rj * sy;
      coef[4 * j + 2] = cj * rj * sg - rj * wg;
      coef[4 * j + 3] = -rj * sg;
    }
  }
  T gm;
  if (count == 0) {  // H_0 = gamma I (bfgs_solver.py:159-167)
    T sy = 0, yy = 0;
    for (int64_t i = tid; i < P; i += kBlock) { sy += sr[i] * yl[i]; yy += yl[i] * yl[i]; }
    sy = block_sum_n(sy, red);
    yy = block_sum_n(yy, red);
    gm = clamp_min(sy / clamp_min(yy, T(1e-5)), T(1e-4));
    if (tid == 0) gamma[b] = gm;
  } else {
    __syncthreads();  // coefficients complete
    gm = gamma[b];
  }
  // pass 2: H'y and H'g column by column (consecutive threads read consecutive columns of every row); H'y is
  // the new entry's w row, H'g is parked in d until the curvature sums are known
  T* wn = Wb + count * Pv;
  T* sn = Sb + count * Pv;
  T r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  for (int64_t i = tid; i < P; i += kBlock) {
    const T yi = yl[i], gi = gl[i], si = sr[i];
    T hy = gm * yi, hg = gm * gi;
    int64_t j = 0;
    for (; j + 4 <= count; j += 4) {  // four entries' loads in flight
      T a[4], w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { a[u] = Sb[(j + u) * Pv + i]; w[u] = Wb[(j + u) * Pv + i]; }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const T* cf = coef + 4 * (j + u);
        hy += cf[0] * a[u] + cf[1] * w[u];
        hg += cf[2] * a[u] + cf[3] * w[u];
      }
    }
    for (; j < count; ++j) {
      const T a = Sb[j * Pv + i], w = Wb[j * Pv + i];
      const T* cf = coef + 4 * j;
      hy += cf[0] * a + cf[1] * w;
      hg += cf[2] * a + cf[3] * w;
    }
    wn[i] = hy;
    sn[i] = si;
    dr[i] = hg;
    r0 += si * yi; r1 += hy * yi; r2 += si * gi; r3 += hy * gi;
  }
  for (int64_t i = P + tid; i < Pv; i += kBlock) { wn[i] = 0; sn[i] = 0; }
  r0 = block_sum_n(r0, red);
  r1 = block_sum_n(r1, red);
  r2 = block_sum_n(r2, red);
  r3 = block_sum_n(r3, red);
  const T rh = r0 <= T(0) ? T(0) : T(1) / r0;
  const T c = T(1) + rh * r1;
  const T sg = r2, hyg = r3, rsg = rh * sg;
  for (int64_t i = tid; i < P; i += kBlock) {  // (each thread reads back what it wrote)
    const T sri = sr[i] * rh;
    dr[i] = T(-1) * (dr[i] + sri * (c * sg) - sri * hyg - wn[i] * rsg);
  }
  if (tid == 0) {
    rho[b * cap + count] = rh;
    cc[b * cap + count] = c;
  }
}

template <typename T>
int compact_direction(int64_t n_active, int64_t P, int64_t Pv, int64_t cap, int64_t count, const int64_t* idx,
                      const T* g, const T* y, const T* s, T* S, T* W, T* rho, T* c, T* gamma, T* d, void* stream) {
  if (n_active < 0 || P < 1 || Pv < P || count < 0 || count >= cap) return DAVA_ERR_INVALID_ARGUMENT;
  if (n_active == 0) return DAVA_OK;
  if (!idx || !g || !y || !s || !S || !W || !rho || !c || !gamma || !d) return DAVA_ERR_INVALID_ARGUMENT;
  const size_t lds = (2 * (size_t)Pv + 4 * (size_t)count) * sizeof(T);
  if (lds > 150 * 1024) return DAVA_ERR_UNSUPPORTED;
  const auto kernel = compact_direction_kernel<T>;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(kernel, dim3((unsigned)n_active), dim3(kBlock), lds, static_cast<hipStream_t>(stream), P, Pv,
                     cap, count, idx, g, y, s, S, W, rho, c, gamma, d);
  return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH;
}

// state columns
enum { S_ALO = 0, S_AHI, S_A, S_FLO, S_FHI, S_FA, S_DFA, S_F0, S_DPHI0, S_COLS };

template <typename T>
__global__ __launch_bounds__(kBlock) void wolfe_init_kernel(int64_t n, const T* dir, const T* f0, const T* g0, T* state,
                                                            uint8_t* flags) {
  __shared__ T red[kWaves];
  const int64_t b = blockIdx.x;
  T acc = 0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) acc += dir[b * n + i] * g0[b * n + i];
  acc = block_sum1(acc, red);
  if (threadIdx.x == 0) {
    T* st = state + b * S_COLS;
    const T f = f0[b];
    st[S_ALO] = 0; st[S_AHI] = 0; st[S_A] = 1;
    st[S_FLO] = f; st[S_FHI] = f; st[S_FA] = f;
    st[S_DFA] = acc; st[S_F0] = f; st[S_DPHI0] = acc;
    flags[b * 2 + 0] = 1;
    flags[b * 2 + 1] = 0;
  }
}

template <typename T>
__global__ void wolfe_propose_kernel(int64_t batch, T* state, const uint8_t* flags) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= batch) return;
  T* st = state + b * S_COLS;
  if (flags[b * 2]) {
    st[S_AHI] = st[S_A];
    st[S_FHI] = st[S_FA];
    st[S_A] = T(2) * st[S_A];
  }
  if (flags[b * 2 + 1]) st[S_A] = T(0.5) * (st[S_ALO] + st[S_AHI]);
}

template <typename T>
__global__ void wolfe_update_kernel(int64_t batch, int trial, T c1, T c2, int strong, T* state, uint8_t* flags) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= batch) return;
  T* st = state + b * S_COLS;
  bool widen = flags[b * 2], zoom = flags[b * 2 + 1];
  T a_lo = st[S_ALO], a_hi = st[S_AHI];
  T f_lo = st[S_FLO], f_hi = st[S_FHI];
  if (widen || zoom) {
    const T a = st[S_A], fa = st[S_FA], dfa = st[S_DFA], f0 = st[S_F0], dphi0 = st[S_DPHI0];
    bool fail = fa > f0 + (c1 * a) * dphi0;
    if (zoom) fail = fail || (fa >= f_lo);
    if (trial > 0 && widen) fail = fail || (fa >= f_hi);
    const T lim = (T(-1) * c2) * dphi0;
    const bool curv = strong ? (fabs(dfa) <= lim) : (T(-1) * dfa <= lim);
    const bool up = widen ? (dfa >= T(0)) : (dfa * (a_hi - a_lo) >= T(0));
    if (zoom) {
      const bool done = !fail && curv, flip = !fail && !curv && up, setlo = !fail && !curv;
      if (fail || done) { a_hi = a; f_hi = fa; }
      if (flip) { a_hi = a_lo; f_hi = f_lo; }
      if (setlo || done) { a_lo = a; f_lo = fa; }
      if (done) zoom = false;
    } else {
      const bool bracket = fail, done = !fail && curv, flip = !fail && !curv && up;
      if (bracket) { a_lo = a_hi; f_lo = f_hi; }
      if (bracket || done) { a_hi = a; f_hi = fa; }
      if (done || flip) { a_lo = a; f_lo = fa; }
      if (bracket || flip) zoom = true;
      if (bracket || done || flip) widen = false;
    }
  }
  if (a_lo == a_hi) zoom = false;
  st[S_ALO] = a_lo; st[S_AHI] = a_hi; st[S_FLO] = f_lo; st[S_FHI] = f_hi;
  flags[b * 2] = widen;
  flags[b * 2 + 1] = zoom;
}

inline int launched() { return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH; }

template <typename T>
int update_inverse_hessian(int64_t batch, int64_t n, const T* h, const T* s, const T* y, T* out, void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!h || !s || !y || !out || out == h) return DAVA_ERR_INVALID_ARGUMENT;
  const size_t lds = 2 * (size_t)n * sizeof(T);
  if (lds > 150 * 1024) return DAVA_ERR_UNSUPPORTED;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(update_inverse_hessian_kernel<T>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(update_inverse_hessian_kernel<T>, dim3((unsigned)batch), dim3(kBlock), lds,
                     static_cast<hipStream_t>(stream), n, h, s, y, out);
  return launched();
}

template <typename T>
int initial_scale(int64_t batch, int64_t n, const T* s, const T* y, T* out, void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0) return DAVA_OK;
  if (!s || !y || !out) return DAVA_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(initial_scale_kernel<T>, dim3((unsigned)batch), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), n, s, y, out);
  return launched();
}

template <typename T>
int scale_matrix(int64_t batch, int64_t n, const T* scale, const T* h, T* out, void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!scale || !h || !out) return DAVA_ERR_INVALID_ARGUMENT;
  const int64_t total = batch * n * n;
  const unsigned grid = (unsigned)((total + kBlock - 1) / kBlock < 4096 ? (total + kBlock - 1) / kBlock : 4096);
  hipLaunchKernelGGL(scale_matrix_kernel<T>, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), batch,
                     n * n, scale, h, out);
  return launched();
}

template <typename T>
int search_direction(int64_t batch, int64_t n, const T* h, const T* g, T* d, void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!h || !g || !d) return DAVA_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(search_direction_kernel<T>, dim3((unsigned)batch), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), n, h, g, d);
  return launched();
}

template <typename T>
int wolfe_init(int64_t batch, int64_t n, const T* dir, const T* f0, const T* g0, T* state, uint8_t* flags,
               void* stream) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0) return DAVA_OK;
  if (!dir || !f0 || !g0 || !state || !flags) return DAVA_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(wolfe_init_kernel<T>, dim3((unsigned)batch), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     n, dir, f0, g0, state, flags);
  return launched();
}

template <typename T>
int wolfe_propose(int64_t batch, T* state, const uint8_t* flags, void* stream) {
  if (batch < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0) return DAVA_OK;
  if (!state || !flags) return DAVA_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(wolfe_propose_kernel<T>, dim3((unsigned)((batch + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), batch, state, flags);
  return launched();
}

template <typename T>
int wolfe_update(int64_t batch, int32_t trial, T c1, T c2, int32_t strong, T* state, uint8_t* flags, void* stream) {
  if (batch < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0) return DAVA_OK;
  if (!state || !flags) return DAVA_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(wolfe_update_kernel<T>, dim3((unsigned)((batch + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), batch, (int)trial, c1, c2, (int)strong, state, flags);
  return launched();
}

}  // namespace dava

using namespace dava;

extern "C" int dava_bfgs_update_inverse_hessian_f32(int64_t batch, int64_t n, const float* h, const float* s,
                                                    const float* y, float* h_out, void* stream) {
  return update_inverse_hessian<float>(batch, n, h, s, y, h_out, stream);
}
extern "C" int dava_bfgs_update_inverse_hessian_f64(int64_t batch, int64_t n, const double* h, const double* s,
                                                    const double* y, double* h_out, void* stream) {
  return update_inverse_hessian<double>(batch, n, h, s, y, h_out, stream);
}
extern "C" int dava_bfgs_initial_scale_f32(int64_t batch, int64_t n, const float* s, const float* y,
                                           float* scale_out, void* stream) {
  return initial_scale<float>(batch, n, s, y, scale_out, stream);
}
extern "C" int dava_bfgs_initial_scale_f64(int64_t batch, int64_t n, const double* s, const double* y,
                                           double* scale_out, void* stream) {
  return initial_scale<double>(batch, n, s, y, scale_out, stream);
}
extern "C" int dava_bfgs_scale_matrix_f32(int64_t batch, int64_t n, const float* scale, const float* h, float* h_out,
                                          void* stream) {
  return scale_matrix<float>(batch, n, scale, h, h_out, stream);
}
extern "C" int dava_bfgs_scale_matrix_f64(int64_t batch, int64_t n, const double* scale, const double* h,
                                          double* h_out, void* stream) {
  return scale_matrix<double>(batch, n, scale, h, h_out, stream);
}
extern "C" int dava_bfgs_search_direction_f32(int64_t batch, int64_t n, const float* h, const float* g, float* d_out,
                                              void* stream) {
  return search_direction<float>(batch, n, h, g, d_out, stream);
}
extern "C" int dava_bfgs_search_direction_f64(int64_t batch, int64_t n, const double* h, const double* g,
                                              double* d_out, void* stream) {
  return search_direction<double>(batch, n, h, g, d_out, stream);
}
extern "C" int dava_bfgs_compact_direction_f32(int64_t n_active, int64_t n, int64_t row_stride, int64_t capacity,
                                               int64_t count, const int64_t* problem_index, const float* g,
                                               const float* y, const float* s, float* S, float* W, float* rho,
                                               float* c, float* gamma, float* d_out, void* stream) {
  return compact_direction<float>(n_active, n, row_stride, capacity, count, problem_index, g, y, s, S, W, rho, c,
                                  gamma, d_out, stream);
}
extern "C" int dava_bfgs_compact_direction_f64(int64_t n_active, int64_t n, int64_t row_stride, int64_t capacity,
                                               int64_t count, const int64_t* problem_index, const double* g,
                                               const double* y, const double* s, double* S, double* W, double* rho,
                                               double* c, double* gamma, double* d_out, void* stream) {
  return compact_direction<double>(n_active, n, row_stride, capacity, count, problem_index, g, y, s, S, W, rho, c,
                                   gamma, d_out, stream);
}
extern "C" int dava_wolfe_init_f32(int64_t batch, int64_t n, const float* direction, const float* f0, const float* g0,
                                   float* state, uint8_t* flags, void* stream) {
  return wolfe_init<float>(batch, n, direction, f0, g0, state, flags, stream);
}
extern "C" int dava_wolfe_init_f64(int64_t batch, int64_t n, const double* direction, const double* f0,
                                   const double* g0, double* state, uint8_t* flags, void* stream) {
  return wolfe_init<double>(batch, n, direction, f0, g0, state, flags, stream);
}
extern "C" int dava_wolfe_propose_f32(int64_t batch, float* state, const uint8_t* flags, void* stream) {
  return wolfe_propose<float>(batch, state, flags, stream);
}
extern "C" int dava_wolfe_propose_f64(int64_t batch, double* state, const uint8_t* flags, void* stream) {
  return wolfe_propose<double>(batch, state, flags, stream);
}
extern "C" int dava_wolfe_update_f32(int64_t batch, int32_t trial, float c1, float c2, int32_t strong, float* state,
                                     uint8_t* flags, void* stream) {
  return wolfe_update<float>(batch, trial, c1, c2, strong, state, flags, stream);
}
extern "C" int dava_wolfe_update_f64(int64_t batch, int32_t trial, double c1, double c2, int32_t strong,
                                     double* state, uint8_t* flags, void* stream) {
  return wolfe_update<double>(batch, trial, c1, c2, strong, state, flags, stream);
}

extern "C" const char* dava_status_string(int status) {
  switch (status) {
    case DAVA_OK: return "ok";
    case DAVA_ERR_INVALID_ARGUMENT: return "invalid argument";
    case DAVA_ERR_WORKSPACE: return "workspace missing or too small";
    case DAVA_ERR_LAUNCH: return "HIP kernel launch failed";
    case DAVA_ERR_UNSUPPORTED: return "shape not supported by this build";
    default: return "unknown status";
  }
}
extern "C" int dava_abi_version(void) { return DAVA_ABI_VERSION; }
extern "C" const char* dava_device_arch(void) { return "gfx950"; }
