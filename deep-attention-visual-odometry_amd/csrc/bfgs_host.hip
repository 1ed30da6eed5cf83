// The generic BFGS building blocks on HOST memory (fp32, fp64): what `BFGSSolver` runs when the
// caller's tensors live on the CPU, as the reference's solver does (autograd_solvers/bfgs_solver.py:94-117
// allocates on `parameters.device`; BASELINE configuration C1 is "BFGS on PyTorch CPU").  Host C++ in the
// same library as the device kernels: a device tensor never reaches these (the operators dispatch on the
// tensor's device), and with the library missing both paths raise.
//   dava_cpu_bfgs_update_inverse_hessian_*   bfgs_solver.py:235-303 (+ InverseCurvature, utils/func_inverse_curvature.py:21-51)
//   dava_cpu_bfgs_initial_scale_*            bfgs_solver.py:217-233
//   dava_cpu_bfgs_scale_matrix_*             bfgs_solver.py:159-167
//   dava_cpu_bfgs_search_direction_*         bfgs_solver.py:173-176
//   dava_cpu_wolfe_{init,propose,update}_*   line_search/wolfe_conditions.py:76-237
// and the reverse mode of the first four (csrc/bfgs_grad.hip has the derivation).  Same formulas and
// operation order per element as the device kernels; sums run in index order.
#include <cmath>
#include <cstdint>
#include <vector>

#include "dava_ba.h"

namespace dava_host {

template <typename T>
static T clamp_min(T v, T lo) { return v < lo ? lo : v; }

template <typename T>
static int update(int64_t batch, int64_t n, const T* h, const T* s, const T* y, T* out) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!h || !s || !y || !out || out == h) return DAVA_ERR_INVALID_ARGUMENT;
  std::vector<T> yH(n), Hy(n);
  for (int64_t b = 0; b < batch; ++b) {
    const T* H = h + b * n * n;
    const T* sv = s + b * n;
    const T* yv = y + b * n;
    T* O = out + b * n * n;
    for (int64_t j = 0; j < n; ++j) yH[j] = 0;
    for (int64_t i = 0; i < n; ++i) {
      T acc = 0;
      for (int64_t j = 0; j < n; ++j) {
        yH[j] += yv[i] * H[i * n + j];
        acc += H[i * n + j] * yv[j];
      }
      Hy[i] = acc;
    }
    T sy = 0;
    for (int64_t i = 0; i < n; ++i) sy += sv[i] * yv[i];
    const T rho = sy <= T(0) ? T(0) : T(1) / sy;  // InverseCurvature
    T yhy = 0;
    for (int64_t j = 0; j < n; ++j) yhy += yH[j] * (yv[j] * rho);
    const T c = T(1) + yhy;
    for (int64_t i = 0; i < n; ++i) {
      const T sri = sv[i] * rho, hyi = Hy[i];
      for (int64_t j = 0; j < n; ++j) {
        const T srj = sv[j] * rho;
        T t = H[i * n + j] + (sri * sv[j]) * c;
        t = t - sri * yH[j];
        O[i * n + j] = t - hyi * srj;
      }
    }
  }
  return DAVA_OK;
}

template <typename T>
static int initial_scale(int64_t batch, int64_t n, const T* s, const T* y, T* out) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0) return DAVA_OK;
  if (!s || !y || !out) return DAVA_ERR_INVALID_ARGUMENT;
  for (int64_t b = 0; b < batch; ++b) {
    T yy = 0, sy = 0;
    for (int64_t i = 0; i < n; ++i) {
      const T yi = y[b * n + i];
      yy += yi * yi;
      sy += s[b * n + i] * yi;
    }
    out[b] = clamp_min(sy / clamp_min(yy, T(1e-5)), T(1e-4));
  }
  return DAVA_OK;
}

template <typename T>
static int scale_matrix(int64_t batch, int64_t n, const T* scale, const T* h, T* out) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!scale || !h || !out) return DAVA_ERR_INVALID_ARGUMENT;
  const int64_t nn = n * n;
  for (int64_t e = 0; e < batch * nn; ++e) out[e] = scale[e / nn] * h[e];
  return DAVA_OK;
}

template <typename T>
static int search_direction(int64_t batch, int64_t n, const T* h, const T* g, T* d) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!h || !g || !d) return DAVA_ERR_INVALID_ARGUMENT;
  for (int64_t b = 0; b < batch; ++b)
    for (int64_t i = 0; i < n; ++i) {
      T acc = 0;
      for (int64_t j = 0; j < n; ++j) acc += h[b * n * n + i * n + j] * g[b * n + j];
      d[b * n + i] = T(-1) * acc;
    }
  return DAVA_OK;
}

enum { S_ALO = 0, S_AHI, S_A, S_FLO, S_FHI, S_FA, S_DFA, S_F0, S_DPHI0, S_COLS };

template <typename T>
static int wolfe_init(int64_t batch, int64_t n, const T* dir, const T* f0, const T* g0, T* state, uint8_t* flags) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0) return DAVA_OK;
  if (!dir || !f0 || !g0 || !state || !flags) return DAVA_ERR_INVALID_ARGUMENT;
  for (int64_t b = 0; b < batch; ++b) {
    T acc = 0;
    for (int64_t i = 0; i < n; ++i) acc += dir[b * n + i] * g0[b * n + i];
    T* st = state + b * S_COLS;
    const T f = f0[b];
    st[S_ALO] = 0; st[S_AHI] = 0; st[S_A] = 1;
    st[S_FLO] = f; st[S_FHI] = f; st[S_FA] = f;
    st[S_DFA] = acc; st[S_F0] = f; st[S_DPHI0] = acc;
    flags[b * 2] = 1;
    flags[b * 2 + 1] = 0;
  }
  return DAVA_OK;
}

template <typename T>
static int wolfe_propose(int64_t batch, T* state, const uint8_t* flags) {
  if (batch < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0) return DAVA_OK;
  if (!state || !flags) return DAVA_ERR_INVALID_ARGUMENT;
  for (int64_t b = 0; b < batch; ++b) {
    T* st = state + b * S_COLS;
    if (flags[b * 2]) {
      st[S_AHI] = st[S_A];
      st[S_FHI] = st[S_FA];
      st[S_A] = T(2) * st[S_A];
    }
    if (flags[b * 2 + 1]) st[S_A] = T(0.5) * (st[S_ALO] + st[S_AHI]);
  }
  return DAVA_OK;
}

// N&W 3.5 / 3.6 as wolfe_conditions.py:116-237 (NaN-blind comparisons kept on purpose)
template <typename T>
static int wolfe_update(int64_t batch, int32_t trial, T c1, T c2, int32_t strong, T* state, uint8_t* flags) {
  if (batch < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0) return DAVA_OK;
  if (!state || !flags) return DAVA_ERR_INVALID_ARGUMENT;
  for (int64_t b = 0; b < batch; ++b) {
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
      const bool curv = strong ? (std::fabs(dfa) <= lim) : (T(-1) * dfa <= lim);
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
  return DAVA_OK;
}

// ---- reverse mode (csrc/bfgs_grad.hip has the derivation) ----
template <typename T>
static int update_backward(int64_t batch, int64_t n, const T* h, const T* s, const T* y, const T* g, T* gh, T* gs,
                           T* gy) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!h || !s || !y || !g) return DAVA_ERR_INVALID_ARGUMENT;
  std::vector<T> yH(n), Hy(n), Gs(n), GyH(n), GTsr(n), GTHy(n), yHbar(n), t1(n), t2(n);
  for (int64_t b = 0; b < batch; ++b) {
    const T* H = h + b * n * n;
    const T* G = g + b * n * n;
    const T* sv = s + b * n;
    const T* yv = y + b * n;
    T sy = 0;
    for (int64_t i = 0; i < n; ++i) sy += sv[i] * yv[i];
    const T r = sy <= T(0) ? T(0) : T(1) / sy;
    for (int64_t j = 0; j < n; ++j) yH[j] = GTsr[j] = GTHy[j] = 0;
    for (int64_t i = 0; i < n; ++i) {
      T hy = 0;
      for (int64_t j = 0; j < n; ++j) {
        yH[j] += yv[i] * H[i * n + j];
        hy += H[i * n + j] * yv[j];
      }
      Hy[i] = hy;
    }
    T gip = 0, yyh = 0;
    for (int64_t j = 0; j < n; ++j) {
      gip += yH[j] * (yv[j] * r);
      yyh += yv[j] * yH[j];
    }
    const T q = T(1) + gip;
    for (int64_t i = 0; i < n; ++i) {
      T a = 0, c = 0;
      for (int64_t j = 0; j < n; ++j) {
        a += G[i * n + j] * sv[j];
        c += G[i * n + j] * yH[j];
        GTsr[j] += (sv[i] * r) * G[i * n + j];
        GTHy[j] += Hy[i] * G[i * n + j];
      }
      Gs[i] = a;
      GyH[i] = c;
    }
    T gipbar = 0;
    for (int64_t i = 0; i < n; ++i) gipbar += (sv[i] * r) * Gs[i];
    for (int64_t j = 0; j < n; ++j) yHbar[j] = gipbar * (yv[j] * r) - GTsr[j];
    for (int64_t j = 0; j < n; ++j) t2[j] = 0;
    for (int64_t i = 0; i < n; ++i) {
      T a = 0;
      const T u = T(-1) * r * Gs[i];
      for (int64_t j = 0; j < n; ++j) {
        a += H[i * n + j] * yHbar[j];
        t2[j] += u * H[i * n + j];
      }
      t1[i] = a;
    }
    T rbar = 0;
    for (int64_t i = 0; i < n; ++i) rbar += sv[i] * (q * Gs[i] - GyH[i] - GTHy[i]);
    rbar = rbar + gipbar * yyh;
    const T go = T(-1) * r * r * rbar;
    for (int64_t i = 0; i < n; ++i) {
      const T sbar_r = q * Gs[i] - GyH[i] - GTHy[i];
      if (gs) gs[b * n + i] = q * GTsr[i] + r * sbar_r + go * yv[i];
      if (gy) gy[b * n + i] = t1[i] + t2[i] + r * gipbar * yH[i] + go * sv[i];
    }
    if (gh)
      for (int64_t i = 0; i < n; ++i) {
        const T yi = yv[i], hyb = T(-1) * r * Gs[i];
        for (int64_t j = 0; j < n; ++j) gh[b * n * n + i * n + j] = G[i * n + j] + yi * yHbar[j] + hyb * yv[j];
      }
  }
  return DAVA_OK;
}

template <typename T>
static int initial_scale_backward(int64_t batch, int64_t n, const T* s, const T* y, const T* gout, T* gs, T* gy) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!s || !y || !gout) return DAVA_ERR_INVALID_ARGUMENT;
  for (int64_t b = 0; b < batch; ++b) {
    T yy = 0, sy = 0;
    for (int64_t i = 0; i < n; ++i) {
      const T yi = y[b * n + i];
      yy += yi * yi;
      sy += s[b * n + i] * yi;
    }
    const T dc = clamp_min(yy, T(1e-5));
    const T t = sy / dc;
    const T tbar = t >= T(1e-4) ? gout[b] : T(0);  // clamp backward passes where input >= min
    const T numbar = tbar / dc;
    const T dcbar = T(-1) * tbar * sy / (dc * dc);
    const T denbar = yy >= T(1e-5) ? dcbar : T(0);
    for (int64_t i = 0; i < n; ++i) {
      const T si = s[b * n + i], yi = y[b * n + i];
      if (gs) gs[b * n + i] = numbar * yi;
      if (gy) gy[b * n + i] = numbar * si + denbar * T(2) * yi;
    }
  }
  return DAVA_OK;
}

template <typename T>
static int scale_matrix_backward(int64_t batch, int64_t n, const T* scale, const T* h, const T* g, T* gscale, T* gh) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!scale || !h || !g) return DAVA_ERR_INVALID_ARGUMENT;
  const int64_t nn = n * n;
  for (int64_t b = 0; b < batch; ++b) {
    T acc = 0;
    for (int64_t e = 0; e < nn; ++e) {
      const T ge = g[b * nn + e];
      if (gscale) acc += ge * h[b * nn + e];
      if (gh) gh[b * nn + e] = scale[b] * ge;
    }
    if (gscale) gscale[b] = acc;
  }
  return DAVA_OK;
}

template <typename T>
static int search_direction_backward(int64_t batch, int64_t n, const T* h, const T* g, const T* dbar, T* gh, T* gg) {
  if (batch < 0 || n < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || n == 0) return DAVA_OK;
  if (!h || !g || !dbar) return DAVA_ERR_INVALID_ARGUMENT;
  for (int64_t b = 0; b < batch; ++b) {
    const T* H = h + b * n * n;
    const T* db = dbar + b * n;
    if (gg) {
      for (int64_t j = 0; j < n; ++j) gg[b * n + j] = 0;
      for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) gg[b * n + j] += (T(-1) * db[i]) * H[i * n + j];
    }
    if (gh)
      for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) gh[b * n * n + i * n + j] = (T(-1) * db[i]) * g[b * n + j];
  }
  return DAVA_OK;
}

}  // namespace dava_host

using namespace dava_host;

#define DAVA_CPU_ENTRY_POINTS(SUFFIX, T)                                                                          \
  extern "C" int dava_cpu_bfgs_update_inverse_hessian_##SUFFIX(int64_t batch, int64_t n, const T* h, const T* s, \
                                                               const T* y, T* h_out) {                          \
    return update<T>(batch, n, h, s, y, h_out);                                                                 \
  }                                                                                                              \
  extern "C" int dava_cpu_bfgs_initial_scale_##SUFFIX(int64_t batch, int64_t n, const T* s, const T* y,          \
                                                      T* scale_out) {                                           \
    return initial_scale<T>(batch, n, s, y, scale_out);                                                         \
  }                                                                                                              \
  extern "C" int dava_cpu_bfgs_scale_matrix_##SUFFIX(int64_t batch, int64_t n, const T* scale, const T* h,       \
                                                     T* h_out) {                                                \
    return scale_matrix<T>(batch, n, scale, h, h_out);                                                          \
  }                                                                                                              \
  extern "C" int dava_cpu_bfgs_search_direction_##SUFFIX(int64_t batch, int64_t n, const T* h, const T* g,       \
                                                         T* d_out) {                                            \
    return search_direction<T>(batch, n, h, g, d_out);                                                          \
  }                                                                                                              \
  extern "C" int dava_cpu_wolfe_init_##SUFFIX(int64_t batch, int64_t n, const T* direction, const T* f0,         \
                                              const T* g0, T* state, uint8_t* flags) {                          \
    return wolfe_init<T>(batch, n, direction, f0, g0, state, flags);                                            \
  }                                                                                                              \
  extern "C" int dava_cpu_wolfe_propose_##SUFFIX(int64_t batch, T* state, const uint8_t* flags) {                \
    return wolfe_propose<T>(batch, state, flags);                                                               \
  }                                                                                                              \
  extern "C" int dava_cpu_wolfe_update_##SUFFIX(int64_t batch, int32_t trial, T c1, T c2, int32_t strong,         \
                                                T* state, uint8_t* flags) {                                     \
    return wolfe_update<T>(batch, trial, c1, c2, strong, state, flags);                                         \
  }                                                                                                              \
  extern "C" int dava_cpu_bfgs_update_inverse_hessian_backward_##SUFFIX(int64_t batch, int64_t n, const T* h,   \
                                                                        const T* s, const T* y,                 \
                                                                        const T* grad_out, T* grad_h,           \
                                                                        T* grad_s, T* grad_y) {                 \
    return update_backward<T>(batch, n, h, s, y, grad_out, grad_h, grad_s, grad_y);                             \
  }                                                                                                              \
  extern "C" int dava_cpu_bfgs_initial_scale_backward_##SUFFIX(int64_t batch, int64_t n, const T* s, const T* y, \
                                                               const T* grad_out, T* grad_s, T* grad_y) {       \
    return initial_scale_backward<T>(batch, n, s, y, grad_out, grad_s, grad_y);                                 \
  }                                                                                                              \
  extern "C" int dava_cpu_bfgs_scale_matrix_backward_##SUFFIX(int64_t batch, int64_t n, const T* scale,          \
                                                              const T* h, const T* grad_out, T* grad_scale,     \
                                                              T* grad_h) {                                      \
    return scale_matrix_backward<T>(batch, n, scale, h, grad_out, grad_scale, grad_h);                          \
  }                                                                                                              \
  extern "C" int dava_cpu_bfgs_search_direction_backward_##SUFFIX(int64_t batch, int64_t n, const T* h,          \
                                                                  const T* g, const T* grad_d, T* grad_h,       \
                                                                  T* grad_g) {                                  \
    return search_direction_backward<T>(batch, n, h, g, grad_d, grad_h, grad_g);                                \
  }

DAVA_CPU_ENTRY_POINTS(f32, float)
DAVA_CPU_ENTRY_POINTS(f64, double)
