// Multi-view pinhole (+ Brown-Conrady) squared reprojection objective on gfx950.
//
// E(x) = sum_{m,n} vis[m,n] * || pi_m(X_n) - obs[m,n] ||^2      
//
// One problem per 256-thread workgroup.  Threads own points (n = tid, tid+256,
// ...); each thread sweeps every view for its points, so a point's gradient
// never needs a cross-thread reduction.  Per-view gradients (translation,
// rotation) are wave-reduced per view and summed across the 4 waves once, and
// the intrinsics / scale-path sums go through one deterministic block
// reduction.  Three flavours share the code:
//   GRAD  : reverse mode, writes dE/dx into an LDS vector (replaces
//           torch.autograd.grad in bfgs_solver.py:133-135),
//   SLOPE : forward mode along a direction d, returns phi'(alpha) = d . grad E
//           (replaces the autograd-w.r.t.-alpha trick of wolfe_conditions.py:134-143),
//   TRIAL : evaluate at x + alpha*d formed on the fly, rounded exactly as the
//           reference forms `parameters + alpha * direction`.
// Forward-model references:
//   scale normalisation   camera_model/calibration_pinhole_camera_model.py:97-104
//   Rodrigues             geometry/axis_angle_rotation.py:25-48
//   Taylor branches       utils/func_sin_x_on_x.py:5-98, utils/func_one_minus_cos_x_on_x_squared.py:6-51
//   pinhole               geometry/camera_projection.py:20-35
//   Brown-Conrady         camera_model/distorted_camera_model.py:59-86 (fx = fy = f, s = 0)
// Derivatives are derived here by hand (the reference's analytic BC Jacobian is
// wrong) and checked against autograd of the oracle in tests/.
#pragma once

#include "dava_common.hpp"
#include "dava_dual.hpp"

#include <type_traits>

namespace dava {

// Diagnostic builds only (DAVA_PHASE_TIMING): thread 0 of every workgroup adds the shader
// cycles of each section of ba_eval (float instantiations) to g_eval_cycles.
#ifndef DAVA_PHASE_TIMING
#define DAVA_PHASE_TIMING 0
#endif
constexpr int kEvalSections = 6;  // view constants, point sums, setup, pair sweep, final sums, gradient assembly
#if DAVA_PHASE_TIMING
__device__ unsigned long long g_eval_cycles[kEvalSections];
#define DAVA_ESTAMP(i)                                                           \
  do {                                                                           \
    if (std::is_same<S, float>::value && threadIdx.x == 0) {                     \
      const unsigned long long t1_ = clock64();                                  \
      atomicAdd(&g_eval_cycles[i], t1_ - et0_);                                  \
      et0_ = t1_;                                                                \
    }                                                                            \
  } while (0)
#else
#define DAVA_ESTAMP(i) \
  do {                 \
  } while (0)
#endif

// Two points' worth of fp32 in one register pair: the packed pair sweep (PACK) runs the
// per-(view, point) arithmetic on v_pk_{fma,mul,add}_f32, two points per instruction.
typedef float pf2 __attribute__((ext_vector_type(2)));

struct Layout {
  int M, N, P, distort;
  __device__ __forceinline__ int pt(int n) const { return 3 + 3 * n; }
  __device__ __forceinline__ int tr(int m) const { return 3 + 3 * N + 3 * (m - 1); }
  __device__ __forceinline__ int rot(int m) const { return 3 + 3 * N + 3 * (M - 1) + 3 * (m - 1); }
  __device__ __forceinline__ int dist() const { return 3 + 3 * N + 6 * (M - 1); }
};

// ---- Taylor-branched ratios, same thresholds and series as the reference ----
// (templated on the scalar: float, or Dual for second derivatives, dava_dual.hpp)
// sx, cx: sin x and cos x, computed once by the caller (sincos_)
template <typename S>
__device__ __forceinline__ S sinc(S x, S sx) {
  if (fabs_(x) < 0.01f) {
    const S x2 = x * x, x4 = x2 * x2, x6 = x4 * x2;
    return 1.0f - x2 / 6.0f + x4 / 120.0f - x6 / 5040.0f;
  }
  return sx / x;
}
template <typename S>
__device__ __forceinline__ S sinc_slope(S x, S sx, S cx) {  // cos/x^2 - sin/x^3
  const S x2 = x * x;
  if (fabs_(x) < 0.01f) {
    const S x4 = x2 * x2, x6 = x4 * x2;
    return -1.0f / 3.0f + x2 / 30.0f - x4 / 840.0f + x6 / 45360.0f;
  }
  return cx / x2 - sx / (x * x2);
}
template <typename S>
__device__ __forceinline__ S versine_ratio(S x, S cx) {  // (1 - cos x)/x^2
  const S x2 = x * x;
  if (fabs_(x) < 0.05f) {
    const S x4 = x2 * x2, x6 = x4 * x2;
    return 0.5f - x2 / 24.0f + x4 / 720.0f - x6 / 40320.0f;
  }
  return (1.0f - cx) / x2;
}

// ---- per-view constants, kept in LDS (one row of kViewStride floats per view >= 1) ----
constexpr int kViewStride = 24;
enum ViewField {
  VW0 = 0, VW1, VW2,     // rotation (trial value)
  VCOS, VA, VB, VSIN,    // cos th, (1-cos)/th^2, sin/th, sin th
  VRCP, VAP, VTC,        // 1/th (0 at 0), dA/dth, dB/dth
  VDW0, VDW1, VDW2, VDTH,// direction of w, d th
  VT0, VT1, VT2,         // translation (trial value, unnormalised)
  VDT0, VDT1, VDT2       // direction of t
};

// Partial sums per view kept by each wave: 8 floats {gw_direct xyz, g_theta, g_t~ xyz, -}
constexpr int kViewPart = 8;

// LDS footprint helpers (floats)
__host__ __device__ inline int views_floats(int M) { return (M - 1) * kViewStride; }
__host__ __device__ inline int vpart_floats(int M, int nw = kWaves) { return M * nw * kViewPart; }

template <typename S>
struct Intrinsics {
  S f, cx, cy, k1, k2, k3, p1, p2;
};

template <bool TRIAL, typename S>
__device__ __forceinline__ S trial_value(const S* x, const S* d, float a, int i) {
  if constexpr (TRIAL) return fadd_rn(x[i], fmul_rn(S(a), d[i]));
  else return x[i];
}

// ---- ray-angle residual (the error CalibrationNetwork minimises) ----------------------
// calibration_network.py:58-67: angle between the observation's ray
// (pixel_coordinates_to_homogeneous, geometry/homogeneous_projection.py:21-44:
// (u - cx, v - cy, elu(f) + 1)) and the camera-relative point p, in Kahan's form
// 2 atan2(|a^ - b^|, |a^ + b^|) with both norms clamped at 2^-52
// (geometry/projective_plane_angle_distance.py:20-64).  Derivatives follow torch's
// conventions: a zero norm has zero subgradient, a clamped norm passes none.
template <typename S>
struct RayAngle {
  S cx, cy, F, Fp;  // principal point, focal elu(f) + 1 and its derivative
  S dcx, dcy, dF;   // SLOPE: tangents
};
constexpr float kRayEps = 2.220446049250313e-16f;

// Every division by a norm is a multiplication by its reciprocal (one IEEE division per norm instead
// of one per component: ~16 -> 7 division sequences per (view, point) pair; C3 ray 180k -> 204k
// problems/s, profiles/r02_ab_ray_rcp.log).  Results move by an ulp against torch's per-component
// division; every ray-angle parity test is unchanged.
// unit vector x / clamp(|x|, eps) and the projection of a cotangent / tangent through it (inv_n = 1 / n)
template <typename S>
__device__ __forceinline__ void ray_unit_backward(S r, S inv_n, const S (&u)[3], const S (&g)[3], S (&out)[3]) {
  const S k = r >= kRayEps ? u[0] * g[0] + u[1] * g[1] + u[2] * g[2] : S(0.0f);
#pragma unroll
  for (int c = 0; c < 3; ++c) out[c] = (g[c] - u[c] * k) * inv_n;
}

template <bool GRAD, bool SLOPE, typename S>
__device__ __forceinline__ void ray_angle_pair(const RayAngle<S>& ra, const S (&ob)[2], uint8_t visible, S p0,
                                               S p1, S p2, S dp0, S dp1, S dp2, S& e,
                                               S& sl, S (&gin)[8], S& G0, S& G1, S& G2, S& go0, S& go1) {
  const float wgt = visible ? 1.0f : 0.0f;
  const S h[3] = {ob[0] - ra.cx, ob[1] - ra.cy, ra.F};
  const S hr = sqrt_(h[0] * h[0] + h[1] * h[1] + h[2] * h[2]);
  const S hn = clamp_min(hr, kRayEps);
  const S pr = sqrt_(p0 * p0 + p1 * p1 + p2 * p2);
  const S pn = clamp_min(pr, kRayEps);
  const S ihn = 1.0f / hn, ipn = 1.0f / pn;
  const S a[3] = {h[0] * ihn, h[1] * ihn, h[2] * ihn};
  const S b[3] = {p0 * ipn, p1 * ipn, p2 * ipn};
  const S su[3] = {a[0] + b[0], a[1] + b[1], a[2] + b[2]};
  const S df[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  const S Sn = sqrt_(su[0] * su[0] + su[1] * su[1] + su[2] * su[2]);
  const S Dn = sqrt_(df[0] * df[0] + df[1] * df[1] + df[2] * df[2]);
  e += 2.0f * atan2_(Dn, Sn) * wgt;
  const S den = Sn * Sn + Dn * Dn;
  // reciprocals shared by the forward (slope) and reverse (gradient) parts
  const S iden = (GRAD || SLOPE) ? 1.0f / den : S(0.0f);
  const S iSn = (GRAD || SLOPE) && Sn > 0.0f ? 1.0f / Sn : S(0.0f);
  const S iDn = (GRAD || SLOPE) && Dn > 0.0f ? 1.0f / Dn : S(0.0f);
  if constexpr (SLOPE) {
    const S dh[3] = {-ra.dcx, -ra.dcy, ra.dF};
    const S dp[3] = {dp0, dp1, dp2};
    S da[3], db[3];
    ray_unit_backward(hr, ihn, a, dh, da);  // the Jacobian of x -> x/|x| is symmetric
    ray_unit_backward(pr, ipn, b, dp, db);
    const S nS = su[0] * (da[0] + db[0]) + su[1] * (da[1] + db[1]) + su[2] * (da[2] + db[2]);
    const S nD = df[0] * (da[0] - db[0]) + df[1] * (da[1] - db[1]) + df[2] * (da[2] - db[2]);
    const S dS = Sn > 0.0f ? nS * iSn : S(0.0f);
    const S dD = Dn > 0.0f ? nD * iDn : S(0.0f);
    sl += 2.0f * wgt * (Sn * dD - Dn * dS) * iden;
  }
  if constexpr (GRAD) {
    const S gD = 2.0f * wgt * Sn * iden;  // atan2 backward
    const S gS = -2.0f * wgt * Dn * iden;
    const S cD = Dn > 0.0f ? gD * iDn : S(0.0f);
    const S cS = Sn > 0.0f ? gS * iSn : S(0.0f);
    const S ga[3] = {cS * su[0] + cD * df[0], cS * su[1] + cD * df[1], cS * su[2] + cD * df[2]};
    const S gb[3] = {cS * su[0] - cD * df[0], cS * su[1] - cD * df[1], cS * su[2] - cD * df[2]};
    S gh[3], gp[3];
    ray_unit_backward(hr, ihn, a, ga, gh);
    ray_unit_backward(pr, ipn, b, gb, gp);
    gin[0] += gh[2] * ra.Fp;
    gin[1] -= gh[0];
    gin[2] -= gh[1];
    G0 = gp[0]; G1 = gp[1]; G2 = gp[2];
    go0 = gh[0]; go1 = gh[1];  // dE/d obs (u, v): h = obs - c
  }
}

// Evaluate E (and optionally its gradient and/or slope along d) for one problem.
// All 256 threads must call; E / slope come back identical in every thread.
//   x, d, grad, obs, vis, views, vpart, scratch : LDS (or HBM in GV mode)
//   buf : reduction double-buffer toggle (updated)
// DOT   (with GRAD): slope_out = d . grad E, assembled from the gradient's parts inside
//        the final reduction (no extra barrier) -- the contraction the reference's
//        autograd w.r.t. alpha performs.
// CHECK (with TRIAL): if x + alpha d rounds to x in every component, return false right
//        after the first reduction without evaluating (the caller knows the answer:
//        f(x) and phi'(0)); otherwise evaluate and return true.
// PPT > 0: every thread keeps its (at most PPT) points' trial coordinates, directions and
//        gradients in registers for the whole view sweep (requires N <= PPT * threads);
//        PPT = 0: they are re-read from / accumulated into x, d, grad view after view.
template <bool GRAD, bool SLOPE, bool TRIAL, bool DOT = false, bool CHECK = false,
          int RES = DAVA_RESIDUAL_SQUARED_REPROJECTION, typename S = float, int NW = kWaves, int PPT = 0,
          bool PACK = false>
__device__ __forceinline__ bool ba_eval(const Layout& L, const S* x, const S* d, float alpha, const float* obs,
                                        const uint8_t* vis, S* grad, S* views, S* vpart, float* scratch, int& buf,
                                        S& E_out, S& slope_out, S* obs_grad = nullptr,
                                        float* obs_tangent_acc = nullptr, const float* obs_dir = nullptr) {
  constexpr int BLOCK = kWave * NW;  // threads in the workgroup
  static_assert(!DOT || (GRAD && !SLOPE), "DOT derives the slope from the reverse-mode gradient");
  static_assert(!CHECK || TRIAL, "CHECK needs a trial point");
  constexpr int PR = PPT > 0 ? PPT : 1;
  S Xr[PR][3], Dr[PR][3], Gr[PR][3];  // PPT > 0: this thread's points (n = tid + u BLOCK)
#if DAVA_PHASE_TIMING
  unsigned long long et0_ = clock64();
#endif
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wave = tid / kWave;
  const int M = L.M, N = L.N;

  // 1. per-view rotation constants (views 1..M-1), one thread per view; the same thread adds
  //    its view's |t| (and sgn(t) dt) to the scale-normalisation sums of step 2
  S t_abs = 0.f, t_dir = 0.f;
  for (int m = 1 + tid; m < M; m += BLOCK) {
    S* v = views + (m - 1) * kViewStride;
    const int r = L.rot(m), t = L.tr(m);
    const S w0 = trial_value<TRIAL>(x, d, alpha, r + 0);
    const S w1 = trial_value<TRIAL>(x, d, alpha, r + 1);
    const S w2 = trial_value<TRIAL>(x, d, alpha, r + 2);
    const S th = sqrt_(w0 * w0 + w1 * w1 + w2 * w2);
    S sth, cth;
    sincos_(th, sth, cth);
    const S A = versine_ratio(th, cth), B = sinc(th, sth);
    const S rcp = th == 0.0f ? S(0.0f) : 1.0f / th;
    v[VW0] = w0; v[VW1] = w1; v[VW2] = w2;
    v[VCOS] = cth; v[VA] = A; v[VB] = B; v[VSIN] = sth;
    v[VRCP] = rcp;
    v[VAP] = rcp * (B - 2.0f * A);       // d/dth (1-cos)/th^2, reference backward form
    v[VTC] = th * sinc_slope(th, sth, cth);  // d/dth sin(th)/th
    const S t0 = trial_value<TRIAL>(x, d, alpha, t + 0);
    const S t1 = trial_value<TRIAL>(x, d, alpha, t + 1);
    const S t2 = trial_value<TRIAL>(x, d, alpha, t + 2);
    v[VT0] = t0; v[VT1] = t1; v[VT2] = t2;
    t_abs += fabs_(t0);
    t_abs += fabs_(t1);
    t_abs += fabs_(t2);
    if constexpr (SLOPE) {
      const S d0 = d[r], d1 = d[r + 1], d2 = d[r + 2];
      v[VDW0] = d0; v[VDW1] = d1; v[VDW2] = d2;
      v[VDTH] = (w0 * d0 + w1 * d1 + w2 * d2) * rcp;
      v[VDT0] = d[t]; v[VDT1] = d[t + 1]; v[VDT2] = d[t + 2];
      t_dir += sgn(t0) * d[t];
      t_dir += sgn(t1) * d[t + 1];
      t_dir += sgn(t2) * d[t + 2];
    }
  }

  DAVA_ESTAMP(0);
  // 2. scale normalisation s = (mean|X| N + mean|t| M)/(N+M), and its slope
  // sum|X|, sum sgn(X) dX (SLOPE or DOT), moved (CHECK), sum|t|, sum sgn(t) dt (SLOPE)
  S sums[5] = {0.f, 0.f, 0.f, t_abs, t_dir};
  bool moved = false;
  auto point_sums = [&](int n, S (&Xp)[3], S (&Dp)[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const S X = trial_value<TRIAL>(x, d, alpha, L.pt(n) + c);
      Xp[c] = X;
      Dp[c] = (SLOPE || DOT) ? d[L.pt(n) + c] : S(0.0f);
      sums[0] += fabs_(X);
      if constexpr (SLOPE || DOT) sums[1] += sgn(X) * Dp[c];
      if constexpr (CHECK) moved |= X != x[L.pt(n) + c];
    }
  };
  if constexpr (PPT > 0) {
#pragma unroll
    for (int u = 0; u < PPT; ++u)
      if (tid + u * BLOCK < N) point_sums(tid + u * BLOCK, Xr[u], Dr[u]);
  } else {
    for (int n = tid; n < N; n += BLOCK) point_sums(n, Xr[0], Dr[0]);
  }
  if constexpr (CHECK) {
    // the parameters that are not point coordinates: intrinsics, views, distortion
    const int other = L.P - 3 * N;
    for (int k = tid; k < other; k += BLOCK) {
      const int i = k < 3 ? k : k + 3 * N;
      moved |= trial_value<true>(x, d, alpha, i) != x[i];
    }
    sums[2] = moved ? 1.f : 0.f;
  }
  block_sum<5, NW>(sums, scratch, buf);
  buf ^= 1;  // (this barrier also publishes the view constants)
  DAVA_ESTAMP(1);
  if constexpr (CHECK) {
    if (sums[2] == 0.f) return false;  // uniform: every thread holds the same sums
  }
  const S tsum = sums[3], tdsum = sums[4];
  (void)tdsum;
  const float fN = (float)N, fM = (float)M, fNM = (float)(N + M);
  const S ps = sums[0] / (3.0f * fN);
  const S cs = tsum / (3.0f * (float)(M - 1));
  const S s = (ps * fN + cs * fM) / fNM;
  const S inv_s = 1.0f / s;
  // the distorted model's z' == 0 -> 1e-8 (distorted_camera_model.py:57); -0 for the pinhole model
  const float z_nudge = L.distort ? 1e-8f : -0.0f;
  S ds_over_s = 0.f;
  if constexpr (SLOPE) {
    const S ds = ((sums[1] / (3.0f * fN)) * fN + (tdsum / (3.0f * (float)(M - 1))) * fM) / fNM;
    ds_over_s = ds * inv_s;
  }

  // 3. intrinsics (trial values + directions)
  Intrinsics<S> in, din;
  in.f = trial_value<TRIAL>(x, d, alpha, 0);
  in.cx = trial_value<TRIAL>(x, d, alpha, 1);
  in.cy = trial_value<TRIAL>(x, d, alpha, 2);
  in.k1 = in.k2 = in.k3 = in.p1 = in.p2 = 0.f;
  din = Intrinsics<S>{0, 0, 0, 0, 0, 0, 0, 0};
  const int kd = L.dist();
  if (L.distort) {
    in.k1 = trial_value<TRIAL>(x, d, alpha, kd + 0);
    in.k2 = trial_value<TRIAL>(x, d, alpha, kd + 1);
    in.k3 = trial_value<TRIAL>(x, d, alpha, kd + 2);
    in.p1 = trial_value<TRIAL>(x, d, alpha, kd + 3);
    in.p2 = trial_value<TRIAL>(x, d, alpha, kd + 4);
  }
  if constexpr (SLOPE) {
    din.f = d[0]; din.cx = d[1]; din.cy = d[2];
    if (L.distort) { din.k1 = d[kd]; din.k2 = d[kd + 1]; din.k3 = d[kd + 2]; din.p1 = d[kd + 3]; din.p2 = d[kd + 4]; }
  }

  RayAngle<S> ra{};
  if constexpr (RES == DAVA_RESIDUAL_RAY_ANGLE) {
    ra.cx = in.cx;
    ra.cy = in.cy;
    ra.F = (in.f > 0.0f ? in.f : expm1_(in.f)) + 1.0f;  // elu(f) + 1
    ra.Fp = in.f > 0.0f ? 1.0f : exp_(in.f);
    if constexpr (SLOPE) { ra.dcx = din.cx; ra.dcy = din.cy; ra.dF = ra.Fp * din.f; }
  }

  S e_loc = 0.f, sl_loc = 0.f;
  S gin[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // f cx cy k1 k2 k3 p1 p2
  S gsx = 0.f;                          // sum gX~ . X  (scale path)
  S gdx = 0.f;                          // DOT: sum gX~ . dX

  DAVA_ESTAMP(2);
  // 4. sweep views (outer) x own points (inner)
  for (int m = 0; m < M; ++m) {
    const S* v = views + (m > 0 ? (m - 1) * kViewStride : 0);
    S vc = 1.f, vA = 0.f, vB = 0.f, vs = 0.f, vAp = 0.f, vTC = 0.f;
    S w0 = 0.f, w1 = 0.f, w2 = 0.f, tt0 = 0.f, tt1 = 0.f, tt2 = 0.f;
    S dw0 = 0.f, dw1 = 0.f, dw2 = 0.f, dth = 0.f, dtt0 = 0.f, dtt1 = 0.f, dtt2 = 0.f;
    if (m > 0) {
      w0 = v[VW0]; w1 = v[VW1]; w2 = v[VW2];
      vc = v[VCOS]; vA = v[VA]; vB = v[VB]; vs = v[VSIN]; vAp = v[VAP]; vTC = v[VTC];
      tt0 = v[VT0] * inv_s; tt1 = v[VT1] * inv_s; tt2 = v[VT2] * inv_s;  // t~ = t / s
      if constexpr (SLOPE) {
        dw0 = v[VDW0]; dw1 = v[VDW1]; dw2 = v[VDW2]; dth = v[VDTH];
        dtt0 = (v[VDT0] - tt0 * (ds_over_s * s)) * inv_s;
        dtt1 = (v[VDT1] - tt1 * (ds_over_s * s)) * inv_s;
        dtt2 = (v[VDT2] - tt2 * (ds_over_s * s)) * inv_s;
      }
    }
    S vg[7] = {0, 0, 0, 0, 0, 0, 0};  // gw_direct xyz, g_theta, g_t~ xyz

    // Packed sweeps (global-vector mode, squared objective): the view's Rodrigues rotation as a 3x3 matrix
    // R = c I + A w w^T + B [w]x, formed once per view: p = R X~ + t~ (9 FMAs per pair instead of the
    // vector form's 18), dE/dX~ = R^T G, and the view's rotation gradient from the per-thread sums
    // Mg = sum_n G_n X~_n^T (9 FMAs per pair): every direct-w and theta term of the vector form is linear
    // in Mg (sum (X~.w) G = Mg w, sum (G.w) X~ = Mg^T w, sum X~ x G = axial(Mg), sum G.X~ = tr Mg,
    // sum (X~.w)(G.w) = w^T Mg w).  SLOPE: dp = R dX~ + Rdot X~ + dt~ with Rdot = dc I + dA w w^T +
    // A (w dw^T + dw w^T) + B [dw]x + dB [w]x.  The same math in another rounding; the LDS-mode sweeps
    // keep the vector form (there the matrix form measured C2 -3.5%, C3 -1.2%); C5 +1.9..2.4%
    // (profiles/r04_ab_variants_c5.log, profiles/r04_ab_gv_rotmat.log, profiles/r04_ab_c5_dma_stream_rotmat.log).
    constexpr bool kRotMat = PACK && std::is_same<S, float>::value && RES == DAVA_RESIDUAL_SQUARED_REPROJECTION;
    S R[9], Rd[9], Mg[9];
    if constexpr (kRotMat) {
      const S ww[3] = {w0, w1, w2};
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          R[3 * i + j] = vA * ww[i] * ww[j] + (i == j ? vc : S(0.0f));
          Mg[3 * i + j] = 0.f;
        }
      R[1] -= vB * w2; R[2] += vB * w1; R[3] += vB * w2; R[5] -= vB * w0; R[6] -= vB * w1; R[7] += vB * w0;
      if constexpr (SLOPE) {
        const S dc = -vs * dth, dA = vAp * dth, dB = vTC * dth;
        const S dd[3] = {dw0, dw1, dw2};
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            Rd[3 * i + j] = dA * ww[i] * ww[j] + vA * (ww[i] * dd[j] + dd[i] * ww[j]) + (i == j ? dc : S(0.0f));
        Rd[1] -= vB * dw2 + dB * w2; Rd[2] += vB * dw1 + dB * w1; Rd[3] += vB * dw2 + dB * w2;
        Rd[5] -= vB * dw0 + dB * w0; Rd[6] -= vB * dw1 + dB * w1; Rd[7] += vB * dw0 + dB * w0;
      }
    }
    (void)R; (void)Rd; (void)Mg;

    // one (view m, point n) pair.  X / dX: the point's trial coordinates and direction;
    // q: its gradient, accumulated view after view (registers when PPT > 0, else loaded from
    // and stored back to `grad` by the caller below -- the same additions in the same order)
    auto pair = [&](int n, const S X0, const S X1, const S X2, const S dX0, const S dX1, const S dX2, S& q0, S& q1,
                    S& q2) {
      // the pair's observation; for dual numbers with an observation direction (second derivatives in the
      // observations, ba_second_order) it carries that tangent
      S ob[2] = {obs[2 * (m * N + n)], obs[2 * (m * N + n) + 1]};
      if constexpr (!std::is_same<S, float>::value) {
        if (obs_dir) {
          ob[0] = S(obs[2 * (m * N + n)], obs_dir[2 * (m * N + n)]);
          ob[1] = S(obs[2 * (m * N + n) + 1], obs_dir[2 * (m * N + n) + 1]);
        }
      }
      const uint8_t visible = vis[m * N + n];
      const S a0 = X0 * inv_s, a1 = X1 * inv_s, a2 = X2 * inv_s;  // X~ = X / s
      S da0 = 0.f, da1 = 0.f, da2 = 0.f;
      if constexpr (SLOPE) {
        da0 = (dX0 - a0 * (ds_over_s * s)) * inv_s;
        da1 = (dX1 - a1 * (ds_over_s * s)) * inv_s;
        da2 = (dX2 - a2 * (ds_over_s * s)) * inv_s;
      }
      // camera-relative point p (and dp)
      S p0, p1, p2, dp0 = 0.f, dp1 = 0.f, dp2 = 0.f;
      S vw = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f;  // v.w and w x v
      if (m == 0) {
        p0 = a0; p1 = a1; p2 = a2;
        if constexpr (SLOPE) { dp0 = da0; dp1 = da1; dp2 = da2; }
      } else if constexpr (kRotMat) {
        p0 = R[0] * a0 + R[1] * a1 + R[2] * a2 + tt0;
        p1 = R[3] * a0 + R[4] * a1 + R[5] * a2 + tt1;
        p2 = R[6] * a0 + R[7] * a1 + R[8] * a2 + tt2;
        if constexpr (SLOPE) {
          dp0 = (R[0] * da0 + R[1] * da1 + R[2] * da2) + (Rd[0] * a0 + Rd[1] * a1 + Rd[2] * a2) + dtt0;
          dp1 = (R[3] * da0 + R[4] * da1 + R[5] * da2) + (Rd[3] * a0 + Rd[4] * a1 + Rd[5] * a2) + dtt1;
          dp2 = (R[6] * da0 + R[7] * da1 + R[8] * da2) + (Rd[6] * a0 + Rd[7] * a1 + Rd[8] * a2) + dtt2;
        }
      } else {
        vw = a0 * w0 + a1 * w1 + a2 * w2;
        c0 = w1 * a2 - w2 * a1;
        c1 = w2 * a0 - w0 * a2;
        c2 = w0 * a1 - w1 * a0;
        const S Avw = vA * vw;
        p0 = a0 * vc + Avw * w0 + c0 * vB + tt0;
        p1 = a1 * vc + Avw * w1 + c1 * vB + tt1;
        p2 = a2 * vc + Avw * w2 + c2 * vB + tt2;
        if constexpr (SLOPE) {
          const S dc = -vs * dth, dA = vAp * dth, dB = vTC * dth;
          const S dvw = (da0 * w0 + da1 * w1 + da2 * w2) + (a0 * dw0 + a1 * dw1 + a2 * dw2);
          const S e0 = (dw1 * a2 - dw2 * a1) + (w1 * da2 - w2 * da1);
          const S e1 = (dw2 * a0 - dw0 * a2) + (w2 * da0 - w0 * da2);
          const S e2 = (dw0 * a1 - dw1 * a0) + (w0 * da1 - w1 * da0);
          const S k = dA * vw + vA * dvw;
          dp0 = da0 * vc + a0 * dc + k * w0 + Avw * dw0 + e0 * vB + c0 * dB + dtt0;
          dp1 = da1 * vc + a1 * dc + k * w1 + Avw * dw1 + e1 * vB + c1 * dB + dtt1;
          dp2 = da2 * vc + a2 * dc + k * w2 + Avw * dw2 + e2 * vB + c2 * dB + dtt2;
        }
      }
      S G0 = 0.f, G1 = 0.f, G2 = 0.f;  // dE/dp
      S go0 = 0.f, go1 = 0.f;          // dE/d obs (second-order instantiations only)
      if constexpr (RES == DAVA_RESIDUAL_SQUARED_REPROJECTION) {
        // projection; the distorted model nudges z' == 0 by 1e-8 (distorted_camera_model.py:57)
        // branch-free: + (-0) leaves every p2 (signed zeros included) bit for bit, so the pinhole
        // model is untouched; a runtime-uniform branch here cost C2 5% (profiles/r03_ab_c2_regression_bisect.log)
        p2 = p2 + (p2 == S(0.0f) ? z_nudge : -0.0f);
        const S iz = 1.0f / p2;
        const S qx = p0 * iz, qy = p1 * iz;
        const S ub = in.f * qx, vb = in.f * qy;
        S u, vv, dub = 0.f, dvb = 0.f;
        S Juu = 1.f, Juv = 0.f, Jvv = 1.f, r2 = 0.f;
        if constexpr (SLOPE) {
          const S dqx = (dp0 - qx * dp2) * iz, dqy = (dp1 - qy * dp2) * iz;
          dub = din.f * qx + in.f * dqx;
          dvb = din.f * qy + in.f * dqy;
        }
        if (L.distort) {
          r2 = ub * ub + vb * vb;
          const S D = 1.0f + in.k1 * r2 + in.k2 * r2 * r2 + in.k3 * r2 * r2 * r2;
          const S Dr = in.k1 + 2.0f * in.k2 * r2 + 3.0f * in.k3 * r2 * r2;
          const S uvb = ub * vb;
          u = ub * D + 2.0f * in.p1 * uvb + in.p2 * (r2 + 2.0f * ub * ub) + in.cx;
          vv = vb * D + 2.0f * in.p2 * uvb + in.p1 * (r2 + 2.0f * vb * vb) + in.cy;
          Juu = D + 2.0f * ub * ub * Dr + 2.0f * in.p1 * vb + 6.0f * in.p2 * ub;
          Juv = 2.0f * uvb * Dr + 2.0f * in.p1 * ub + 2.0f * in.p2 * vb;
          Jvv = D + 2.0f * vb * vb * Dr + 2.0f * in.p2 * ub + 6.0f * in.p1 * vb;
        } else {
          u = ub + in.cx;
          vv = vb + in.cy;
        }
        const float wgt = visible ? 1.0f : 0.0f;
        const S ru = u - ob[0], rv = vv - ob[1];
        e_loc += (ru * ru + rv * rv) * wgt;
        if constexpr (SLOPE) {
          S du = Juu * dub + Juv * dvb + din.cx;
          S dv = Juv * dub + Jvv * dvb + din.cy;
          if (L.distort) {
            const S r4 = r2 * r2;
            du += ub * (r2 * din.k1 + r4 * din.k2 + r4 * r2 * din.k3) + 2.0f * ub * vb * din.p1 +
                  (r2 + 2.0f * ub * ub) * din.p2;
            dv += vb * (r2 * din.k1 + r4 * din.k2 + r4 * r2 * din.k3) + (r2 + 2.0f * vb * vb) * din.p1 +
                  2.0f * ub * vb * din.p2;
          }
          sl_loc += 2.0f * wgt * (ru * du + rv * dv);
        }
        if constexpr (GRAD) {
          const S gu = 2.0f * wgt * ru, gv = 2.0f * wgt * rv;
          go0 = -gu;
          go1 = -gv;
          gin[1] += gu;
          gin[2] += gv;
          S gub = gu, gvb = gv;
          if (L.distort) {
            gub = gu * Juu + gv * Juv;
            gvb = gu * Juv + gv * Jvv;
            const S r4 = r2 * r2;
            const S gr = gu * ub + gv * vb;
            gin[3] += gr * r2;
            gin[4] += gr * r4;
            gin[5] += gr * r4 * r2;
            gin[6] += gu * 2.0f * ub * vb + gv * (r2 + 2.0f * vb * vb);
            gin[7] += gu * (r2 + 2.0f * ub * ub) + gv * 2.0f * ub * vb;
          }
          gin[0] += gub * qx + gvb * qy;
          const S fi = in.f * iz;
          G0 = gub * fi; G1 = gvb * fi; G2 = -(gub * ub + gvb * vb) * iz;
        }
      } else {
        ray_angle_pair<GRAD, SLOPE, S>(ra, ob, visible, p0, p1, p2, dp0, dp1, dp2, e_loc, sl_loc, gin, G0, G1, G2,
                                       go0, go1);
      }
      if constexpr (GRAD && !std::is_same<S, float>::value) {
        const int pr = m * N + n;
        if (obs_grad) {
          obs_grad[2 * pr] = go0;
          obs_grad[2 * pr + 1] = go1;
        }
        if (obs_tangent_acc) {  // (d2E/dobs dx) v added straight into a float accumulator (one owner per pair)
          obs_tangent_acc[2 * pr] += go0.t;
          obs_tangent_acc[2 * pr + 1] += go1.t;
        }
      }
      if constexpr (GRAD) {
        S gx0, gx1, gx2;
        if (m == 0) {
          gx0 = G0; gx1 = G1; gx2 = G2;
        } else if constexpr (kRotMat) {
          gx0 = R[0] * G0 + R[3] * G1 + R[6] * G2;  // R^T G
          gx1 = R[1] * G0 + R[4] * G1 + R[7] * G2;
          gx2 = R[2] * G0 + R[5] * G1 + R[8] * G2;
          Mg[0] += G0 * a0; Mg[1] += G0 * a1; Mg[2] += G0 * a2;
          Mg[3] += G1 * a0; Mg[4] += G1 * a1; Mg[5] += G1 * a2;
          Mg[6] += G2 * a0; Mg[7] += G2 * a1; Mg[8] += G2 * a2;
          vg[4] += G0; vg[5] += G1; vg[6] += G2;  // dE/dt~
        } else {
          const S Gw = G0 * w0 + G1 * w1 + G2 * w2;
          const S Gv = G0 * a0 + G1 * a1 + G2 * a2;
          const S Gx = G0 * c0 + G1 * c1 + G2 * c2;
          const S AGw = vA * Gw, Avw = vA * vw;
          // dE/dX~ = c G + A (G.w) w + B (G x w)
          gx0 = vc * G0 + AGw * w0 + vB * (G1 * w2 - G2 * w1);
          gx1 = vc * G1 + AGw * w1 + vB * (G2 * w0 - G0 * w2);
          gx2 = vc * G2 + AGw * w2 + vB * (G0 * w1 - G1 * w0);
          // dE/dw (direct) = A vw G + A (G.w) X~ + B (X~ x G)
          vg[0] += Avw * G0 + AGw * a0 + vB * (a1 * G2 - a2 * G1);
          vg[1] += Avw * G1 + AGw * a1 + vB * (a2 * G0 - a0 * G2);
          vg[2] += Avw * G2 + AGw * a2 + vB * (a0 * G1 - a1 * G0);
          vg[3] += -vs * Gv + vAp * vw * Gw + vTC * Gx;  // dE/dth
          vg[4] += G0; vg[5] += G1; vg[6] += G2;          // dE/dt~
        }
        if (m == 0) { q0 = gx0; q1 = gx1; q2 = gx2; }
        else { q0 += gx0; q1 += gx1; q2 += gx2; }
        if (m == M - 1) {
          gsx += q0 * X0 + q1 * X1 + q2 * X2;
          if constexpr (DOT) gdx += q0 * dX0 + q1 * dX1 + q2 * dX2;
        }
      }
    };
    // PACK: two of this thread's points (n0, n1 = n0 + BLOCK) per step, the same formulas as
    // `pair` (squared reprojection, fp32) on packed pairs.  Every accumulator still takes point n0's
    // term, then n1's -- the order of the scalar sweep; only the rounding of FMA contraction
    // inside a term may differ from the scalar form.
    if constexpr (PPT > 0) {
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        const int n = tid + u * BLOCK;
        if (n < N) pair(n, Xr[u][0], Xr[u][1], Xr[u][2], Dr[u][0], Dr[u][1], Dr[u][2], Gr[u][0], Gr[u][1], Gr[u][2]);
      }
    } else {
      int n0 = tid;
      if constexpr (PACK && RES == DAVA_RESIDUAL_SQUARED_REPROJECTION && std::is_same<S, float>::value) {
        // the pair's observations and visibility (read in place from HBM in GV mode).  (Loading the next
        // pair's one step ahead measured C5 -7%: registers, profiles/r02_ab_prefetch_c5.log.)
        struct ScenePair {
          pf2 u, v, w;
        };
        auto fetch = [&](int a, int b) {
          const int i0 = m * N + a, i1 = m * N + b;
          return ScenePair{pf2{obs[2 * i0], obs[2 * i1]}, pf2{obs[2 * i0 + 1], obs[2 * i1 + 1]},
                           pf2{vis[i0] ? 1.0f : 0.0f, vis[i1] ? 1.0f : 0.0f}};
        };
        auto pair2 = [&](const ScenePair& sp, const pf2 X0, const pf2 X1, const pf2 X2, const pf2 dX0,
                         const pf2 dX1, const pf2 dX2, pf2& q0, pf2& q1, pf2& q2) {
          const pf2 obu = sp.u, obv = sp.v, wgt = sp.w;
          auto acc = [](S& a, const pf2 t) {  // point n0's term, then n1's
            a += t.x;
            a += t.y;
          };
          const pf2 a0 = X0 * inv_s, a1 = X1 * inv_s, a2 = X2 * inv_s;
          pf2 da0 = 0.f, da1 = 0.f, da2 = 0.f;
          if constexpr (SLOPE) {
            da0 = (dX0 - a0 * (ds_over_s * s)) * inv_s;
            da1 = (dX1 - a1 * (ds_over_s * s)) * inv_s;
            da2 = (dX2 - a2 * (ds_over_s * s)) * inv_s;
          }
          pf2 p0, p1, p2, dp0 = 0.f, dp1 = 0.f, dp2 = 0.f;
          pf2 vw = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f;
          if (m == 0) {
            p0 = a0; p1 = a1; p2 = a2;
            if constexpr (SLOPE) { dp0 = da0; dp1 = da1; dp2 = da2; }
          } else if constexpr (kRotMat) {
            p0 = R[0] * a0 + R[1] * a1 + R[2] * a2 + tt0;
            p1 = R[3] * a0 + R[4] * a1 + R[5] * a2 + tt1;
            p2 = R[6] * a0 + R[7] * a1 + R[8] * a2 + tt2;
            if constexpr (SLOPE) {
              dp0 = (R[0] * da0 + R[1] * da1 + R[2] * da2) + (Rd[0] * a0 + Rd[1] * a1 + Rd[2] * a2) + dtt0;
              dp1 = (R[3] * da0 + R[4] * da1 + R[5] * da2) + (Rd[3] * a0 + Rd[4] * a1 + Rd[5] * a2) + dtt1;
              dp2 = (R[6] * da0 + R[7] * da1 + R[8] * da2) + (Rd[6] * a0 + Rd[7] * a1 + Rd[8] * a2) + dtt2;
            }
          } else {
            vw = a0 * w0 + a1 * w1 + a2 * w2;
            c0 = w1 * a2 - w2 * a1;
            c1 = w2 * a0 - w0 * a2;
            c2 = w0 * a1 - w1 * a0;
            const pf2 Avw = vA * vw;
            p0 = a0 * vc + Avw * w0 + c0 * vB + tt0;
            p1 = a1 * vc + Avw * w1 + c1 * vB + tt1;
            p2 = a2 * vc + Avw * w2 + c2 * vB + tt2;
            if constexpr (SLOPE) {
              const S dc = -vs * dth, dA = vAp * dth, dB = vTC * dth;
              const pf2 dvw = (da0 * w0 + da1 * w1 + da2 * w2) + (a0 * dw0 + a1 * dw1 + a2 * dw2);
              const pf2 e0 = (dw1 * a2 - dw2 * a1) + (w1 * da2 - w2 * da1);
              const pf2 e1 = (dw2 * a0 - dw0 * a2) + (w2 * da0 - w0 * da2);
              const pf2 e2 = (dw0 * a1 - dw1 * a0) + (w0 * da1 - w1 * da0);
              const pf2 k = dA * vw + vA * dvw;
              dp0 = da0 * vc + a0 * dc + k * w0 + Avw * dw0 + e0 * vB + c0 * dB + dtt0;
              dp1 = da1 * vc + a1 * dc + k * w1 + Avw * dw1 + e1 * vB + c1 * dB + dtt1;
              dp2 = da2 * vc + a2 * dc + k * w2 + Avw * dw2 + e2 * vB + c2 * dB + dtt2;
            }
          }
          // z' == 0 nudge (distorted_camera_model.py:57), branch-free
          p2.x = p2.x + (p2.x == 0.0f ? z_nudge : -0.0f);
          p2.y = p2.y + (p2.y == 0.0f ? z_nudge : -0.0f);
          const pf2 iz = 1.0f / p2;
          const pf2 qx = p0 * iz, qy = p1 * iz;
          const pf2 ub = in.f * qx, vb = in.f * qy;
          pf2 u, vv, dub = 0.f, dvb = 0.f;
          pf2 Juu = 1.f, Juv = 0.f, Jvv = 1.f, r2 = 0.f;
          if constexpr (SLOPE) {
            const pf2 dqx = (dp0 - qx * dp2) * iz, dqy = (dp1 - qy * dp2) * iz;
            dub = din.f * qx + in.f * dqx;
            dvb = din.f * qy + in.f * dqy;
          }
          if (L.distort) {
            r2 = ub * ub + vb * vb;
            const pf2 D = 1.0f + in.k1 * r2 + in.k2 * r2 * r2 + in.k3 * r2 * r2 * r2;
            const pf2 Dr = in.k1 + 2.0f * in.k2 * r2 + 3.0f * in.k3 * r2 * r2;
            const pf2 uvb = ub * vb;
            u = ub * D + 2.0f * in.p1 * uvb + in.p2 * (r2 + 2.0f * ub * ub) + in.cx;
            vv = vb * D + 2.0f * in.p2 * uvb + in.p1 * (r2 + 2.0f * vb * vb) + in.cy;
            Juu = D + 2.0f * ub * ub * Dr + 2.0f * in.p1 * vb + 6.0f * in.p2 * ub;
            Juv = 2.0f * uvb * Dr + 2.0f * in.p1 * ub + 2.0f * in.p2 * vb;
            Jvv = D + 2.0f * vb * vb * Dr + 2.0f * in.p2 * ub + 6.0f * in.p1 * vb;
          } else {
            u = ub + in.cx;
            vv = vb + in.cy;
          }
          const pf2 ru = u - obu, rv = vv - obv;
          acc(e_loc, (ru * ru + rv * rv) * wgt);
          if constexpr (SLOPE) {
            pf2 du = Juu * dub + Juv * dvb + din.cx;
            pf2 dv = Juv * dub + Jvv * dvb + din.cy;
            if (L.distort) {
              const pf2 r4 = r2 * r2;
              du += ub * (r2 * din.k1 + r4 * din.k2 + r4 * r2 * din.k3) + 2.0f * ub * vb * din.p1 +
                    (r2 + 2.0f * ub * ub) * din.p2;
              dv += vb * (r2 * din.k1 + r4 * din.k2 + r4 * r2 * din.k3) + (r2 + 2.0f * vb * vb) * din.p1 +
                    2.0f * ub * vb * din.p2;
            }
            acc(sl_loc, 2.0f * wgt * (ru * du + rv * dv));
          }
          if constexpr (GRAD) {
            const pf2 gu = 2.0f * wgt * ru, gv = 2.0f * wgt * rv;
            acc(gin[1], gu);
            acc(gin[2], gv);
            pf2 gub = gu, gvb = gv;
            if (L.distort) {
              gub = gu * Juu + gv * Juv;
              gvb = gu * Juv + gv * Jvv;
              const pf2 r4 = r2 * r2;
              const pf2 gr = gu * ub + gv * vb;
              acc(gin[3], gr * r2);
              acc(gin[4], gr * r4);
              acc(gin[5], gr * r4 * r2);
              acc(gin[6], gu * 2.0f * ub * vb + gv * (r2 + 2.0f * vb * vb));
              acc(gin[7], gu * (r2 + 2.0f * ub * ub) + gv * 2.0f * ub * vb);
            }
            acc(gin[0], gub * qx + gvb * qy);
            const pf2 fi = in.f * iz;
            const pf2 G0 = gub * fi, G1 = gvb * fi, G2 = -(gub * ub + gvb * vb) * iz;
            pf2 gx0, gx1, gx2;
            if (m == 0) {
              gx0 = G0; gx1 = G1; gx2 = G2;
            } else if constexpr (kRotMat) {
              gx0 = R[0] * G0 + R[3] * G1 + R[6] * G2;
              gx1 = R[1] * G0 + R[4] * G1 + R[7] * G2;
              gx2 = R[2] * G0 + R[5] * G1 + R[8] * G2;
              acc(Mg[0], G0 * a0); acc(Mg[1], G0 * a1); acc(Mg[2], G0 * a2);
              acc(Mg[3], G1 * a0); acc(Mg[4], G1 * a1); acc(Mg[5], G1 * a2);
              acc(Mg[6], G2 * a0); acc(Mg[7], G2 * a1); acc(Mg[8], G2 * a2);
              acc(vg[4], G0); acc(vg[5], G1); acc(vg[6], G2);
            } else {
              const pf2 Gw = G0 * w0 + G1 * w1 + G2 * w2;
              const pf2 Gv = G0 * a0 + G1 * a1 + G2 * a2;
              const pf2 Gx = G0 * c0 + G1 * c1 + G2 * c2;
              const pf2 AGw = vA * Gw, Avw = vA * vw;
              gx0 = vc * G0 + AGw * w0 + vB * (G1 * w2 - G2 * w1);
              gx1 = vc * G1 + AGw * w1 + vB * (G2 * w0 - G0 * w2);
              gx2 = vc * G2 + AGw * w2 + vB * (G0 * w1 - G1 * w0);
              acc(vg[0], Avw * G0 + AGw * a0 + vB * (a1 * G2 - a2 * G1));
              acc(vg[1], Avw * G1 + AGw * a1 + vB * (a2 * G0 - a0 * G2));
              acc(vg[2], Avw * G2 + AGw * a2 + vB * (a0 * G1 - a1 * G0));
              acc(vg[3], -vs * Gv + vAp * vw * Gw + vTC * Gx);
              acc(vg[4], G0); acc(vg[5], G1); acc(vg[6], G2);
            }
            if (m == 0) { q0 = gx0; q1 = gx1; q2 = gx2; }
            else { q0 += gx0; q1 += gx1; q2 += gx2; }
            if (m == M - 1) {
              acc(gsx, q0 * X0 + q1 * X1 + q2 * X2);
              if constexpr (DOT) acc(gdx, q0 * dX0 + q1 * dX1 + q2 * dX2);
            }
          }
        };
        for (; n0 + BLOCK < N; n0 += 2 * BLOCK) {
          const int n1 = n0 + BLOCK, ia = L.pt(n0), ib = L.pt(n1);
          const ScenePair cur = fetch(n0, n1);
          pf2 X[3], dX[3] = {0.f, 0.f, 0.f}, q[3] = {0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            X[c] = pf2{trial_value<TRIAL>(x, d, alpha, ia + c), trial_value<TRIAL>(x, d, alpha, ib + c)};
            if constexpr (SLOPE || DOT) dX[c] = pf2{d[ia + c], d[ib + c]};
            if constexpr (GRAD) {
              if (m > 0) q[c] = pf2{grad[ia + c], grad[ib + c]};
            }
          }
          pair2(cur, X[0], X[1], X[2], dX[0], dX[1], dX[2], q[0], q[1], q[2]);
          if constexpr (GRAD) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              grad[ia + c] = q[c].x;
              grad[ib + c] = q[c].y;
            }
          }
        }
      }
      for (int n = n0; n < N; n += BLOCK) {
        const int ip = L.pt(n);
        const S X0 = trial_value<TRIAL>(x, d, alpha, ip + 0);
        const S X1 = trial_value<TRIAL>(x, d, alpha, ip + 1);
        const S X2 = trial_value<TRIAL>(x, d, alpha, ip + 2);
        S dX0 = 0.f, dX1 = 0.f, dX2 = 0.f, q0 = 0.f, q1 = 0.f, q2 = 0.f;
        if constexpr (SLOPE || DOT) { dX0 = d[ip]; dX1 = d[ip + 1]; dX2 = d[ip + 2]; }
        if constexpr (GRAD) {
          if (m > 0) { q0 = grad[ip]; q1 = grad[ip + 1]; q2 = grad[ip + 2]; }
        }
        pair(n, X0, X1, X2, dX0, dX1, dX2, q0, q1, q2);
        if constexpr (GRAD) { grad[ip] = q0; grad[ip + 1] = q1; grad[ip + 2] = q2; }
      }
    }
    if constexpr (GRAD && kRotMat) {
      if (m > 0) {  // the vector form's direct-w and theta sums, from this thread's Mg
        const S Mw0 = Mg[0] * w0 + Mg[1] * w1 + Mg[2] * w2;
        const S Mw1 = Mg[3] * w0 + Mg[4] * w1 + Mg[5] * w2;
        const S Mw2 = Mg[6] * w0 + Mg[7] * w1 + Mg[8] * w2;
        const S MTw0 = Mg[0] * w0 + Mg[3] * w1 + Mg[6] * w2;
        const S MTw1 = Mg[1] * w0 + Mg[4] * w1 + Mg[7] * w2;
        const S MTw2 = Mg[2] * w0 + Mg[5] * w1 + Mg[8] * w2;
        const S ax0 = Mg[7] - Mg[5], ax1 = Mg[2] - Mg[6], ax2 = Mg[3] - Mg[1];  // sum X~ x G
        vg[0] = vA * (Mw0 + MTw0) + vB * ax0;
        vg[1] = vA * (Mw1 + MTw1) + vB * ax1;
        vg[2] = vA * (Mw2 + MTw2) + vB * ax2;
        vg[3] = -vs * (Mg[0] + Mg[4] + Mg[8]) + vAp * (w0 * Mw0 + w1 * Mw1 + w2 * Mw2) +
                vTC * (w0 * ax0 + w1 * ax1 + w2 * ax2);
      }
    }
    if constexpr (GRAD) {
      if (m > 0) {
        if constexpr (std::is_same<S, float>::value) {
          float w[7];
#pragma unroll
          for (int k = 0; k < 7; ++k) w[k] = vg[k];
          wave_sums<7>(w);  // transposed: two wave_sum4 instead of seven wave_sum
#pragma unroll
          for (int k = 0; k < 7; ++k)
            if (lane == 0) vpart[(m * NW + wave) * kViewPart + k] = w[k];
        } else {
#pragma unroll
          for (int k = 0; k < 7; ++k) {
            const S w = wave_sum(vg[k]);
            if (lane == 0) vpart[(m * NW + wave) * kViewPart + k] = w;
          }
        }
        // scale path, translation part: sum_m g_t~ . t (this thread's share) joins gsx in the
        // final block reduction
        gsx += vg[4] * v[VT0] + vg[5] * v[VT1] + vg[6] * v[VT2];
      }
    }
  }

  DAVA_ESTAMP(3);
  // 5. block reduction of error, slope, intrinsics gradient and scale-path sum
  if constexpr (GRAD) {
    S r[12] = {e_loc, sl_loc, gin[0], gin[1], gin[2], gin[3], gin[4], gin[5], gin[6], gin[7], gsx, gdx};
    if constexpr (DOT) block_sum<12, NW>(r, scratch, buf);
    else block_sum<11, NW>(reinterpret_cast<S(&)[11]>(r), scratch, buf);
    buf ^= 1;
    DAVA_ESTAMP(4);
    E_out = r[0];
    slope_out = r[1];
    // scale path: s = (ps N + cs M)/(N+M); X~ = X/s, t~ = t/s.  r[10] = sum gX~ . X + sum g_t~ . t
    const S gs = -r[10] * inv_s * inv_s;
    const S g_ps = gs * fN / fNM, g_cs = gs * fM / fNM;
    const S gabsX = g_ps / (3.0f * fN);
    const S gabsT = g_cs / (3.0f * (float)(M - 1));
    // DOT (every thread forms d . grad, which reads all the per-view totals): the 7 (M - 1) totals are
    // summed once, in parallel, into the reduction half the next block_sum writes (free until then:
    // its last reads were before this reduction's barrier; the closing barrier below ends these
    // reads) -- the same sums in the same order, instead of every thread re-adding NW partials each.
    S* vtot = nullptr;
    if constexpr (DOT && std::is_same<S, float>::value) {
      if (7 * (M - 1) <= NW * 32) {
        vtot = scratch + buf * (NW * 32);
        for (int q = tid; q < 7 * (M - 1); q += BLOCK)
          vtot[q] = wave_partials_total<NW>(vpart + ((1 + q / 7) * NW) * kViewPart + q % 7, kViewPart);
        __syncthreads();
      }
    }
    if constexpr (DOT) {
      // d . grad = (1/s) sum d.gX~ + gabsX sum d.sgn(X) + views + intrinsics (all threads, same order)
      S dv = 0.f;
      for (int m = 1; m < M; ++m) {
        const S* v = views + (m - 1) * kViewStride;
        auto vs = [&](int k) {
          if (vtot) return vtot[(m - 1) * 7 + k];
          const S* p = vpart + (m * NW) * kViewPart + k;
          return wave_partials_total<NW>(p, kViewPart);
        };
        const S gth = vs(3) * v[VRCP];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          dv += d[L.tr(m) + c] * (vs(4 + c) * inv_s + sgn(v[VT0 + c]) * gabsT);
          dv += d[L.rot(m) + c] * (vs(c) + gth * v[VW0 + c]);
        }
      }
      S di = d[0] * r[2] + d[1] * r[3] + d[2] * r[4];
      if (L.distort) {
#pragma unroll
        for (int k = 0; k < 5; ++k) di += d[kd + k] * r[5 + k];
      }
      slope_out = (r[11] * inv_s + gabsX * sums[1]) + dv + di;
    }
    if constexpr (PPT > 0) {
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        const int n = tid + u * BLOCK;
        if (n < N) {
#pragma unroll
          for (int c = 0; c < 3; ++c) grad[L.pt(n) + c] = Gr[u][c] * inv_s + sgn(Xr[u][c]) * gabsX;
        }
      }
    } else {
      for (int n = tid; n < N; n += BLOCK) {
        S* gp = grad + L.pt(n);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const S X = trial_value<TRIAL>(x, d, alpha, L.pt(n) + c);
          gp[c] = gp[c] * inv_s + sgn(X) * gabsX;
        }
      }
    }
    for (int q = tid; q < 6 * (M - 1); q += BLOCK) {
      const int m = 1 + q / 6, c = q % 6;
      const S* v = views + (m - 1) * kViewStride;
      auto vsum = [&](int k) {
        if (vtot) return vtot[(m - 1) * 7 + k];
        const S* p = vpart + (m * NW) * kViewPart + k;
        return wave_partials_total<NW>(p, kViewPart);
      };
      if (c < 3) {
        grad[L.tr(m) + c] = vsum(4 + c) * inv_s + sgn(v[VT0 + c]) * gabsT;
      } else {
        const int k = c - 3;
        grad[L.rot(m) + k] = vsum(k) + vsum(3) * v[VRCP] * v[VW0 + k];
      }
    }
    if (tid == 0) {
      grad[0] = r[2]; grad[1] = r[3]; grad[2] = r[4];
      if (L.distort) {
#pragma unroll
        for (int k = 0; k < 5; ++k) grad[kd + k] = r[5 + k];
      }
    }
    __syncthreads();
    DAVA_ESTAMP(5);
  } else {
    S r[2] = {e_loc, sl_loc};
    if constexpr (SLOPE) block_sum<2, NW>(r, scratch, buf);
    else block_sum<1, NW>(reinterpret_cast<S(&)[1]>(r), scratch, buf);
    buf ^= 1;
    E_out = r[0];
    slope_out = r[1];
  }
  return true;
}

}  // namespace dava
