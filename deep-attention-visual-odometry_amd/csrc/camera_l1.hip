// The legacy IOptimisableFunction camera model (PinholeCameraModelL1) on gfx950.
//
// Reference: camera_model/pinhole_camera_model_l1.py.  One workgroup per
// (batch, estimate); each of the 4 waves owns views m = wave, wave + 4, ...,
// each lane owns points n = lane, lane + 64, ...  For every (view, point) pair:
//   world point  (:405-432)   p0 = 0, p1 = (1,0,0), p2 = (w0x, w0y, 0), p_{n>=3} = w_{n-2}
//   camera point (:434-466)   R(omega_m) p_n + t_m with z clamped to
//                             max(z, clamp(max(|r x|, |r y|), min=minimum_z_distance)),
//                             r = 1 / maximum_pixel_ratio, R from LieRotation.rotate_vector
//                             (geometry/lie_rotation.py, Taylor branches of utils/func_*.py)
//   projection   (:468-500)   u = f x / z + cx, v = f y / z + cy
//   error        (:132-190)   scale * sum |(u - u~) vis| + scale * sum |(v - v~) vis|,
//                             scale = fp32(sqrt(1 / (M N)))
//   gradient     (:192-285, _compute_gradient_from_intermediates :529-642,
//                 _stack_gradients :645-712): the reference's HAND-WRITTEN partials,
//                 reproduced as written -- including the max_gradient clipping (with
//                 torch.clip's max-wins rule when max_gradient < 0) and the use of
//                 dv/dz' in du/dy -- because this object must return exactly what the
//                 reference's get_gradient() returns, which is what its BFGSCameraSolver
//                 consumes.
// Deterministic: per-view sums are wave butterflies, per-point sums over views
// are added in view order from LDS, globals in a fixed wave order.
#include "dava_common.hpp"

#include <type_traits>

namespace dava {

template <typename T>
struct LieTrig {
  T cos_t, sinc, versine, c_term, d_term;  // cos th, sin th/th, (1-cos)/th^2, C(th), D(th)
};

// utils/func_sin_x_on_x.py, func_one_minus_cos_x_on_x_squared.py,
// func_sin_x_on_x_cubed_minus_two_one_minus_cos_x_on_x_fourth.py (value branches)
template <typename T>
__device__ __forceinline__ LieTrig<T> lie_trig(T th) {
  LieTrig<T> r;
  const T a = th < T(0) ? -th : th;
  const T x2 = th * th, x4 = x2 * x2, x6 = x4 * x2;
  r.cos_t = cos(th);
  const T s = sin(th);
  r.sinc = a < T(0.01) ? T(1) - x2 / T(6) + x4 / T(120) - x6 / T(5040) : s / th;
  r.versine = a < T(0.05) ? T(0.5) - x2 / T(24) + x4 / T(720) - x6 / T(40320) : (T(1) - r.cos_t) / x2;
  r.c_term = a < T(0.01) ? T(-1) / T(3) + x2 / T(30) - x4 / T(840) + x6 / T(45360)
                         : r.cos_t / x2 - s / (th * x2);
  r.d_term = a < T(0.25) ? T(-1) / T(12) + x2 / T(180) - x4 / T(6720) + x6 / T(362880)
                         : s / (th * x2) - T(2) * (T(1) - r.cos_t) / x4;
  return r;
}

template <typename T>
__device__ __forceinline__ T clip(T v, T lo, T hi) {  // torch.clip: max(min) then min(max) -> max wins
  v = v < lo ? lo : v;
  return v > hi ? hi : v;
}

template <typename T>
__device__ __forceinline__ T sign_of(T v) { return v > T(0) ? T(1) : (v < T(0) ? T(-1) : T(0)); }

// Forward-mode dual numbers over T (float or double) for the model's JVPs (autograd through the
// model, enable_error_gradients / enable_grad_gradients): branches, clamps and clips follow the
// value, and take the derivative of the branch taken, as torch's autograd does; sign() is flat.
using ::cos;  // the LDual overloads below must not hide the scalar ones
using ::sin;
using ::sqrt;
template <typename T>
struct LDual {
  T v, t;
  __device__ __forceinline__ LDual() = default;
  __device__ __forceinline__ constexpr LDual(T value) : v(value), t(T(0)) {}  // NOLINT: constants
  __device__ __forceinline__ constexpr LDual(T value, T tangent) : v(value), t(tangent) {}
};
template <typename T> __device__ __forceinline__ LDual<T> operator+(LDual<T> a, LDual<T> b) { return {a.v + b.v, a.t + b.t}; }
template <typename T> __device__ __forceinline__ LDual<T> operator-(LDual<T> a, LDual<T> b) { return {a.v - b.v, a.t - b.t}; }
template <typename T> __device__ __forceinline__ LDual<T> operator-(LDual<T> a) { return {-a.v, -a.t}; }
template <typename T> __device__ __forceinline__ LDual<T> operator*(LDual<T> a, LDual<T> b) {
  return {a.v * b.v, a.t * b.v + a.v * b.t};
}
template <typename T> __device__ __forceinline__ LDual<T> operator/(LDual<T> a, LDual<T> b) {
  const T q = a.v / b.v;
  return {q, (a.t - q * b.t) / b.v};
}
template <typename T> __device__ __forceinline__ LDual<T>& operator+=(LDual<T>& a, LDual<T> b) { return a = a + b; }
template <typename T> __device__ __forceinline__ bool operator<(LDual<T> a, LDual<T> b) { return a.v < b.v; }
template <typename T> __device__ __forceinline__ bool operator>(LDual<T> a, LDual<T> b) { return a.v > b.v; }
template <typename T> __device__ __forceinline__ LDual<T> sqrt(LDual<T> a) {
  const T r = sqrt(a.v);
  return {r, r > T(0) ? a.t / (T(2) * r) : T(0)};
}
template <typename T> __device__ __forceinline__ LDual<T> sin(LDual<T> a) { return {sin(a.v), cos(a.v) * a.t}; }
template <typename T> __device__ __forceinline__ LDual<T> cos(LDual<T> a) { return {cos(a.v), -sin(a.v) * a.t}; }
template <typename T> __device__ __forceinline__ LDual<T> sign_of(LDual<T> a) { return LDual<T>(sign_of(a.v)); }
template <typename T> __device__ __forceinline__ LDual<T> wave_sum(LDual<T> a) {
  return {wave_sum(a.v), wave_sum(a.t)};
}
template <typename T> __device__ __forceinline__ void detach(LDual<T>& a) { a.t = T(0); }
__device__ __forceinline__ void detach(float&) {}
__device__ __forceinline__ void detach(double&) {}

// the VJP launch's seed: workgroup (estimate be, direction d) puts tangent 1 on one input element
// (directions: 0 focal, 1 cx, 2 cy, 3 + 3m + c translation, 3 + 3M + 3m + c lie vector,
//  3 + 6M + 3k + c world point k)
enum L1Input { L1_FOCAL, L1_CX, L1_CY, L1_TRANS, L1_LIE, L1_WORLD };

template <typename T>
struct L1Args {
  int M, N, P, E;
  const T *focal, *cx, *cy, *trans, *lie, *world, *target;
  const uint8_t* vis;
  T min_z, pixel_ratio, max_grad, scale;
  T *err, *grad;
};

// One (batch, estimate): error and hand-written gradient in scalar type S (T, or LDual<T> seeded
// along direction `dir`).  store_err(S) / store_grad(index, S) receive the outputs.
// detach_points: the world and camera-relative points carry no tangent (the reference's
// enable_grad_gradients = False detaches them in get_gradient, :185-198).
template <typename T, typename S, class StoreErr, class StoreGrad>
__device__ __forceinline__ void l1_body(const L1Args<T>& a, int64_t be, int dir, bool want_grad, bool detach_points,
                                        StoreErr store_err, StoreGrad store_grad) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  S* pp = reinterpret_cast<S*>(smem);  // [M][N][4] per-view point-gradient terms
  const int M = a.M, N = a.N;
  const int64_t b = be / a.E;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  auto in = [&](int kind, T value, int idx) -> S {  // input element `idx` of `kind`, seeded if it is `dir`
    if constexpr (std::is_same<S, T>::value) {
      return value;
    } else {
      const int base = kind == L1_FOCAL ? 0 : kind == L1_CX ? 1 : kind == L1_CY ? 2
                     : kind == L1_TRANS ? 3 : kind == L1_LIE ? 3 + 3 * M : 3 + 6 * M;
      return S(value, base + idx == dir ? T(1) : T(0));
    }
  };
  const S f = in(L1_FOCAL, a.focal[be], 0), cx = in(L1_CX, a.cx[be], 0), cy = in(L1_CY, a.cy[be], 0);
  const T* trp = a.trans + be * M * 3;
  const T* om = a.lie + be * M * 3;
  const T* wpp = a.world + be * (int64_t)(N - 2) * 3;
  auto tr = [&](int i) { return in(L1_TRANS, trp[i], i); };
  auto wp = [&](int i) { return in(L1_WORLD, wpp[i], i); };
  const T* tgt = a.target + b * (int64_t)M * N * 2;
  const uint8_t* vs = a.vis + b * (int64_t)M * N;
  const bool g = want_grad;
  // parameter offsets (pinhole_camera_model_l1.py:366-378)
  const int oa = 3, ob = oa + M, oc = ob + M, otx = oc + M, oty = otx + M, otz = oty + M;
  const int ox = otz + M, oy = ox + (N - 2), oz = oy + (N - 2);

  S eu = T(0), ev = T(0), gcx = T(0), gcy = T(0), gf = T(0);
  for (int m = wave; m < M; m += kWaves) {
    const S w0 = in(L1_LIE, om[3 * m], 3 * m), w1 = in(L1_LIE, om[3 * m + 1], 3 * m + 1);
    const S w2 = in(L1_LIE, om[3 * m + 2], 3 * m + 2);
    const S th = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const LieTrig<S> L = lie_trig(th);
    // LieRotation.vector_gradient: A w w^T + [[cos, -c, b], [c, cos, -a], [-b, a, cos]], (a,b,c) = w sinc
    const S sa = w0 * L.sinc, sb = w1 * L.sinc, sc = w2 * L.sinc;
    S RG[3][3];
    const S wv[3] = {w0, w1, w2};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) RG[i][j] = wv[j] * wv[i] * L.versine;
    RG[0][0] += L.cos_t; RG[0][1] += -sc;     RG[0][2] += sb;
    RG[1][0] += sc;      RG[1][1] += L.cos_t; RG[1][2] += -sa;
    RG[2][0] += -sb;     RG[2][1] += sa;      RG[2][2] += L.cos_t;
    S va[6] = {T(0), T(0), T(0), T(0), T(0), T(0)};  // a, b, c, tx, ty, tz for this view
    for (int n = lane; n < N; n += kWave) {
      S v[3];
      if (n == 0) { v[0] = T(0); v[1] = T(0); v[2] = T(0); }
      else if (n == 1) { v[0] = T(1); v[1] = T(0); v[2] = T(0); }
      else if (n == 2) { v[0] = wp(0); v[1] = wp(1); v[2] = T(0); }
      else { v[0] = wp(3 * (n - 2)); v[1] = wp(3 * (n - 2) + 1); v[2] = wp(3 * (n - 2) + 2); }
      if (detach_points) { detach(v[0]); detach(v[1]); detach(v[2]); }
      const S dot = v[0] * w0 + v[1] * w1 + v[2] * w2;
      const S cr[3] = {w1 * v[2] - w2 * v[1], w2 * v[0] - w0 * v[2], w0 * v[1] - w1 * v[0]};
      S p[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) p[c] = v[c] * L.cos_t + L.versine * dot * wv[c] + cr[c] * L.sinc + tr(3 * m + c);
      if (detach_points) { detach(p[0]); detach(p[1]); detach(p[2]); }
      S mz = S(a.pixel_ratio) * p[0];
      mz = mz < S(T(0)) ? -mz : mz;
      S my = S(a.pixel_ratio) * p[1];
      my = my < S(T(0)) ? -my : my;
      mz = mz > my ? mz : my;
      mz = mz < S(a.min_z) ? S(a.min_z) : mz;  // clamp(min=): the bound carries no tangent
      const S z = p[2] > mz ? p[2] : mz;  // torch.maximum
      const S u = f * p[0] / z + cx, vv = f * p[1] / z + cy;
      const int pair = m * N + n;
      const T wgt = vs[pair] ? T(1) : T(0);
      const S du = u - S(tgt[2 * pair]), dv = vv - S(tgt[2 * pair + 1]);
      S au = du * S(wgt), av = dv * S(wgt);
      au = au < S(T(0)) ? -au : au;
      av = av < S(T(0)) ? -av : av;
      eu += S(a.scale) * au;
      ev += S(a.scale) * av;
      if (g) {
        const S ru = S(a.scale * wgt) * sign_of(du), rv = S(a.scale * wgt) * sign_of(dv);
        // _compute_gradient_from_intermediates
        const S mg = a.max_grad;
        const S inv_z = S(T(1)) / z;
        S sf = mg * inv_z;
        sf = sf > S(T(1)) ? S(T(1)) : sf;
        S mfm = mg / f;
        mfm = mfm < S(T(0)) ? -mfm : mfm;
        const S f_on_z = f * clip(inv_z, -mfm, mfm);
        const S x_on_z = p[0] * inv_z, y_on_z = p[1] * inv_z;
        const S du_dxp = clip(sf * f_on_z, -mg, mg);
        const S dv_dyp = clip(sf * f_on_z, -mg, mg);
        const S du_dzp = clip(-sf * f_on_z * x_on_z, -mg, mg);
        const S dv_dzp = clip(-sf * f_on_z * y_on_z, -mg, mg);
        const S du_df = clip(sf * x_on_z, -mg, mg);
        const S dv_df = clip(sf * y_on_z, -mg, mg);
        const S du_dtx = clip(sf * du_dxp, -mg, mg);
        const S dv_dty = clip(sf * dv_dyp, -mg, mg);
        const S du_dtz = clip(sf * du_dzp, -mg, mg);
        const S dv_dtz = clip(sf * dv_dzp, -mg, mg);
        // LieRotation.parameter_gradient(v): [i][j] = d rotated_i / d omega_j
        S OG[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const S t1 = S(T(-1)) * (v[i] * wv[j]) * L.sinc;
            const S t2 = (dot * L.d_term) * (wv[j] * wv[i]);
            const S t3 = L.versine * (v[j] * wv[i] + (i == j ? dot : S(T(0))));
            const S t4 = (wv[j] * cr[i]) * L.c_term;
            OG[i][j] = t1 + t2 + t3 + t4;
          }
        OG[0][1] += v[2] * L.sinc; OG[0][2] += -v[1] * L.sinc;
        OG[1][0] += -v[2] * L.sinc; OG[1][2] += v[0] * L.sinc;
        OG[2][0] += v[1] * L.sinc; OG[2][1] += -v[0] * L.sinc;
        gcx += ru;
        gcy += rv;
        gf += ru * du_df + rv * dv_df;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const S dua = clip(sf * (du_dxp * OG[0][j] + du_dzp * OG[2][j]), -mg, mg);
          const S dva = clip(sf * (dv_dyp * OG[1][j] + dv_dzp * OG[2][j]), -mg, mg);
          va[j] += ru * dua + rv * dva;
        }
        va[3] += ru * du_dtx;
        va[4] += rv * dv_dty;
        va[5] += ru * du_dtz + rv * dv_dtz;
        // world-point partials (the reference uses dv/dz' in du/dy)
        const S du_dx = clip(sf * (du_dxp * RG[0][0] + du_dzp * RG[2][0]), -mg, mg);
        const S dv_dx = clip(sf * (dv_dyp * RG[1][0] + dv_dzp * RG[2][0]), -mg, mg);
        const S du_dy = clip(sf * (du_dxp * RG[0][1] + dv_dzp * RG[2][1]), -mg, mg);
        const S dv_dy = clip(sf * (dv_dyp * RG[1][1] + dv_dzp * RG[2][1]), -mg, mg);
        const S du_dz = clip(sf * (du_dxp * RG[0][2] + du_dzp * RG[2][2]), -mg, mg);
        const S dv_dz = clip(sf * (dv_dyp * RG[1][2] + dv_dzp * RG[2][2]), -mg, mg);
        S* q = pp + ((int64_t)pair) * 4;
        q[0] = ru * du_dx;
        q[1] = rv * dv_dx;
        q[2] = ru * du_dy + rv * dv_dy;
        q[3] = ru * du_dz + rv * dv_dz;
      }
    }
    if (g) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const S s = wave_sum(va[k]);
        if (lane == 0) {
          const int off = k == 0 ? oa : k == 1 ? ob : k == 2 ? oc : k == 3 ? otx : k == 4 ? oty : otz;
          store_grad(off + m, s);
        }
      }
    }
  }
  // globals: wave partials added in wave order
  S r5[5] = {eu, ev, gcx, gcy, gf};
  __shared__ S gl[kWaves][5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const S s = wave_sum(r5[k]);
    if (lane == 0) gl[wave][k] = s;
  }
  __syncthreads();
  if (tid == 0) {
    S t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = ((gl[0][k] + gl[1][k]) + gl[2][k]) + gl[3][k];
    store_err(t[0] + t[1]);
    if (g) { store_grad(0, t[2]); store_grad(1, t[3]); store_grad(2, t[4]); }
  }
  if (g) {
    // world points n >= 2: sums over views in view order
    for (int n = 2 + tid; n < N; n += kBlock) {
      S sx0 = T(0), sx1 = T(0), sy = T(0), sz = T(0);
      for (int m = 0; m < M; ++m) {
        const S* q = pp + ((int64_t)(m * N + n)) * 4;
        sx0 += q[0]; sx1 += q[1]; sy += q[2]; sz += q[3];
      }
      store_grad(ox + (n - 2), sx0 + sx1);
      store_grad(oy + (n - 2), sy);
      if (n >= 3) store_grad(oz + (n - 3), sz);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void l1_camera_kernel(L1Args<T> a) {
  const int64_t be = blockIdx.x;  // (b, e) flattened
  T* g = a.grad ? a.grad + be * a.P : nullptr;
  l1_body<T, T>(a, be, -1, g != nullptr, false, [&](T e) { if (a.err) a.err[be] = e; },
                [&](int i, T v) { g[i] = v; });
}

// Reverse mode for autograd through the model, one forward-mode pass per input direction:
// workgroup (be, d) evaluates estimate be with tangent 1 on its input element d and contracts the
// output tangents with the cotangents, vjp[be, d] = e_bar[be] de/dd + sum_q g_bar[be, q] dg_q/dd
// (error_cot / grad_cot may be null).  The sum is per thread in a fixed order, then wave
// butterflies and the 4 wave partials in wave order: deterministic.
template <typename T>
__global__ __launch_bounds__(kBlock) void l1_camera_vjp_kernel(L1Args<T> a, int D, const T* error_cot,
                                                                const T* grad_cot, int detach_points, T* vjp) {
  const int64_t be = blockIdx.x / D;
  const int d = blockIdx.x % D;
  const T* gb = grad_cot ? grad_cot + be * a.P : nullptr;
  T acc = T(0);
  l1_body<T, LDual<T>>(a, be, d, gb != nullptr, detach_points != 0,
                       [&](LDual<T> e) { if (error_cot) acc += error_cot[be] * e.t; },
                       [&](int i, LDual<T> v) { acc += gb[i] * v.t; });
  __shared__ T red[kWaves];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  acc = wave_sum(acc);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) vjp[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

template <typename T>
L1Args<T> l1_args(int64_t estimates, int32_t views, int32_t points, const T* focal, const T* cx, const T* cy,
                  const T* trans, const T* lie, const T* world, const T* target, const uint8_t* vis, T min_z,
                  T pixel_ratio, T max_grad, T scale) {
  L1Args<T> a;
  a.M = views; a.N = points; a.P = 3 + 6 * views + 3 * points - 7; a.E = (int)estimates;
  a.focal = focal; a.cx = cx; a.cy = cy; a.trans = trans; a.lie = lie; a.world = world; a.target = target;
  a.vis = vis; a.min_z = min_z; a.pixel_ratio = pixel_ratio; a.max_grad = max_grad; a.scale = scale;
  a.err = nullptr; a.grad = nullptr;
  return a;
}

template <typename T>
int l1_camera_vjp(int64_t batch, int32_t estimates, int32_t views, int32_t points, const T* focal, const T* cx,
                  const T* cy, const T* trans, const T* lie, const T* world, const T* target, const uint8_t* vis,
                  T min_z, T pixel_ratio, T max_grad, T scale, const T* error_cot, const T* grad_cot,
                  int32_t detach_points, T* vjp, void* stream) {
  if (batch < 0 || estimates < 0 || views < 1 || points < 3) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || estimates == 0) return DAVA_OK;
  if (!focal || !cx || !cy || !trans || !lie || !world || !target || !vis || !vjp) return DAVA_ERR_INVALID_ARGUMENT;
  const int64_t D = 3 + 6 * (int64_t)views + 3 * ((int64_t)points - 2);
  if (batch * estimates * D > 0x7fffffff) return DAVA_ERR_UNSUPPORTED;
  const size_t lds = grad_cot ? (size_t)views * points * 4 * sizeof(LDual<T>) : 0;
  if (lds > 150 * 1024) return DAVA_ERR_UNSUPPORTED;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(l1_camera_vjp_kernel<T>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const L1Args<T> a = l1_args(estimates, views, points, focal, cx, cy, trans, lie, world, target, vis, min_z,
                              pixel_ratio, max_grad, scale);
  hipLaunchKernelGGL(l1_camera_vjp_kernel<T>, dim3((unsigned)(batch * estimates * D)), dim3(kBlock), lds,
                     static_cast<hipStream_t>(stream), a, (int)D, error_cot, grad_cot, (int)detach_points, vjp);
  return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH;
}

template <typename T>
int l1_camera_evaluate(int64_t batch, int32_t estimates, int32_t views, int32_t points, const T* focal, const T* cx,
                       const T* cy, const T* trans, const T* lie, const T* world, const T* target,
                       const uint8_t* vis, T min_z, T pixel_ratio, T max_grad, T scale, T* err, T* grad,
                       void* stream) {
  if (batch < 0 || estimates < 0 || views < 1 || points < 3) return DAVA_ERR_INVALID_ARGUMENT;
  if (batch == 0 || estimates == 0) return DAVA_OK;
  if (!focal || !cx || !cy || !trans || !lie || !world || !target || !vis) return DAVA_ERR_INVALID_ARGUMENT;
  if (!err && !grad) return DAVA_OK;
  const size_t lds = grad ? (size_t)views * points * 4 * sizeof(T) : 0;
  if (lds > 150 * 1024) return DAVA_ERR_UNSUPPORTED;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(l1_camera_kernel<T>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  L1Args<T> a = l1_args(estimates, views, points, focal, cx, cy, trans, lie, world, target, vis, min_z, pixel_ratio,
                        max_grad, scale);
  a.err = err; a.grad = grad;
  hipLaunchKernelGGL(l1_camera_kernel<T>, dim3((unsigned)(batch * estimates)), dim3(kBlock), lds,
                     static_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH;
}

}  // namespace dava

using namespace dava;

#define DAVA_L1_ENTRY(SUFFIX, T)                                                                                 \
  extern "C" int dava_l1_camera_evaluate_##SUFFIX(                                                              \
      int64_t batch, int32_t estimates, int32_t views, int32_t points, const T* focal, const T* cx, const T* cy,  \
      const T* translation, const T* lie_vector, const T* world_points, const T* true_points,                    \
      const uint8_t* visibility, T minimum_z_distance, T inverse_pixel_ratio, T max_gradient, T error_scale,     \
      T* error_out, T* gradient_out, void* stream) {                                                             \
    return l1_camera_evaluate<T>(batch, estimates, views, points, focal, cx, cy, translation, lie_vector,        \
                                 world_points, true_points, visibility, minimum_z_distance, inverse_pixel_ratio, \
                                 max_gradient, error_scale, error_out, gradient_out, stream);                    \
  }

DAVA_L1_ENTRY(f32, float)
DAVA_L1_ENTRY(f64, double)

#define DAVA_L1_VJP_ENTRY(SUFFIX, T)                                                                             \
  extern "C" int dava_l1_camera_vjp_##SUFFIX(                                                                   \
      int64_t batch, int32_t estimates, int32_t views, int32_t points, const T* focal, const T* cx, const T* cy,  \
      const T* translation, const T* lie_vector, const T* world_points, const T* true_points,                    \
      const uint8_t* visibility, T minimum_z_distance, T inverse_pixel_ratio, T max_gradient, T error_scale,     \
      const T* error_cotangent, const T* gradient_cotangent, int32_t detach_points, T* input_cotangent_out,      \
      void* stream) {                                                                                            \
    return l1_camera_vjp<T>(batch, estimates, views, points, focal, cx, cy, translation, lie_vector,            \
                            world_points, true_points, visibility, minimum_z_distance, inverse_pixel_ratio,      \
                            max_gradient, error_scale, error_cotangent, gradient_cotangent, detach_points,       \
                            input_cotangent_out, stream);                                                        \
  }

DAVA_L1_VJP_ENTRY(f32, float)
DAVA_L1_VJP_ENTRY(f64, double)
