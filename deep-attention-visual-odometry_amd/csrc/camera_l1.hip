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

template <typename T>
struct L1Args {
  int M, N, P, E;
  const T *focal, *cx, *cy, *trans, *lie, *world, *target;
  const uint8_t* vis;
  T min_z, pixel_ratio, max_grad, scale;
  T *err, *grad;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void l1_camera_kernel(L1Args<T> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* pp = reinterpret_cast<T*>(smem);  // [M][N][4] per-view point-gradient terms
  const int M = a.M, N = a.N, P = a.P;
  const int64_t be = blockIdx.x;      // (b, e) flattened
  const int64_t b = be / a.E;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const T f = a.focal[be], cx = a.cx[be], cy = a.cy[be];
  const T* tr = a.trans + be * M * 3;
  const T* om = a.lie + be * M * 3;
  const T* wp = a.world + be * (int64_t)(N - 2) * 3;
  const T* tgt = a.target + b * (int64_t)M * N * 2;
  const uint8_t* vs = a.vis + b * (int64_t)M * N;
  T* g = a.grad ? a.grad + be * P : nullptr;
  // parameter offsets (pinhole_camera_model_l1.py:366-378)
  const int oa = 3, ob = oa + M, oc = ob + M, otx = oc + M, oty = otx + M, otz = oty + M;
  const int ox = otz + M, oy = ox + (N - 2), oz = oy + (N - 2);

  T eu = 0, ev = 0, gcx = 0, gcy = 0, gf = 0;
  for (int m = wave; m < M; m += kWaves) {
    const T w0 = om[3 * m], w1 = om[3 * m + 1], w2 = om[3 * m + 2];
    const T th = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const LieTrig<T> L = lie_trig(th);
    // LieRotation.vector_gradient: A w w^T + [[cos, -c, b], [c, cos, -a], [-b, a, cos]], (a,b,c) = w sinc
    const T sa = w0 * L.sinc, sb = w1 * L.sinc, sc = w2 * L.sinc;
    T RG[3][3];
    const T wv[3] = {w0, w1, w2};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) RG[i][j] = wv[j] * wv[i] * L.versine;
    RG[0][0] += L.cos_t; RG[0][1] += -sc;     RG[0][2] += sb;
    RG[1][0] += sc;      RG[1][1] += L.cos_t; RG[1][2] += -sa;
    RG[2][0] += -sb;     RG[2][1] += sa;      RG[2][2] += L.cos_t;
    T va[6] = {0, 0, 0, 0, 0, 0};  // a, b, c, tx, ty, tz for this view
    for (int n = lane; n < N; n += kWave) {
      T v[3];
      if (n == 0) { v[0] = 0; v[1] = 0; v[2] = 0; }
      else if (n == 1) { v[0] = 1; v[1] = 0; v[2] = 0; }
      else if (n == 2) { v[0] = wp[0]; v[1] = wp[1]; v[2] = 0; }
      else { v[0] = wp[3 * (n - 2)]; v[1] = wp[3 * (n - 2) + 1]; v[2] = wp[3 * (n - 2) + 2]; }
      const T dot = v[0] * w0 + v[1] * w1 + v[2] * w2;
      const T cr[3] = {w1 * v[2] - w2 * v[1], w2 * v[0] - w0 * v[2], w0 * v[1] - w1 * v[0]};
      T p[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) p[c] = v[c] * L.cos_t + L.versine * dot * wv[c] + cr[c] * L.sinc + tr[3 * m + c];
      T mz = a.pixel_ratio * p[0];
      mz = mz < T(0) ? -mz : mz;
      T my = a.pixel_ratio * p[1];
      my = my < T(0) ? -my : my;
      mz = mz > my ? mz : my;
      mz = clamp_min(mz, a.min_z);
      const T z = p[2] > mz ? p[2] : mz;  // torch.maximum
      const T u = f * p[0] / z + cx, vv = f * p[1] / z + cy;
      const int pair = m * N + n;
      const T wgt = vs[pair] ? T(1) : T(0);
      const T du = u - tgt[2 * pair], dv = vv - tgt[2 * pair + 1];
      T au = du * wgt, av = dv * wgt;
      au = au < T(0) ? -au : au;
      av = av < T(0) ? -av : av;
      eu += a.scale * au;
      ev += a.scale * av;
      if (g) {
        const T ru = a.scale * wgt * sign_of(du), rv = a.scale * wgt * sign_of(dv);
        // _compute_gradient_from_intermediates
        const T mg = a.max_grad;
        const T inv_z = T(1) / z;
        T sf = mg * inv_z;
        sf = sf > T(1) ? T(1) : sf;
        T mfm = mg / f;
        mfm = mfm < T(0) ? -mfm : mfm;
        const T f_on_z = f * clip(inv_z, -mfm, mfm);
        const T x_on_z = p[0] * inv_z, y_on_z = p[1] * inv_z;
        const T du_dxp = clip(sf * f_on_z, -mg, mg);
        const T dv_dyp = clip(sf * f_on_z, -mg, mg);
        const T du_dzp = clip(-sf * f_on_z * x_on_z, -mg, mg);
        const T dv_dzp = clip(-sf * f_on_z * y_on_z, -mg, mg);
        const T du_df = clip(sf * x_on_z, -mg, mg);
        const T dv_df = clip(sf * y_on_z, -mg, mg);
        const T du_dtx = clip(sf * du_dxp, -mg, mg);
        const T dv_dty = clip(sf * dv_dyp, -mg, mg);
        const T du_dtz = clip(sf * du_dzp, -mg, mg);
        const T dv_dtz = clip(sf * dv_dzp, -mg, mg);
        // LieRotation.parameter_gradient(v): [i][j] = d rotated_i / d omega_j
        T OG[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const T t1 = T(-1) * (v[i] * wv[j]) * L.sinc;
            const T t2 = (dot * L.d_term) * (wv[j] * wv[i]);
            const T t3 = L.versine * (v[j] * wv[i] + (i == j ? dot : T(0)));
            const T t4 = (wv[j] * cr[i]) * L.c_term;
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
          const T dua = clip(sf * (du_dxp * OG[0][j] + du_dzp * OG[2][j]), -mg, mg);
          const T dva = clip(sf * (dv_dyp * OG[1][j] + dv_dzp * OG[2][j]), -mg, mg);
          va[j] += ru * dua + rv * dva;
        }
        va[3] += ru * du_dtx;
        va[4] += rv * dv_dty;
        va[5] += ru * du_dtz + rv * dv_dtz;
        // world-point partials (the reference uses dv/dz' in du/dy)
        const T du_dx = clip(sf * (du_dxp * RG[0][0] + du_dzp * RG[2][0]), -mg, mg);
        const T dv_dx = clip(sf * (dv_dyp * RG[1][0] + dv_dzp * RG[2][0]), -mg, mg);
        const T du_dy = clip(sf * (du_dxp * RG[0][1] + dv_dzp * RG[2][1]), -mg, mg);
        const T dv_dy = clip(sf * (dv_dyp * RG[1][1] + dv_dzp * RG[2][1]), -mg, mg);
        const T du_dz = clip(sf * (du_dxp * RG[0][2] + du_dzp * RG[2][2]), -mg, mg);
        const T dv_dz = clip(sf * (dv_dyp * RG[1][2] + dv_dzp * RG[2][2]), -mg, mg);
        T* q = pp + ((int64_t)pair) * 4;
        q[0] = ru * du_dx;
        q[1] = rv * dv_dx;
        q[2] = ru * du_dy + rv * dv_dy;
        q[3] = ru * du_dz + rv * dv_dz;
      }
    }
    if (g) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const T s = wave_sum(va[k]);
        if (lane == 0) {
          const int off = k == 0 ? oa : k == 1 ? ob : k == 2 ? oc : k == 3 ? otx : k == 4 ? oty : otz;
          g[off + m] = s;
        }
      }
    }
  }
  // globals: wave partials added in wave order
  T r5[5] = {eu, ev, gcx, gcy, gf};
  __shared__ T gl[kWaves][5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const T s = wave_sum(r5[k]);
    if (lane == 0) gl[wave][k] = s;
  }
  __syncthreads();
  if (tid == 0) {
    T t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = ((gl[0][k] + gl[1][k]) + gl[2][k]) + gl[3][k];
    if (a.err) a.err[be] = t[0] + t[1];
    if (g) { g[0] = t[2]; g[1] = t[3]; g[2] = t[4]; }
  }
  if (g) {
    // world points n >= 2: sums over views in view order
    for (int n = 2 + tid; n < N; n += kBlock) {
      T sx0 = 0, sx1 = 0, sy = 0, sz = 0;
      for (int m = 0; m < M; ++m) {
        const T* q = pp + ((int64_t)(m * N + n)) * 4;
        sx0 += q[0]; sx1 += q[1]; sy += q[2]; sz += q[3];
      }
      g[ox + (n - 2)] = sx0 + sx1;
      g[oy + (n - 2)] = sy;
      if (n >= 3) g[oz + (n - 3)] = sz;
    }
  }
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
  L1Args<T> a;
  a.M = views; a.N = points; a.P = 3 + 6 * views + 3 * points - 7; a.E = estimates;
  a.focal = focal; a.cx = cx; a.cy = cy; a.trans = trans; a.lie = lie; a.world = world; a.target = target;
  a.vis = vis; a.min_z = min_z; a.pixel_ratio = pixel_ratio; a.max_grad = max_grad; a.scale = scale;
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
