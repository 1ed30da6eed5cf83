// Forward-mode dual numbers for second derivatives of the BA objectives.
//
// The objective's reverse-mode gradient code (ba_objective.hpp) is templated on
// its scalar type; instantiated with Dual {value, tangent} and the parameters
// seeded with a direction v, the same code returns grad E (values) and the
// Hessian-vector product H v (tangents) -- forward-over-reverse, exactly the
// second derivative of the first derivative the solver uses.  This is what
// differentiating THROUGH a solve needs from the objective (the reference gets
// it from autograd's double backward, bfgs_solver.py:133-135 create_graph).
#pragma once

#include <hip/hip_runtime.h>

#include "dava_common.hpp"

namespace dava {

struct Dual {
  float v, t;
  __device__ __forceinline__ Dual() = default;
  __device__ __forceinline__ constexpr Dual(float value) : v(value), t(0.0f) {}  // NOLINT: constants
  __device__ __forceinline__ constexpr Dual(float value, float tangent) : v(value), t(tangent) {}
};

__device__ __forceinline__ Dual operator+(Dual a, Dual b) { return {a.v + b.v, a.t + b.t}; }
__device__ __forceinline__ Dual operator-(Dual a, Dual b) { return {a.v - b.v, a.t - b.t}; }
__device__ __forceinline__ Dual operator-(Dual a) { return {-a.v, -a.t}; }
__device__ __forceinline__ Dual operator*(Dual a, Dual b) { return {a.v * b.v, a.t * b.v + a.v * b.t}; }
__device__ __forceinline__ Dual operator/(Dual a, Dual b) {
  const float q = a.v / b.v;
  return {q, (a.t - q * b.t) / b.v};
}
__device__ __forceinline__ Dual operator+(Dual a, float b) { return {a.v + b, a.t}; }
__device__ __forceinline__ Dual operator+(float a, Dual b) { return {a + b.v, b.t}; }
__device__ __forceinline__ Dual operator-(Dual a, float b) { return {a.v - b, a.t}; }
__device__ __forceinline__ Dual operator-(float a, Dual b) { return {a - b.v, -b.t}; }
__device__ __forceinline__ Dual operator*(Dual a, float b) { return {a.v * b, a.t * b}; }
__device__ __forceinline__ Dual operator*(float a, Dual b) { return {a * b.v, a * b.t}; }
__device__ __forceinline__ Dual operator/(Dual a, float b) { return {a.v / b, a.t / b}; }
__device__ __forceinline__ Dual operator/(float a, Dual b) {
  const float q = a / b.v;
  return {q, -q * b.t / b.v};
}
__device__ __forceinline__ Dual& operator+=(Dual& a, Dual b) { return a = a + b; }
__device__ __forceinline__ Dual& operator-=(Dual& a, Dual b) { return a = a - b; }
__device__ __forceinline__ Dual& operator*=(Dual& a, Dual b) { return a = a * b; }
// branches and clamps follow the value (their derivative is the taken branch's)
__device__ __forceinline__ bool operator<(Dual a, Dual b) { return a.v < b.v; }
__device__ __forceinline__ bool operator>(Dual a, Dual b) { return a.v > b.v; }
__device__ __forceinline__ bool operator<=(Dual a, Dual b) { return a.v <= b.v; }
__device__ __forceinline__ bool operator>=(Dual a, Dual b) { return a.v >= b.v; }
__device__ __forceinline__ bool operator==(Dual a, Dual b) { return a.v == b.v; }

// ---- elementary functions, float and Dual ----
__device__ __forceinline__ float sqrt_(float x) { return sqrtf(x); }
__device__ __forceinline__ float sin_(float x) { return sinf(x); }
__device__ __forceinline__ float cos_(float x) { return cosf(x); }
__device__ __forceinline__ float fabs_(float x) { return fabsf(x); }
__device__ __forceinline__ float exp_(float x) { return expf(x); }
__device__ __forceinline__ float expm1_(float x) { return expm1f(x); }
__device__ __forceinline__ float atan2_(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ float fmul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd_rn(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float value_of(float x) { return x; }

__device__ __forceinline__ Dual sqrt_(Dual x) {
  const float r = sqrtf(x.v);
  return {r, r > 0.0f ? x.t / (2.0f * r) : 0.0f};  // torch: 0 subgradient handled by callers' norms
}
__device__ __forceinline__ Dual sin_(Dual x) { return {sinf(x.v), cosf(x.v) * x.t}; }
__device__ __forceinline__ Dual cos_(Dual x) { return {cosf(x.v), -sinf(x.v) * x.t}; }
__device__ __forceinline__ Dual fabs_(Dual x) { return {fabsf(x.v), sgn(x.v) * x.t}; }
__device__ __forceinline__ Dual exp_(Dual x) {
  const float e = expf(x.v);
  return {e, e * x.t};
}
__device__ __forceinline__ Dual expm1_(Dual x) { return {expm1f(x.v), expf(x.v) * x.t}; }
__device__ __forceinline__ Dual atan2_(Dual y, Dual x) {
  const float den = x.v * x.v + y.v * y.v;
  return {atan2f(y.v, x.v), (x.v * y.t - y.v * x.t) / den};
}
// sin and cos of one argument through one range reduction
__device__ __forceinline__ void sincos_(float x, float& s, float& c) { sincosf(x, &s, &c); }
__device__ __forceinline__ void sincos_(Dual x, Dual& s, Dual& c) {
  float sv, cv;
  sincosf(x.v, &sv, &cv);
  s = {sv, cv * x.t};
  c = {cv, -sv * x.t};
}
__device__ __forceinline__ Dual fmul_rn(Dual a, Dual b) { return a * b; }
__device__ __forceinline__ Dual fadd_rn(Dual a, Dual b) { return a + b; }
__device__ __forceinline__ float value_of(Dual x) { return x.v; }
// sign(x) as torch.abs backward uses it: piecewise constant, zero derivative
__device__ __forceinline__ Dual sgn(Dual x) { return Dual(sgn(x.v)); }
__device__ __forceinline__ Dual clamp_min(Dual v, float lo) { return v.v < lo ? Dual(lo) : v; }

template <>
__device__ __forceinline__ Dual wave_sum<Dual>(Dual x) {
  return {wave_sum<float>(x.v), wave_sum<float>(x.t)};
}

// block_sum over R duals = block_sum over the 2R floats they are made of
template <int R, int NW = kWaves>
__device__ __forceinline__ void block_sum(Dual (&v)[R], float* scratch, int buf) {
  static_assert(2 * R <= 32, "scratch rows hold 32 floats");
  block_sum<2 * R, NW>(reinterpret_cast<float(&)[2 * R]>(v), scratch, buf);
}

}  // namespace dava
