// Shared device helpers for the gfx950 BA solver (wave64, 256-thread workgroups).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dava_ba.h"

namespace dava {

constexpr int kWave = 64;        // CDNA wavefront width
constexpr int kBlock = 256;      // one problem per 256-thread workgroup (4 waves)
constexpr int kWaves = kBlock / kWave;

__host__ __device__ inline int round_up(int v, int m) { return (v + m - 1) / m * m; }

// torch.clamp(min=lo) semantics: NaN propagates (fmaxf would swallow it).
template <typename T>
__device__ __forceinline__ T clamp_min(T v, T lo) { return v < lo ? lo : v; }

// sign() as torch.abs backward uses it: 0 at 0.
__device__ __forceinline__ float sgn(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// fp32 all-lanes wave sum entirely in registers (gfx950): DPP butterflies inside each
// 16-lane row, then v_permlane16_swap / v_permlane32_swap across rows.  12 VALU ops;
// the __shfl_xor form costs an LDS round trip (ds_bpermute) plus index math per step.
template <>
__device__ __forceinline__ float wave_sum<float>(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
  v += dpp_mov<0x141>(v);  // row_half_mirror: xor 4 on quad-uniform data
  v += dpp_mov<0x140>(v);  // row_mirror: xor 8 on 8-lane-uniform data
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);  // xor 16
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);  // xor 32
}

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

// packed fp32 FMA (v_pk_fma_f32): a * b + c on two lanes of a float pair
__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
// k * v + c on a float4 as two packed FMAs
__device__ __forceinline__ f4v pk_fma4(float k, f4v v, f4v c) {
  const f2v kk = {k, k};
  const f2v lo = pk_fma(kk, v.lo, c.lo), hi = pk_fma(kk, v.hi, c.hi);
  return f4v{lo.x, lo.y, hi.x, hi.y};
}

__device__ __forceinline__ float lane_value(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Sums of FOUR per-lane values over the wave, returned wave-uniform (read out of fixed lanes, so
// SGPR-resident and bit-identical for every lane).  A transposed butterfly: the xor-32 step
// exchanges half of the value SET between the lane halves (v0, v1 stay low, v2, v3 go high) and
// the xor-16 step half of what is left, so each 16-lane row ends up reducing ONE value with four
// DPP steps -- 14 VALU ops for the four sums instead of 4 x 8 for four wave_sum calls.
// (v_permlane32_swap: lanes 32-63 of the first operand <-> lanes 0-31 of the second;
//  v_permlane16_swap: odd rows of the first <-> even rows of the second.)
__device__ __forceinline__ float4 wave_sum4(float v0, float v1, float v2, float v3) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v0), __float_as_uint(v2), false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v1), __float_as_uint(v3), false, false);
  const float h0 = __uint_as_float(a[0]) + __uint_as_float(a[1]);  // lanes 0-31: v0, lanes 32-63: v2
  const float h1 = __uint_as_float(b[0]) + __uint_as_float(b[1]);  // lanes 0-31: v1, lanes 32-63: v3
  const auto c = __builtin_amdgcn_permlane16_swap(__float_as_uint(h0), __float_as_uint(h1), false, false);
  float r = __uint_as_float(c[0]) + __uint_as_float(c[1]);  // 16-lane row q holds value q
  r += dpp_mov<0xB1>(r);
  r += dpp_mov<0x4E>(r);
  r += dpp_mov<0x141>(r);
  r += dpp_mov<0x140>(r);
  return make_float4(lane_value(r, 0), lane_value(r, 16), lane_value(r, 32), lane_value(r, 48));
}

// Wave sums of R values in place (wave-uniform results), four at a time through wave_sum4.
template <int R>
__device__ __forceinline__ void wave_sums(float (&v)[R]) {
#pragma unroll
  for (int r = 0; r < R; r += 4) {
    const float4 t = wave_sum4(v[r], r + 1 < R ? v[r + 1] : 0.f, r + 2 < R ? v[r + 2] : 0.f,
                               r + 3 < R ? v[r + 3] : 0.f);
    v[r] = t.x;
    if (r + 1 < R) v[r + 1] = t.y;
    if (r + 2 < R) v[r + 2] = t.z;
    if (r + 3 < R) v[r + 3] = t.w;
  }
}

// Deterministic block-wide sum of R values: wave butterflies, then the 4 wave
// partials are added in a fixed order by every thread, so all threads hold
// bit-identical results (the solver's control flow depends on them being
// uniform).  `scratch` is double-buffered by the caller (alternate `buf`),
// so ONE barrier per reduction suffices (NW = waves in the workgroup): a wave cannot reach the next use of
// the same buffer before every wave has passed the intervening reduction's
// barrier, i.e. before every wave finished reading this one.
// SCALAR_WAVE: the wave index as a scalar (readfirstlane), so the partials' LDS address needs no
// long-lived VGPR -- for the LDS-staged history passes, where a spilled address reload (a scratch load
// and its vmcnt wait) would also wait for the staged copies in flight.
template <int R, int NW = kWaves, bool SCALAR_WAVE = false>
__device__ __forceinline__ void block_sum(float (&v)[R], float* scratch, int buf) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = SCALAR_WAVE ? __builtin_amdgcn_readfirstlane(threadIdx.x / kWave) : threadIdx.x / kWave;
  float* s = scratch + buf * (NW * 32);
  if constexpr (R >= 2) {
    float w[R];
#pragma unroll
    for (int r = 0; r < R; ++r) w[r] = v[r];
    wave_sums<R>(w);
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane == 0) s[wave * 32 + r] = w[r];
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float w = wave_sum(v[r]);
      if (lane == 0) s[wave * 32 + r] = w;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float t = s[r];  // wave partials added in wave order
#pragma unroll
    for (int w = 1; w < NW; ++w) t += s[w * 32 + r];
    v[r] = t;
  }
}

// Buffer loads (SRD in SGPRs, 32-bit per-lane byte offset): no 64-bit address arithmetic per
// load, and the descriptor's range check returns zeros past `bytes` with no branch.
typedef float f4buf __attribute__((ext_vector_type(4)));
__device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<const float*>(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ f4buf buf_ld4(__amdgpu_buffer_rsrc_t r, int voff) {
  return __builtin_bit_cast(f4buf, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}

// Sum of NW per-wave partials stored `stride` apart, in wave order.
template <int NW, typename T>
__device__ __forceinline__ T wave_partials_total(const T* p, int stride) {
  T t = p[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) t += p[w * stride];
  return t;
}

}  // namespace dava
