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

// Deterministic block-wide sum of R values: wave butterflies, then the 4 wave
// partials are added in a fixed order by every thread, so all threads hold
// bit-identical results (the solver's control flow depends on them being
// uniform).  `scratch` is double-buffered by the caller (alternate `buf`),
// so ONE barrier per reduction suffices (NW = waves in the workgroup): a wave cannot reach the next use of
// the same buffer before every wave has passed the intervening reduction's
// barrier, i.e. before every wave finished reading this one.
template <int R, int NW = kWaves>
__device__ __forceinline__ void block_sum(float (&v)[R], float* scratch, int buf) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  float* s = scratch + buf * (NW * 32);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float w = wave_sum(v[r]);
    if (lane == 0) s[wave * 32 + r] = w;
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

// Sum of NW per-wave partials stored `stride` apart, in wave order.
template <int NW, typename T>
__device__ __forceinline__ T wave_partials_total(const T* p, int stride) {
  T t = p[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) t += p[w * stride];
  return t;
}

}  // namespace dava
