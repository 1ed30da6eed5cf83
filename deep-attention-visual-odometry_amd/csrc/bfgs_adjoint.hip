// Reverse mode of the fused compact BFGS solve: d x_out / d (x0, observations) applied to a
// cotangent, one workgroup per problem, replaying the recorded solve (dava_tape.hpp) backwards.
//
// Replaces, for the fused objectives, differentiating THROUGH BFGSSolver.forward the way the
// reference does (create_graph, autograd_solvers/bfgs_solver.py:85, :133-135, :213-215): every
// iteration's gradient is taken with create_graph, the inverse-Hessian scale and update
// (:159-180, :217-303, utils/func_inverse_curvature.py:21-51) and d = -H g are differentiated, the
// step size of the line search is a constant (it is computed without a graph).
//
// Forward (per problem, k = 0 .. n-1, n = the steps the solve took):
//   g_k = dE/dx(x_k; obs)            d_0 = -g_0,   d_k = -H_k g_k
//   H_k = H_{k-1} + c rho s s^T - rho s w^T - rho w s^T   (entry k-1: s = s_{k-1}, y = g_k - g_{k-1},
//         w = H_{k-1} y, rho = 1 / (s.y) (0 if s.y <= 0), c = 1 + rho y.w),  H_0' = gamma I,
//         gamma = clamp(s_0.y_1 / clamp(y_1.y_1, 1e-5), min 1e-4)
//   s_k = alpha_k d_k,  x_{k+1} = x_k + s_k
// Reverse, with A = adjoint of H_k kept as a sum of outer products sum_j a_j g_j^T: every term the
// forward adds to the adjoint of an inverse Hessian is -dbar_j g_j^T (from d_j = -H_j g_j) or
// wbar_j y_j^T = wbar_j (g_j - g_{j-1})^T (from w_j = H_{j-1} y_j), so ONE row a_j per iteration
// holds all of them (rows a_j in the workspace, g_j in the tape).  Only the symmetric part of A
// is ever contracted (s^T A s, (A + A^T) s, (A + A^T) w, tr A), so the reference's separate
// y^T H / H y products need no separate treatment.  Step k:
//   sbar = xbar + sbar_pend,  dbar = alpha_k sbar
//   k >= 1:  a_k -= dbar;  P1 = (A + A^T) s,  P2 = (A + A^T) w   (one pass over a_j, g_j, j >= k)
//            cbar = rho s.P1 / 2,  rhobar = c s.P1 / 2 - s.P2 + cbar y.w,  tbar = -rho^2 rhobar (s.y > 0)
//            sbar_pend' = c rho P1 - rho P2 + tbar y,  wbar = -rho P1 + cbar rho y
//            ybar = cbar rho w + tbar s + H_{k-1} wbar
//            gbar_k = gbar_pend - H_k dbar + ybar,  gbar_pend' = -ybar,  a_k += wbar,  a_{k-1} = -wbar
//            k = 1: gammabar = tr A = sum_j a_j . g_j, through both clamps into s_0 and y_1
//   k = 0:   gbar_0 = gbar_pend - dbar
//   xbar += Hess E(x_k) gbar_k,  obsbar += (d2E / dobs dx) gbar_k    (forward-over-reverse, Dual)
// H_k dbar and H_{k-1} wbar come from one pass over the history rows (s_j, w_j), like the forward's.
#include "ba_objective.hpp"
#include "dava_debug.hpp"
#include "dava_tape.hpp"

namespace dava {

typedef float f4a __attribute__((ext_vector_type(4)));

struct AdjointArgs {
  Layout L;
  int Pv, K;
  TapeLayout tl;
  const float* tape;
  const float* obs;
  const uint8_t* vis;
  const int32_t* status;
  const float* xbar;  // (B, P) cotangent of x_out
  float* x0_grad;     // (B, P)
  float* obs_grad;    // (B, M, N, 2) or null
  float* arows;       // (B, K, Pv) workspace
  int lcap;           // history entries (s_j, w_j), j < lcap, held in LDS for the H passes
  float* gvws;        // global-vector mode: (B, kAdjGvFloats(Pv)) per-problem vector slices, else null
  int gd_lds;         // global-vector mode: the HVP's dual gradient vector in LDS (carve_adjoint gdl)
  int sc_global;      // LDS mode: the tape's scalar row read in place (bfgs_ba_adjoint_kernel SCG)
};

constexpr int kAdjWaves = 4;
// Entries per wave in flight in the passes: at two workgroups per CU, 1 and 3 are slower
// (profiles/r03_ab_adjoint_inflight.log).  Measured and not kept: the row-streaming waves at
// priority 0 (C3 -1.7%, C2 +1%, profiles/r03_ab_adjoint_prio.log) and C1/C2-shape rows through
// buffer loads (C1 +1%, C2 +-1%, profiles/r03_ab_adjoint_buffer_loads.log).
constexpr int kAdjInflight = 2;
constexpr int kAdjBlock = kWave * kAdjWaves;
constexpr int kAdjMaxGroups = 14;  // GV mode: float4 groups per thread (P <= 14 * 256 * 4 = 14336)
constexpr int kAdjLdsBytes = 160 * 1024;

struct AdjointCarve {
  int xb, sbp, gbp, db, gk, p1, p2, wb, sv, wv, yv, gv, ak, an, sc, xd, gd, views, vpart, obs, obsacc, lh, scratch,
      vis_bytes_off, total_bytes;
  int gv_floats;  // global-vector mode: floats of one problem's workspace slice (the 14 vectors and 2 Dual ones)
};

// lcap: the oldest history entries' rows (s_j, w_j interleaved) kept on chip for the whole reverse
// sweep -- every H pass reads them again, so each one held saves 2 Pv floats of HBM per step.
// gv (global-vector mode, P too large for the LDS image, e.g. C5): the O(P) vectors are offsets into
// the problem's workspace slice instead, the scene is read in place and the observation cotangent is
// accumulated straight into the output; LDS keeps the scalars, view constants and reduction scratch.
// gdl (global-vector mode): the dual gradient vector of the HVP evaluation in LDS instead of the slice
// -- the evaluation accumulates it view after view, one dependent read-modify-write per pair.
__host__ __device__ inline AdjointCarve carve_adjoint(int M, int N, int Pv, int T, int lcap = 0, bool gv = false,
                                                     int nw = kAdjWaves, bool gdl = false) {
  AdjointCarve c;
  int off = 0, voff = 0;
  int& o = gv ? voff : off;
  int* vec[] = {&c.xb, &c.sbp, &c.gbp, &c.db, &c.gk, &c.p1, &c.p2, &c.wb, &c.sv, &c.wv, &c.yv, &c.gv, &c.ak, &c.an};
  for (int* v : vec) { *v = o; o += Pv; }
  c.sc = off; off += T;
  c.xd = o; o += 2 * Pv;  // Dual
  int& og = gv && gdl ? off : o;
  c.gd = og; og += 2 * Pv;  // Dual
  c.gv_floats = gv ? voff : 0;
  c.views = off; off += 2 * round_up(views_floats(M), 4);
  c.vpart = off; off += 2 * round_up(vpart_floats(M, nw), 4);
  c.obs = off; off += gv ? 0 : round_up(2 * M * N, 4);
  c.obsacc = off; off += gv ? 0 : round_up(2 * M * N, 4);
  c.lh = off; off += gv ? 0 : 2 * lcap * Pv;
  c.scratch = off; off += 2 * nw * 32;
  c.vis_bytes_off = off * 4;
  c.total_bytes = c.vis_bytes_off + (gv ? 0 : round_up(M * N, 16));
  return c;
}

__device__ __forceinline__ f4a ldv(const float* p) { return *reinterpret_cast<const f4a*>(p); }
__device__ __forceinline__ void stv(float* p, f4a v) { *reinterpret_cast<f4a*>(p) = v; }

// One pass over entries j0 .. j1-1 with rows R1[j], R2[j] (Pv floats, rows Pv apart): per entry the
// four dots d11 = R1.v1, d21 = R2.v1, d12 = R1.v2, d22 = R2.v2 (one transposed wave reduction),
// then out1 += k1 R1 + k2 R2, out2 += k3 R1 + k4 R2 with (k1..k4) = coef(j, d11, d21, d12, d22).
// Entries are dealt round-robin to the 4 waves (two in flight per wave); the wave partials are added
// in the fixed order (w0 + w2) + (w1 + w3), then base * (v1 | v2).  out / v / spares: LDS vectors.
// Ends with a barrier.
// R1_j0: if not null, entry j0's R1 row comes from this LDS vector instead of R1 + j0 Pv.
// LR, nl: entries j < nl have both rows in LDS, R1 at LR + 2 j Pv, R2 at LR + (2 j + 1) Pv.
// LDS-held rows are consumed in their own steps (each wave's entries in the same order), so the
// HBM rows are read with global loads only: a generic pointer that may point at LDS makes flat
// loads, which count on the LDS counter too and serialise every LDS read behind HBM latency.
template <int GM, class Coef>
__device__ __forceinline__ void pair_pass(int P, int Pv, int j0, int j1, const float* __restrict__ R1,
                                          const float* __restrict__ R2, const float* v1, const float* v2,
                                          float base, Coef coef, float* out1, float* out2, float* sp0, float* sp1,
                                          float* sp2, float* sp3, const float* R1_j0 = nullptr,
                                          const float* LR = nullptr, int nl = 0) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // scalar: row addresses wave-uniform
  const int G = (P + 3) / 4;
  f4a pa[GM], pb[GM];
  bool ok[GM];
#pragma unroll
  for (int m = 0; m < GM; ++m) {
    ok[m] = lane + kWave * m < G;
    pa[m] = pb[m] = f4a{0, 0, 0, 0};
  }
  auto load_from = [&](const float* r1p, const float* r2p, f4a (&r1)[GM], f4a (&r2)[GM]) {
#pragma unroll
    for (int m = 0; m < GM; ++m) {
      const int q = lane + kWave * m;
      r1[m] = ok[m] ? ldv(r1p + 4 * q) : f4a{0, 0, 0, 0};
      r2[m] = ok[m] ? ldv(r2p + 4 * q) : f4a{0, 0, 0, 0};
    }
  };
  // HBM rows
  auto load = [&](int j, f4a (&r1)[GM], f4a (&r2)[GM]) {
    load_from(R1 + (size_t)j * Pv, R2 + (size_t)j * Pv, r1, r2);
  };
  auto consume = [&](int j, const f4a (&r1)[GM], const f4a (&r2)[GM]) {
    // packed 2-wide FMA chains for the dots, packed FMAs for the contributions (as the forward pass)
    f2v d11 = {0.f, 0.f}, d21 = {0.f, 0.f}, d12 = {0.f, 0.f}, d22 = {0.f, 0.f};
#pragma unroll
    for (int m = 0; m < GM; ++m) {
      const int q = lane + kWave * m;
      const f4a a = ok[m] ? ldv(v1 + 4 * q) : f4a{0, 0, 0, 0};
      const f4a c = ok[m] ? ldv(v2 + 4 * q) : f4a{0, 0, 0, 0};
      d11 = pk_fma(r1[m].lo, a.lo, d11); d11 = pk_fma(r1[m].hi, a.hi, d11);
      d21 = pk_fma(r2[m].lo, a.lo, d21); d21 = pk_fma(r2[m].hi, a.hi, d21);
      d12 = pk_fma(r1[m].lo, c.lo, d12); d12 = pk_fma(r1[m].hi, c.hi, d12);
      d22 = pk_fma(r2[m].lo, c.lo, d22); d22 = pk_fma(r2[m].hi, c.hi, d22);
    }
    const float4 t = wave_sum4(d11.x + d11.y, d21.x + d21.y, d12.x + d12.y, d22.x + d22.y);
    float k1, k2, k3, k4;
    coef(j, t.x, t.y, t.z, t.w, k1, k2, k3, k4);
#pragma unroll
    for (int m = 0; m < GM; ++m) {
      pa[m] = pk_fma4(k2, r2[m], pk_fma4(k1, r1[m], pa[m]));
      pb[m] = pk_fma4(k4, r2[m], pk_fma4(k3, r1[m], pb[m]));
    }
  };
  // EF entries of this wave in flight (kAdjInflight)
  int j = j0 + wave;
  for (const int je = min(nl, j1); j < je; j += kAdjWaves) {  // LDS-held entries (wave-uniform)
    f4a r1[GM], r2[GM];
    load_from(LR + (size_t)2 * j * Pv, LR + (size_t)(2 * j + 1) * Pv, r1, r2);
    consume(j, r1, r2);
  }
  if (R1_j0 && j == j0 && j < j1) {  // entry j0's R1 row in LDS (wave 0's first entry)
    f4a r1[GM], r2[GM];
    load_from(R1_j0, R2 + (size_t)j * Pv, r1, r2);
    consume(j, r1, r2);
    j += kAdjWaves;
  }
  for (; j + (kAdjInflight - 1) * kAdjWaves < j1; j += kAdjInflight * kAdjWaves) {
    f4a r1[kAdjInflight][GM], r2[kAdjInflight][GM];
#pragma unroll
    for (int e = 0; e < kAdjInflight; ++e) load(j + e * kAdjWaves, r1[e], r2[e]);
#pragma unroll
    for (int e = 0; e < kAdjInflight; ++e) consume(j + e * kAdjWaves, r1[e], r2[e]);
  }
  for (; j < j1; j += kAdjWaves) {
    f4a r1[GM], r2[GM];
    load(j, r1, r2);
    consume(j, r1, r2);
  }
  auto put = [&](float* A, float* B) {
#pragma unroll
    for (int m = 0; m < GM; ++m)
      if (ok[m]) {
        const int q = lane + kWave * m;
        stv(A + 4 * q, pa[m]);
        stv(B + 4 * q, pb[m]);
      }
  };
  auto add = [&](const float* A, const float* B) {
#pragma unroll
    for (int m = 0; m < GM; ++m)
      if (ok[m]) {
        const int q = lane + kWave * m;
        pa[m] += ldv(A + 4 * q);
        pb[m] += ldv(B + 4 * q);
      }
  };
  if (wave == 2) put(sp0, sp1);
  if (wave == 3) put(sp2, sp3);
  __syncthreads();
  if (wave == 0) add(sp0, sp1);
  if (wave == 1) {
    add(sp2, sp3);
    put(sp2, sp3);
  }
  __syncthreads();
  if (wave == 0) {
    add(sp2, sp3);
#pragma unroll
    for (int m = 0; m < GM; ++m)
      if (ok[m]) {
        const int q = lane + kWave * m;
        pa[m] += base * ldv(v1 + 4 * q);
        pb[m] += base * ldv(v2 + 4 * q);
      }
    put(out1, out2);
  }
  __syncthreads();
}

// Global-vector mode (rows of up to GT float4 groups per thread, P <= GT * 1024): the same contraction
// as pair_pass, workgroup-wide.  Thread t owns float4 column groups t, t + 256, ...; v1, v2 and the two
// running sums stay in registers for the whole pass (one wave per SIMD: up to 512 registers), the rows
// of E entries are loaded per round, and one block reduction per round gives every thread the entries'
// dots in the same order.  R1_j0: entry j0's R1 row from this vector instead of R1 + j0 Pv.  out1 / out2
// may not alias v1 / v2 of another thread's columns (each thread reads and writes only its own).
template <int GT, int NW, class Coef>
__device__ __forceinline__ void wide_pair_pass(int P, int Pv, int j0, int j1, const float* __restrict__ R1,
                                               const float* __restrict__ R2, const float* v1, const float* v2,
                                               float base, Coef coef, float* out1, float* out2, float* scratch,
                                               int& buf, const float* R1_j0 = nullptr, float* stage = nullptr) {
  constexpr int BLOCK = kWave * NW;
  constexpr int E = GT * NW <= 32 ? 2 : 1;  // two entries per reduction while the rows fit the registers
  const int tid = threadIdx.x;
  const int G = (P + 3) / 4;
  const f4a z = f4a{0, 0, 0, 0};
  f4a a[GT], c[GT], pa[GT], pb[GT];
#pragma unroll
  for (int u = 0; u < GT; ++u) {
    const int q = tid + u * BLOCK;
    a[u] = c[u] = pa[u] = pb[u] = z;
    if (q < G) {
      a[u] = ldv(v1 + 4 * q);
      c[u] = ldv(v2 + 4 * q);
    }
  }
  // stage (the HVP's dual gradient vector in LDS, dead during the passes: 2 Pv floats, one entry): the
  // rows come HBM -> LDS by global_load_lds one entry ahead, each thread copying and reading back only
  // its own column groups, as the forward's GV history pass does (bfgs_solve.hip, wide_direction).
  // The same rows in the same order: bitwise the register path.
  bool staged = false;
  if constexpr (E == 1) {
    if (stage != nullptr && j1 > j0) {
      staged = true;
      typedef __attribute__((address_space(3))) float lds_float;
      const int wave = tid / kWave;
      const unsigned stage_off = __builtin_amdgcn_readfirstlane(
          (unsigned)(uintptr_t)((lds_float*)stage) + 16u * (unsigned)(wave * kWave));
      const unsigned r2_bytes = __builtin_amdgcn_readfirstlane(4u * (unsigned)Pv);
      const unsigned voff = 16u * (unsigned)tid;
      auto uniform_ptr64 = [](const float* p) {
        const unsigned long long v = (unsigned long long)(uintptr_t)p;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
        return ((unsigned long long)hi << 32) | lo;
      };
      auto copy = [&](int jj) {
        const float* r1p = (R1_j0 && jj == j0) ? R1_j0 : R1 + (size_t)jj * Pv;
        const float* r2p = R2 + (size_t)jj * Pv;
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          const int q = tid + u * BLOCK;
          const unsigned long long b1 = uniform_ptr64(r1p + 4 * u * BLOCK);
          const unsigned long long b2 = uniform_ptr64(r2p + 4 * u * BLOCK);
          const unsigned d1 = __builtin_amdgcn_readfirstlane(stage_off + 16u * (unsigned)(u * BLOCK));
          const unsigned d2 = __builtin_amdgcn_readfirstlane(d1 + r2_bytes);
          if (q < G) {
            unsigned saved;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(saved)
                : "v"(voff), "s"(b1), "s"(d1)
                : "memory");
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(saved)
                : "v"(voff), "s"(b2), "s"(d2)
                : "memory");
          }
        }
      };
      copy(j0);
      const float* st1 = stage + 4 * tid;
      const float* st2 = stage + Pv + 4 * tid;
      for (int j = j0; j < j1; ++j) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's copies of entry j have landed
        f4a r1[GT], r2[GT];
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          const int q = tid + u * BLOCK;
          r1[u] = r2[u] = z;
          if (q < G) {
            r1[u] = ldv(st1 + 4 * u * BLOCK);
            r2[u] = ldv(st2 + 4 * u * BLOCK);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read back before the next copy overwrites it
        if (j + 1 < j1) copy(j + 1);
        f2v d11 = {0.f, 0.f}, d21 = {0.f, 0.f}, d12 = {0.f, 0.f}, d22 = {0.f, 0.f};
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          d11 = pk_fma(r1[u].lo, a[u].lo, d11); d11 = pk_fma(r1[u].hi, a[u].hi, d11);
          d21 = pk_fma(r2[u].lo, a[u].lo, d21); d21 = pk_fma(r2[u].hi, a[u].hi, d21);
          d12 = pk_fma(r1[u].lo, c[u].lo, d12); d12 = pk_fma(r1[u].hi, c[u].hi, d12);
          d22 = pk_fma(r2[u].lo, c[u].lo, d22); d22 = pk_fma(r2[u].hi, c[u].hi, d22);
        }
        float d[4] = {d11.x + d11.y, d21.x + d21.y, d12.x + d12.y, d22.x + d22.y};
        block_sum<4, NW, true>(d, scratch, buf);
        buf ^= 1;
        float k1, k2, k3, k4;
        coef(j, d[0], d[1], d[2], d[3], k1, k2, k3, k4);
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          pa[u] = pk_fma4(k2, r2[u], pk_fma4(k1, r1[u], pa[u]));
          pb[u] = pk_fma4(k4, r2[u], pk_fma4(k3, r1[u], pb[u]));
        }
      }
    }
  }
  for (int j = j0; j < (staged ? j0 : j1); j += E) {  // (the register path)
    const int ne = min(E, j1 - j);  // uniform
    f4a r1[E][GT], r2[E][GT];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float* r1p = (R1_j0 && j + e == j0) ? R1_j0 : R1 + (size_t)(j + e) * Pv;
      const float* r2p = R2 + (size_t)(j + e) * Pv;
#pragma unroll
      for (int u = 0; u < GT; ++u) {
        const int q = tid + u * BLOCK;
        // (every group exec-masked: the launch rounds GT up to an instantiated width, so unlike the
        // forward's pass groups below GT - 1 may lie past the row)
        r1[e][u] = r2[e][u] = z;
        if (e < ne && q < G) {
          r1[e][u] = ldv(r1p + 4 * q);
          r2[e][u] = ldv(r2p + 4 * q);
        }
      }
    }
    // the four dots as packed 2-wide FMA chains (v_pk_fma_f32) and the contributions as packed FMAs,
    // as the forward's history pass (wide_direction) forms them: 40% fewer VALU ops per entry than
    // per-element products and horizontal adds
    float d[4 * E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      f2v d11 = {0.f, 0.f}, d21 = {0.f, 0.f}, d12 = {0.f, 0.f}, d22 = {0.f, 0.f};
#pragma unroll
      for (int u = 0; u < GT; ++u) {
        d11 = pk_fma(r1[e][u].lo, a[u].lo, d11); d11 = pk_fma(r1[e][u].hi, a[u].hi, d11);
        d21 = pk_fma(r2[e][u].lo, a[u].lo, d21); d21 = pk_fma(r2[e][u].hi, a[u].hi, d21);
        d12 = pk_fma(r1[e][u].lo, c[u].lo, d12); d12 = pk_fma(r1[e][u].hi, c[u].hi, d12);
        d22 = pk_fma(r2[e][u].lo, c[u].lo, d22); d22 = pk_fma(r2[e][u].hi, c[u].hi, d22);
      }
      d[4 * e] = d11.x + d11.y;
      d[4 * e + 1] = d21.x + d21.y;
      d[4 * e + 2] = d12.x + d12.y;
      d[4 * e + 3] = d22.x + d22.y;
    }
    block_sum<4 * E, NW>(d, scratch, buf);
    buf ^= 1;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (e < ne) {
        float k1, k2, k3, k4;
        coef(j + e, d[4 * e], d[4 * e + 1], d[4 * e + 2], d[4 * e + 3], k1, k2, k3, k4);
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          pa[u] = pk_fma4(k2, r2[e][u], pk_fma4(k1, r1[e][u], pa[u]));
          pb[u] = pk_fma4(k4, r2[e][u], pk_fma4(k3, r1[e][u], pb[u]));
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < GT; ++u) {
    const int q = tid + u * BLOCK;
    if (q < G) {
      stv(out1 + 4 * q, pa[u] + base * a[u]);
      stv(out2 + 4 * q, pb[u] + base * c[u]);
    }
  }
  __syncthreads();
}

// LDS mode: two workgroups per CU (registers <= 256 VGPRs, LDS <= 80 KB each), so one problem's
// dual-number evaluation overlaps the other's row passes: C3 solve + gradient 51.7k -> 63.0k problems/s
// (r03, profiles/r03_ab_adjoint_two_wg_per_cu.log; in r02 the same register cap spilled 100-165
// registers and one workgroup per CU was faster, since then the passes' register use went down).
// GT > 0: global-vector mode (the O(P) vectors in the workspace slice a.gvws, wide_pair_pass with up
// to GT float4 groups per thread); GT = 0: everything O(P) in LDS (pair_pass, GM groups per lane).
constexpr int kAdjLdsWpe = 2;
// SCG (LDS mode): the tape's scalar row (alpha_k, rho_j, c_j, gamma: about 4 K floats) read in place
// instead of staged in LDS.  The row is sized by the iteration cap, not by the steps taken: at C3 with
// the reference's default cap (1000) it pushed the image past the 80 KB that two workgroups per CU
// need (profiles/r05_ab_adjoint_scalars.log).  A kernel of its own, as the forward's SLICE.
template <int RES, int GM, int GT = 0, int NW = kAdjWaves, bool SCG = false>
__global__ __launch_bounds__(kWave * NW, GT > 0 ? 1 : kAdjLdsWpe) void bfgs_ba_adjoint_kernel(AdjointArgs a) {
  static_assert(GT > 0 || NW == kAdjWaves, "LDS mode (pair_pass) runs four waves");
  static_assert(!SCG || GT == 0, "SCG is an LDS-mode variant");
  constexpr int BLOCK = kWave * NW;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr bool GVM = GT > 0;
  const Layout L = a.L;
  const int P = L.P, M = L.M, N = L.N, MN = M * N, Pv = a.Pv, K = a.K;
  const int b = blockIdx.x, tid = threadIdx.x;
  const TapeLayout& tl = a.tl;
  const AdjointCarve cv = carve_adjoint(M, N, Pv, SCG ? 0 : tl.T, a.lcap, GVM, NW, GVM && a.gd_lds);
  float* vb = GVM ? a.gvws + (size_t)b * cv.gv_floats : lds;  // base of the O(P) vectors
  float* xb = vb + cv.xb;    // xbar: adjoint of x_{k+1} entering step k, of x_k leaving it
  float* sbp = vb + cv.sbp;  // adjoint of s_k from the update that used it (step k + 1)
  float* gbp = vb + cv.gbp;  // adjoint of g_k from y_{k+1} = g_{k+1} - g_k
  float* db = vb + cv.db;
  float* gk = vb + cv.gk;
  float* p1 = vb + cv.p1;
  float* p2 = vb + cv.p2;
  float* wb = vb + cv.wb;
  // H_{k-1} dbar, H_{k-1} wbar: p1 is dead once wbar / sbar are formed, gk until the final loop
  // (which reads hw[i] before it writes gk[i], in the same thread)
  float* hd = p1;
  float* hw = vb + cv.gk;
  float* sv = vb + cv.sv;
  float* wv = vb + cv.wv;
  float* yv = vb + cv.yv;
  float* gv = vb + cv.gv;
  // the passes' cross-wave spares live in the dual vectors' space (dead until the HVP)
  float* sp0 = vb + cv.xd;
  float* sp1 = sp0 + Pv;
  float* sp2 = vb + cv.gd;
  float* sp3 = sp2 + Pv;
  // a_k lives in LDS while step k updates it (ak) and -wbar_k waits there for step k - 1 (an); the
  // workspace row a_k is written once, final, and only read by later steps (never read-modify-write)
  float* akl = vb + cv.ak;
  float* anl = vb + cv.an;
  const float* sc = SCG ? a.tape + tl.scal + (size_t)b * tl.T : lds + cv.sc;
  Dual* xd = reinterpret_cast<Dual*>(vb + cv.xd);
  Dual* gd = reinterpret_cast<Dual*>((GVM && a.gd_lds ? lds : vb) + cv.gd);
  // GV passes: the rows staged through the dual gradient vector's LDS slots (dead until the HVP)
  // (C5 adjoint 85.8 -> 79.7 ms, interleaved, profiles/r04_ab_adjoint_staged_c5.log)
  float* stage = GVM && a.gd_lds ? lds + cv.gd : nullptr;
  Dual* views = reinterpret_cast<Dual*>(lds + cv.views);
  Dual* vpart = reinterpret_cast<Dual*>(lds + cv.vpart);
  const float* obs = GVM ? a.obs + (size_t)b * 2 * MN : lds + cv.obs;
  // GV: the observation cotangent is accumulated in place in the output (or not at all)
  float* obsacc = GVM ? (a.obs_grad ? a.obs_grad + (size_t)b * 2 * MN : nullptr) : lds + cv.obsacc;
  float* scratch = lds + cv.scratch;
  const uint8_t* vis = GVM ? a.vis + (size_t)b * MN : reinterpret_cast<uint8_t*>(lds) + cv.vis_bytes_off;

  const float* S = a.tape + tl.hist + (size_t)b * 2 * tl.kcap * Pv;  // history rows s_j
  const float* W = S + (size_t)tl.kcap * Pv;                          // w_j
  const float* X = a.tape + tl.x + (size_t)b * K * Pv;
  const float* Gr = a.tape + tl.g + (size_t)b * K * Pv;
  float* Ar = a.arows + (size_t)b * K * Pv;

  for (int i = tid; i < Pv; i += BLOCK) {
    xb[i] = i < P ? a.xbar[(size_t)b * P + i] : 0.f;
    sbp[i] = gbp[i] = anl[i] = 0.f;
  }
  if constexpr (!SCG)
    for (int i = tid; i < tl.T; i += BLOCK) lds[cv.sc + i] = a.tape[tl.scal + (size_t)b * tl.T + i];
  if constexpr (GVM) {
    if (obsacc)
      for (int i = tid; i < 2 * MN; i += BLOCK) obsacc[i] = 0.f;
  } else {
    float* ol = lds + cv.obs;
    uint8_t* vl = reinterpret_cast<uint8_t*>(lds) + cv.vis_bytes_off;
    for (int i = tid; i < 2 * MN; i += BLOCK) {
      ol[i] = a.obs[(size_t)b * 2 * MN + i];
      obsacc[i] = 0.f;
    }
    for (int i = tid; i < MN; i += BLOCK) vl[i] = a.vis[(size_t)b * MN + i] ? 1 : 0;
  }
  const int n = min(a.status[(size_t)b * DAVA_STATUS_WORDS], K);
  float* lh = lds + cv.lh;
  const int nlh = GVM ? 0 : min(a.lcap, max(n - 1, 0));  // history entries 0 .. n-2 exist
  for (int q = tid; q < nlh * (Pv / 4); q += BLOCK) {
    const int j = q / (Pv / 4), i = 4 * (q % (Pv / 4));
    stv(lh + (size_t)2 * j * Pv + i, ldv(S + (size_t)j * Pv + i));
    stv(lh + (size_t)(2 * j + 1) * Pv + i, ldv(W + (size_t)j * Pv + i));
  }
  float trace = 0.f;  // sum_{j > k} a_j . g_j with every a_j final (needed at k = 1: gamma's adjoint)
  int buf = 0;
  __syncthreads();
  // (read after the barrier: sc[3 K] is staged by another thread.  Before it, a thread could read
  // the slot ahead of its writer -- the LDS image's staging loops usually hid that; in global-vector
  // mode nothing stands between the two)
  const float gamma = sc[3 * K];

  // The per-step vector work goes float4-wide: thread t owns column groups t, t + BLOCK, ... (the row
  // passes' ownership), so each element is touched by the same thread in every loop of a step.
  auto each4 = [&](auto f) {
    for (int q = tid; q < Pv / 4; q += BLOCK) f(4 * q);
  };
  auto below_p = [P](int i, f4a v) {  // elements >= P read as 0 (the scalar loops' i < P ? v : 0)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (i + e >= P) v[e] = 0.f;
    return v;
  };
  for (int k = n - 1; k >= 0; --k) {
    const float alpha = sc[k];
    // ---- s_k = alpha d_k, x_{k+1} = x_k + s_k (alpha is a constant of the line search) ----
    each4([&](int i) { stv(db + i, alpha * (ldv(xb + i) + ldv(sbp + i))); });
    if (k == 0) {
      each4([&](int i) { stv(gk + i, ldv(gbp + i) - ldv(db + i)); });  // d_0 = -g_0
    } else {
      const float* gk1 = Gr + (size_t)(k - 1) * Pv;
      const float* gkr = Gr + (size_t)k * Pv;
      const float* srow = S + (size_t)(k - 1) * Pv;
      const float* wrow = W + (size_t)(k - 1) * Pv;
      float* ak = Ar + (size_t)k * Pv;
      each4([&](int i) {
        const f4a g1 = below_p(i, ldv(gkr + i)), g0 = below_p(i, ldv(gk1 + i));
        stv(gv + i, g1);
        stv(yv + i, g1 - g0);
        stv(sv + i, ldv(srow + i));
        stv(wv + i, ldv(wrow + i));
        stv(akl + i, ldv(anl + i) - ldv(db + i));  // d_k = -H_k g_k adds -dbar_k g_k^T to H_k's adjoint
      });
      __syncthreads();
      const float rho = sc[K + k - 1], c = sc[2 * K + k - 1];
      // P1 = (A + A^T) s, P2 = (A + A^T) w over rows (a_j, g_j), j = k .. n-1
      const auto acoef = [](int, float as, float gs, float aw, float gw, float& k1, float& k2, float& k3,
                            float& k4) {
        k1 = gs; k2 = as; k3 = gw; k4 = aw;
      };
      if constexpr (GVM) {
        wide_pair_pass<GT, NW>(P, Pv, k, n, Ar, Gr, sv, wv, 0.f, acoef, p1, p2, scratch, buf, akl, stage);
      } else {
        pair_pass<GM>(P, Pv, k, n, Ar, Gr, sv, wv, 0.f, acoef, p1, p2, sp0, sp1, sp2, sp3, akl);
      }
      float r[7] = {0, 0, 0, 0, 0, 0, 0};
      each4([&](int i) {
        const f4a s4 = ldv(sv + i), w4 = ldv(wv + i), y4 = ldv(yv + i), d4 = ldv(db + i), q1 = ldv(p1 + i),
                  q2 = ldv(p2 + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (i + e < P) {
            const float si = s4[e], wi = w4[e], yi = y4[e], di = d4[e];
            r[0] += si * q1[e]; r[1] += si * q2[e]; r[2] += yi * wi; r[3] += si * di; r[4] += wi * di;
            r[5] += yi * yi; r[6] += si * yi;
          }
        }
      });
      block_sum<7, NW>(r, scratch, buf);
      buf ^= 1;
      const float sAs = 0.5f * r[0], sAw = r[1], yw = r[2], sd = r[3], wd = r[4], yy = r[5], t = r[6];
      const float cbar = rho * sAs;
      const float rhobar = c * sAs - sAw + cbar * yw;
      const float tbar = rho > 0.f ? -(rho * rho) * rhobar : 0.f;  // inverse_curvature backward
      each4([&](int i) {
        const f4a q1 = ldv(p1 + i), q2 = ldv(p2 + i), y4 = ldv(yv + i), w4 = ldv(wv + i), s4 = ldv(sv + i);
        stv(wb + i, -rho * q1 + (cbar * rho) * y4);
        stv(p2 + i, (cbar * rho) * w4 + tbar * s4);  // ybar, direct terms
        stv(sbp + i, (c * rho) * q1 - rho * q2 + tbar * y4);
      });
      __syncthreads();
      // H_{k-1} dbar and H_{k-1} wbar: one pass over history entries 0 .. k-2, plus gamma I
      if (k >= 2) {
        const float* hrho = sc + K;
        const float* hc = sc + 2 * K;
        const auto hcoef = [hrho, hc](int j, float sdv, float wdv, float swv, float wwv, float& k1, float& k2,
                                      float& k3, float& k4) {
          const float rj = hrho[j], cr = hc[j] * rj;
          k1 = cr * sdv - rj * wdv; k2 = -rj * sdv;
          k3 = cr * swv - rj * wwv; k4 = -rj * swv;
        };
        if constexpr (GVM) wide_pair_pass<GT, NW>(P, Pv, 0, k - 1, S, W, db, wb, gamma, hcoef, hd, hw, scratch, buf, nullptr, stage);
        else pair_pass<GM>(P, Pv, 0, k - 1, S, W, db, wb, gamma, hcoef, hd, hw, sp0, sp1, sp2, sp3, nullptr, lh, nlh);
      } else {
        each4([&](int i) {
          stv(hd + i, gamma * ldv(db + i));
          stv(hw + i, gamma * ldv(wb + i));
        });
      }
      // H_k dbar = H_{k-1} dbar + entry k-1's rank-2 term;  gbar_k, a_k, a_{k-1}
      const float e1 = c * rho * sd - rho * wd, e2 = -rho * sd;
      float tr[1] = {0.f};
      const float* g0r = k == 1 ? Gr : nullptr;
      each4([&](int i) {
        const f4a ybar = ldv(p2 + i) + ldv(hw + i);  // (hw aliases gk: read before gk is written)
        const f4a hk = ldv(hd + i) + e1 * ldv(sv + i) + e2 * ldv(wv + i);
        const f4a w4 = ldv(wb + i), g4 = ldv(gv + i);
        stv(gk + i, ldv(gbp + i) - hk + ybar);
        stv(gbp + i, -ybar);
        const f4a af = ldv(akl + i) + w4;
        stv(ak + i, af);  // final a_k (read by the passes of steps < k)
        stv(anl + i, -w4);
        const f4a g0 = k == 1 ? ldv(g0r + i) : f4a{0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          tr[0] += af[e] * g4[e];
          if (k == 1 && i + e < P) tr[0] -= w4[e] * g0[e];  // a_0 = -wbar_1
        }
      });
      block_sum<1, NW>(tr, scratch, buf);
      buf ^= 1;
      trace += tr[0];
      if (k == 1) {
        // gamma = clamp(q, min 1e-4), q = t / clamp(yy, min 1e-5); its adjoint is tr(H_0' adjoint)
        const float yyc = clamp_min(yy, 1e-5f);
        const float q = t / yyc;
        const float qbar = q >= 1e-4f ? trace : 0.f;  // clamp backward passes where input >= min
        const float tg = qbar / yyc;
        const float yybar = yy >= 1e-5f ? -qbar * q / yyc : 0.f;
        each4([&](int i) {
          const f4a y4 = ldv(yv + i);
          const f4a extra = tg * ldv(sv + i) + 2.0f * yybar * y4;
          stv(sbp + i, ldv(sbp + i) + tg * y4);
          stv(gk + i, ldv(gk + i) + extra);
          stv(gbp + i, ldv(gbp + i) - extra);
        });
      }
    }
    // ---- g_k = dE/dx(x_k): xbar += Hess E gbar_k, obsbar += (d2E/dobs dx) gbar_k ----
    // (the loops above own float4 groups, this one elements: gk's last writes -- the k = 0 line, the
    // k = 1 gamma terms -- must land before another thread reads them)
    __syncthreads();
    const float* xk = X + (size_t)k * Pv;
    for (int i = tid; i < Pv; i += BLOCK) {
      xd[i] = Dual(i < P ? xk[i] : 0.f, i < P ? gk[i] : 0.f);
      gd[i] = Dual(0.f);
    }
    __syncthreads();
    Dual E(0.f), unused(0.f);
    ba_eval<true, false, false, false, false, RES, Dual, NW>(L, xd, nullptr, 0.f, obs, vis, gd, views, vpart,
                                                                   scratch, buf, E, unused, nullptr, obsacc);
    for (int i = tid; i < P; i += BLOCK) xb[i] += gd[i].t;
    __syncthreads();
  }
  for (int i = tid; i < P; i += BLOCK) a.x0_grad[(size_t)b * P + i] = xb[i];
  if (a.obs_grad && !GVM)
    for (int i = tid; i < 2 * MN; i += BLOCK) a.obs_grad[(size_t)b * 2 * MN + i] = obsacc[i];
}

// Global-vector mode: waves per workgroup (one workgroup per CU).  Eight: the row passes hold up to 7
// float4 groups per thread and two waves per SIMD hide their latency; the dual-number evaluation then
// runs at the 256-VGPR budget.  Four: up to 14 groups per thread, one wave per SIMD with 512 registers.
// Eight unless the eight-wave LDS image (per-wave view partials and reduction scratch grow with the
// waves) does not fit -- many views -- or the kDbgAdjGVWaves override asks for four.
static int adjoint_gv_waves(const DavaScene* s, const TapeLayout& tl) {
  if (debug_knob(kDbgAdjGVWaves) == 4) return 4;
  return carve_adjoint(s->num_views, s->num_points, tl.Pv, tl.T, 0, true, 8).total_bytes <= kAdjLdsBytes ? 8 : 4;
}

template <int RES>
static void launch_adjoint(const AdjointArgs& a, int B, int lds, int gm, int gt, int nw, hipStream_t s) {
  if (gt == 0 && a.sc_global) {  // LDS mode, the tape's scalar row in place
    auto go = [&](auto kernel) {
      if (lds > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      hipLaunchKernelGGL(kernel, dim3(B), dim3(kAdjBlock), lds, s, a);
    };
    if (gm <= 1) go(bfgs_ba_adjoint_kernel<RES, 1, 0, kAdjWaves, true>);
    else if (gm == 2) go(bfgs_ba_adjoint_kernel<RES, 2, 0, kAdjWaves, true>);
    else if (gm == 3) go(bfgs_ba_adjoint_kernel<RES, 3, 0, kAdjWaves, true>);
    else go(bfgs_ba_adjoint_kernel<RES, 4, 0, kAdjWaves, true>);
    return;
  }
  auto go = [&](auto kernel, int threads) {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(kernel, dim3(B), dim3(threads), lds, s, a);
  };
  if (gt > 0 && nw == 8) {  // global-vector mode, eight waves: 4 or 7 float4 groups per thread
    if (gt <= 4) go(bfgs_ba_adjoint_kernel<RES, 1, 4, 8>, 8 * kWave);
    else go(bfgs_ba_adjoint_kernel<RES, 1, 7, 8>, 8 * kWave);
  } else if (gt > 0) {  // global-vector mode, four waves: 4, 8 or 14 float4 groups per thread
    if (gt <= 4) go(bfgs_ba_adjoint_kernel<RES, 1, 4>, kAdjBlock);
    else if (gt <= 8) go(bfgs_ba_adjoint_kernel<RES, 1, 8>, kAdjBlock);
    else go(bfgs_ba_adjoint_kernel<RES, 1, kAdjMaxGroups>, kAdjBlock);
  } else if (gm <= 1) go(bfgs_ba_adjoint_kernel<RES, 1>, kAdjBlock);
  else if (gm == 2) go(bfgs_ba_adjoint_kernel<RES, 2>, kAdjBlock);
  else if (gm == 3) go(bfgs_ba_adjoint_kernel<RES, 3>, kAdjBlock);
  else go(bfgs_ba_adjoint_kernel<RES, 4>, kAdjBlock);
}

// Global-vector mode when the LDS image does not fit one CU (or P > 1024, past pair_pass's 4 groups
// per lane); the kDbgAdjForceGV override forces it (tests: the same tape through both kernels).
static bool adjoint_gv(const DavaScene* s, const TapeLayout& tl) {
  if (debug_flag(kDbgAdjForceGV)) return true;
  return s->num_parameters > 1024 || carve_adjoint(s->num_views, s->num_points, tl.Pv, tl.T).total_bytes > kAdjLdsBytes;
}
static int adjoint_groups(const TapeLayout& tl) { return (tl.Pv / 4 + kAdjBlock - 1) / kAdjBlock; }

static int adjoint_check(const DavaScene* s, const DavaSolverConfig* c) {
  if (!s || !c) return DAVA_ERR_INVALID_ARGUMENT;
  if (s->batch < 0 || s->num_views < 2 || s->num_points < 1) return DAVA_ERR_INVALID_ARGUMENT;
  const int P = 3 + 3 * s->num_points + 6 * (s->num_views - 1) + (s->distortion ? 5 : 0);
  if (s->num_parameters != P) return DAVA_ERR_INVALID_ARGUMENT;
  if (s->residual != DAVA_RESIDUAL_SQUARED_REPROJECTION && s->residual != DAVA_RESIDUAL_RAY_ANGLE)
    return DAVA_ERR_INVALID_ARGUMENT;
  if (s->residual == DAVA_RESIDUAL_RAY_ANGLE && s->distortion) return DAVA_ERR_UNSUPPORTED;
  if (c->hessian_mode != DAVA_HESSIAN_COMPACT || c->iterations < 1 || c->iterations > 1025) return DAVA_ERR_UNSUPPORTED;
  const TapeLayout tl = tape_layout(s->batch, P, c->iterations);
  if (adjoint_gv(s, tl)) {
    if (adjoint_groups(tl) > kAdjMaxGroups) return DAVA_ERR_UNSUPPORTED;
    // the image of the launch that will run: adjoint_gv_waves() falls back to four waves where eight do not fit
    if (carve_adjoint(s->num_views, s->num_points, tl.Pv, tl.T, 0, true, adjoint_gv_waves(s, tl)).total_bytes >
        kAdjLdsBytes)
      return DAVA_ERR_UNSUPPORTED;
  }
  return DAVA_OK;
}

// LDS mode: the tape's scalar row stays in place (SCG) when staging it would push the image past the two
// workgroups per CU that the rest of it allows
static bool adjoint_sc_global(const DavaScene* s, const TapeLayout& tl) {
  if (adjoint_gv(s, tl)) return false;
  if (debug_knob(kDbgAdjScGlobal) >= 0) return debug_knob(kDbgAdjScGlobal) > 0;  // tests
  const int M = s->num_views, N = s->num_points;
  return carve_adjoint(M, N, tl.Pv, tl.T).total_bytes > kAdjLdsBytes / kAdjLdsWpe &&
         carve_adjoint(M, N, tl.Pv, 0).total_bytes <= kAdjLdsBytes / kAdjLdsWpe;
}

// As many history entries on chip as the CU's LDS leaves room for (one workgroup per CU), at most
// the K - 1 a solve can make; the kDbgAdjLdsEntries override caps it (0: none) for A/B runs.  None in GV mode.
static int adjoint_lds_entries(const DavaScene* s, const TapeLayout& tl) {
  if (adjoint_gv(s, tl)) return 0;
  const int base = carve_adjoint(s->num_views, s->num_points, tl.Pv, adjoint_sc_global(s, tl) ? 0 : tl.T).total_bytes;
  int n = (kAdjLdsBytes / kAdjLdsWpe - base) / (int)(2 * tl.Pv * sizeof(float));
  n = max(0, min(n, tl.K - 1));
  if (debug_knob(kDbgAdjLdsEntries) >= 0) n = max(0, min(n, (int)debug_knob(kDbgAdjLdsEntries)));
  return n;
}

// workspace: the a rows (B, K, Pv), then in GV mode the per-problem vector slices
static size_t adjoint_rows_bytes(const DavaScene* s, const TapeLayout& tl) {
  return (size_t)s->batch * tl.K * tl.Pv * sizeof(float);
}
static size_t adjoint_gv_bytes(const DavaScene* s, const TapeLayout& tl) {
  if (!adjoint_gv(s, tl)) return 0;
  return (size_t)s->batch * carve_adjoint(s->num_views, s->num_points, tl.Pv, tl.T, 0, true).gv_floats * sizeof(float);
}

}  // namespace dava

using namespace dava;

extern "C" size_t dava_ba_solve_backward_workspace_bytes(const DavaScene* scene, const DavaSolverConfig* config) {
  if (adjoint_check(scene, config) != DAVA_OK) return 0;
  const TapeLayout tl = tape_layout(scene->batch, scene->num_parameters, config->iterations);
  return adjoint_rows_bytes(scene, tl) + adjoint_gv_bytes(scene, tl) + 256;
}

extern "C" int dava_ba_solve_backward_lds_entries(const DavaScene* scene, const DavaSolverConfig* config) {
  if (adjoint_check(scene, config) != DAVA_OK) return 0;
  return adjoint_lds_entries(scene, tape_layout(scene->batch, scene->num_parameters, config->iterations));
}

extern "C" int dava_ba_solve_backward(const DavaScene* scene, const DavaSolverConfig* config, const void* tape,
                                      size_t tape_bytes, const int32_t* status, const float* x_out_grad,
                                      float* x0_grad, float* observations_grad, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  const int st = adjoint_check(scene, config);
  if (st != DAVA_OK) return st;
  if (scene->batch == 0) return DAVA_OK;
  if (!scene->observations || !scene->visibility || !tape || !status || !x_out_grad || !x0_grad)
    return DAVA_ERR_INVALID_ARGUMENT;
  const TapeLayout tl = tape_layout(scene->batch, scene->num_parameters, config->iterations);
  if (tape_bytes < tl.queue_byte) return DAVA_ERR_WORKSPACE;
  const size_t rows = adjoint_rows_bytes(scene, tl), gvb = adjoint_gv_bytes(scene, tl);
  if (!workspace || workspace_bytes < rows + gvb) return DAVA_ERR_WORKSPACE;
  const bool gv = adjoint_gv(scene, tl);
  AdjointArgs a;
  a.L = Layout{scene->num_views, scene->num_points, scene->num_parameters, scene->distortion ? 1 : 0};
  a.Pv = tl.Pv;
  a.K = tl.K;
  a.tl = tl;
  a.tape = static_cast<const float*>(tape);
  a.obs = scene->observations;
  a.vis = scene->visibility;
  a.status = status;
  a.xbar = x_out_grad;
  a.x0_grad = x0_grad;
  a.obs_grad = observations_grad;
  a.arows = static_cast<float*>(workspace);
  a.gvws = gv ? reinterpret_cast<float*>(static_cast<char*>(workspace) + rows) : nullptr;
  a.lcap = adjoint_lds_entries(scene, tl);
  a.sc_global = adjoint_sc_global(scene, tl) ? 1 : 0;
  const int nw = gv ? adjoint_gv_waves(scene, tl) : kAdjWaves;
  a.gd_lds = gv && !debug_flag(kDbgAdjGdHbm) &&
             carve_adjoint(scene->num_views, scene->num_points, tl.Pv, tl.T, a.lcap, gv, nw, true).total_bytes <=
                 kAdjLdsBytes;
  const int lds = carve_adjoint(scene->num_views, scene->num_points, tl.Pv, a.sc_global ? 0 : tl.T, a.lcap, gv, nw,
                                a.gd_lds).total_bytes;
  const int gm = (tl.Pv / 4 + kWave - 1) / kWave;
  const int gt = gv ? (tl.Pv / 4 + kWave * nw - 1) / (kWave * nw) : 0;  // float4 groups per thread
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (scene->residual == DAVA_RESIDUAL_RAY_ANGLE) launch_adjoint<DAVA_RESIDUAL_RAY_ANGLE>(a, scene->batch, lds, gm, gt, nw, s);
  else launch_adjoint<DAVA_RESIDUAL_SQUARED_REPROJECTION>(a, scene->batch, lds, gm, gt, nw, s);
  return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH;
}
