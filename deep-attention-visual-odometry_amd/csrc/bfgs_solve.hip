// Fused eval-mode BFGS + strong-Wolfe bundle-adjustment solve on gfx950.
//
// Replaces, for the squared reprojection objective:
//   BFGSSolver.forward                      autograd_solvers/bfgs_solver.py:80-215
//   BFGSSolver.scale_initial_inverse_hessian bfgs_solver.py:217-233
//   BFGSSolver.update_inverse_hessian        bfgs_solver.py:235-303
//   line_search_wolfe_conditions(strong=True) autograd_solvers/line_search/wolfe_conditions.py:23-239
//
// Design (DESIGN.md has the numbers):
//  * one problem per 256-thread workgroup for the WHOLE solve: every host sync
//    of the reference (bfgs_solver.py:144,206, wolfe_conditions.py:120) and
//    every boolean-mask gather/scatter disappears; problems that stop early
//    just retire their workgroup.
//  * all O(P) state (x, g, g_prev, d, s, H y, H g, pending update) and the
//    scene (obs, vis) live in LDS; the only HBM stream is the inverse Hessian.
//  * DENSE mode keeps the reference's dense P x P fp32 inverse Hessian per
//    problem in HBM, with the rank-2 update DEFERRED: iteration k reads
//    H_{k-2}, applies U_{k-1} on the fly, writes H_{k-1} back and in the same
//    sweep forms H_{k-1} y and H_{k-1} g (column sums: lane = column, so no
//    cross-lane reduction).  H_k g then follows algebraically from the rank-2
//    terms, so each BFGS iteration costs exactly one read + one write of H
//    (8 P^2 bytes), the minimum for a materialised dense H.  H_0 = gamma I is
//    never stored (the first sweep synthesises it).
//  * the line search runs in-kernel; trial slopes come from forward-mode
//    (JVP) derivatives, gradients at accepted points from reverse mode.
#include "ba_objective.hpp"

namespace dava {

struct SolveArgs {
  Layout L;
  int B, Pv, Pld;
  const float* obs;
  const uint8_t* vis;
  const float* x0;
  float* x_out;
  float* err_out;
  int32_t* status;
  float* hess;
  float c1, c2, thr, min_step;
  int iters, max_trials, strong, mode;
};

struct LdsCarve {
  int x, d, g0, g1, s0, s1, hy0, hy1, hg, obs, views, vpart, scratch, vis_bytes_off, total_bytes;
};

__host__ __device__ inline LdsCarve carve_lds(int M, int N, int Pv) {
  LdsCarve c;
  int off = 0;
  c.x = off; off += Pv;
  c.d = off; off += Pv;
  c.g0 = off; off += Pv;
  c.g1 = off; off += Pv;
  c.s0 = off; off += Pv;
  c.s1 = off; off += Pv;
  c.hy0 = off; off += Pv;
  c.hy1 = off; off += Pv;
  c.hg = off; off += Pv;
  c.obs = off; off += round_up(2 * M * N, 4);
  c.views = off; off += round_up(views_floats(M), 4);
  c.vpart = off; off += round_up(vpart_floats(M), 4);
  c.scratch = off; off += 2 * kWaves * 32;
  c.vis_bytes_off = off * 4;
  c.total_bytes = c.vis_bytes_off + round_up(M * N, 16);
  return c;
}

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

#ifndef DAVA_SWEEP_ROWS
#define DAVA_SWEEP_ROWS 4
#endif
#ifndef DAVA_SWEEP_NT
#define DAVA_SWEEP_NT 0
#endif
#ifndef DAVA_DIAG_NO_HBM
#define DAVA_DIAG_NO_HBM 0
#endif

// Streaming access to the inverse Hessian: every element is read once and
// written once per BFGS iteration, never reused by another workgroup.
__device__ __forceinline__ f4v h_load(const float* p) {
#if DAVA_SWEEP_NT
  return __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
#else
  return *reinterpret_cast<const f4v*>(p);
#endif
}
__device__ __forceinline__ void h_store(float* p, f4v v) {
#if DAVA_SWEEP_NT
  __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
#else
  *reinterpret_cast<f4v*>(p) = v;
#endif
}

// Apply the pending rank-2 term to one element (bfgs_solver.py:298-303 order:
// ((H + (s_rho_i s_j) c) - s_rho_i yH_j) - Hy_i s_rho_j, no FMA contraction).
__device__ __forceinline__ float rank2(float h, float sri, float sj, float c, float hyj, float hyi, float srj) {
  float t = __fadd_rn(h, __fmul_rn(__fmul_rn(sri, sj), c));
  t = __fsub_rn(t, __fmul_rn(sri, hyj));
  return __fsub_rn(t, __fmul_rn(hyi, srj));
}

// One sweep over the dense inverse Hessian of this problem.
//   H' = Hs + pending,  Hs = stored matrix (or gamma0*I if not materialised)
//   hy_out[j] = sum_i H'_ij y_i,  hg_out[j] = sum_i H'_ij g_i   (y = g - gp)
// Writes H' back.  Column ownership: the ceil(P/4) float4 column groups are
// split evenly over the 4 waves (wave w owns groups [w*Gw, (w+1)*Gw)), one
// group per lane per 64-group block, so every wave streams and every global
// access is a contiguous row piece of up to 1 KiB.  Lane = column means the
// column sums need no cross-lane reduction.  U rows are loaded before any is
// consumed to keep U KiB per wave in flight.
__device__ void dense_sweep(const Layout& L, int Pld, float* __restrict__ H, bool materialized, float gamma0,
                            const float* ps, const float* phy, float prho, float pc, const float* g,
                            const float* gp, float* hy_out, float* hg_out) {
  constexpr int U = DAVA_SWEEP_ROWS;
  const int P = L.P;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int G = (P + 3) / 4;                      // float4 column groups
  const int Gw = (G + kWaves - 1) / kWaves;       // groups per wave
  const int g_end = min(G, (wave + 1) * Gw);
  for (int gb = wave * Gw; gb < g_end; gb += kWave) {
    const int grp = gb + lane;
    const bool act = grp < g_end;
    const int j0 = grp * 4;
    float sj[4] = {0, 0, 0, 0}, hj[4] = {0, 0, 0, 0}, srj[4] = {0, 0, 0, 0};
    if (act) {
      const float4 a = ld4(ps + j0), b = ld4(phy + j0);
      sj[0] = a.x; sj[1] = a.y; sj[2] = a.z; sj[3] = a.w;
      hj[0] = b.x; hj[1] = b.y; hj[2] = b.z; hj[3] = b.w;
#pragma unroll
      for (int k = 0; k < 4; ++k) srj[k] = __fmul_rn(sj[k], prho);
    }
    float ay[4] = {0, 0, 0, 0}, ag[4] = {0, 0, 0, 0};
    float* col = H + j0;
    auto row_update = [&](int r, f4v h) {
      const float gi = g[r], yi = gi - gp[r];
      const float sri = __fmul_rn(ps[r], prho), hyi = phy[r];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        h[k] = rank2(h[k], sri, sj[k], pc, hj[k], hyi, srj[k]);
        ay[k] += h[k] * yi;
        ag[k] += h[k] * gi;
      }
#if !DAVA_DIAG_NO_HBM
      if (act) h_store(col + (size_t)r * Pld, h);
#endif
    };
    auto synth = [&](int r) {  // row r of gamma0 * I restricted to this lane's 4 columns
      f4v h;
      h[0] = r == j0 ? gamma0 : 0.f; h[1] = r == j0 + 1 ? gamma0 : 0.f;
      h[2] = r == j0 + 2 ? gamma0 : 0.f; h[3] = r == j0 + 3 ? gamma0 : 0.f;
      return h;
    };
    int i = 0;
#if DAVA_DIAG_NO_HBM  // timing-only build: no matrix traffic (results are wrong)
    materialized = false;
#endif
    if (materialized) {
      for (; i + U <= P; i += U) {
        f4v h[U];
#pragma unroll
        for (int u = 0; u < U; ++u) h[u] = act ? h_load(col + (size_t)(i + u) * Pld) : f4v{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) row_update(i + u, h[u]);
      }
      for (; i < P; ++i) row_update(i, act ? h_load(col + (size_t)i * Pld) : f4v{0, 0, 0, 0});
    } else {
      for (; i < P; ++i) row_update(i, synth(i));
    }
    if (act) {
      st4(hy_out + j0, make_float4(ay[0], ay[1], ay[2], ay[3]));
      st4(hg_out + j0, make_float4(ag[0], ag[1], ag[2], ag[3]));
    }
  }
}

__global__ __launch_bounds__(kBlock) void bfgs_ba_solve_kernel(SolveArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Layout L = a.L;
  const int P = L.P, M = L.M, N = L.N;
  const int Pv = a.Pv;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const LdsCarve cv = carve_lds(M, N, Pv);
  float* x = lds + cv.x;
  float* d = lds + cv.d;
  float* g = lds + cv.g0;
  float* gp = lds + cv.g1;
  float* s_cur = lds + cv.s0;
  float* s_pend = lds + cv.s1;
  float* hy_new = lds + cv.hy0;
  float* hy_pend = lds + cv.hy1;
  float* hg = lds + cv.hg;
  float* obs = lds + cv.obs;
  float* views = lds + cv.views;
  float* vpart = lds + cv.vpart;
  float* scratch = lds + cv.scratch;
  uint8_t* vis = reinterpret_cast<uint8_t*>(lds) + cv.vis_bytes_off;

  // ---- stage the problem into LDS (zero the vector pads) ----
  const float* x0 = a.x0 + (size_t)b * P;
  for (int i = tid; i < Pv; i += kBlock) {
    x[i] = i < P ? x0[i] : 0.f;
    d[i] = g[i] = gp[i] = s_cur[i] = s_pend[i] = hy_new[i] = hy_pend[i] = hg[i] = 0.f;
  }
  const int MN = M * N;
  const float* ob = a.obs + (size_t)b * 2 * MN;
  for (int i = tid; i < 2 * MN; i += kBlock) obs[i] = ob[i];
  const uint8_t* vb = a.vis + (size_t)b * MN;
  for (int i = tid; i < MN; i += kBlock) vis[i] = vb[i] ? 1 : 0;
  __syncthreads();

  float* H = a.hess ? a.hess + (size_t)b * P * a.Pld : nullptr;
  int buf = 0;
  bool materialized = false;
  float gamma0 = 1.f, pend_rho = 0.f, pend_c = 1.f;
  int steps = 0, reason = DAVA_STOP_ITERATIONS, evals = 0, trials = 0;
  float E = 0.f, unused = 0.f;

  for (int k = 0; k < a.iters; ++k) {
    { float* t = g; g = gp; gp = t; }  // gp <- previous gradient
    ba_eval<true, false, false>(L, x, nullptr, 0.f, obs, vis, g, views, vpart, scratch, buf, E, unused);
    ++evals;
    if (!(E > a.thr)) { reason = DAVA_STOP_ERROR; break; }

    if (k == 0) {
      // first step: no inverse Hessian yet, d = -g (bfgs_solver.py:152-155)
      for (int i = tid; i < P; i += kBlock) d[i] = -1.0f * g[i];
      __syncthreads();
    } else {
      float r[4] = {0, 0, 0, 0};
      float rho, c, sg, hyg;
      if (k == 1) {
        // H_0 = gamma I, gamma from N&W eq. 6.20 (bfgs_solver.py:159-167, 217-233)
        for (int i = tid; i < P; i += kBlock) {
          const float gi = g[i], yi = gi - gp[i], si = s_cur[i];
          r[0] += si * yi; r[1] += yi * yi; r[2] += si * gi; r[3] += yi * gi;
        }
        block_sum<4>(r, scratch, buf); buf ^= 1;
        const float gamma = clamp_min(r[0] / clamp_min(r[1], 1e-5f), 1e-4f);
        gamma0 = gamma;
        rho = r[0] <= 0.f ? 0.f : 1.0f / r[0];
        c = 1.0f + rho * (gamma * r[1]);
        sg = r[2];
        hyg = gamma * r[3];
        for (int i = tid; i < P; i += kBlock) {
          const float gi = g[i], yi = gi - gp[i];
          hy_new[i] = gamma * yi;
          hg[i] = gamma * gi;
        }
        // (no barrier needed: each thread reads back only its own hy_new / hg below)
      } else {
        dense_sweep(L, a.Pld, H, materialized, gamma0, s_pend, hy_pend, pend_rho, pend_c, g, gp, hy_new, hg);
        materialized = true;
        __syncthreads();
        for (int i = tid; i < P; i += kBlock) {
          const float gi = g[i], yi = gi - gp[i], si = s_cur[i], hi = hy_new[i];
          r[0] += si * yi; r[1] += hi * yi; r[2] += si * gi; r[3] += hi * gi;
        }
        block_sum<4>(r, scratch, buf); buf ^= 1;
        rho = r[0] <= 0.f ? 0.f : 1.0f / r[0];  // inverse_curvature (func_inverse_curvature.py:24-28)
        c = 1.0f + rho * r[1];
        sg = r[2];
        hyg = r[3];
      }
      // d = -H_k g,  H_k = H' + c (rho s) s^T - (rho s) (H'y)^T - (H'y) (rho s)^T
      const float rsg = rho * sg;
      for (int i = tid; i < P; i += kBlock) {
        const float sri = s_cur[i] * rho;
        d[i] = -1.0f * (hg[i] + sri * (c * sg) - sri * hyg - hy_new[i] * rsg);
      }
      // the new update becomes the pending one; recycle the old buffers
      { float* t = s_pend; s_pend = s_cur; s_cur = t; }
      { float* t = hy_pend; hy_pend = hy_new; hy_new = t; }
      pend_rho = rho;
      pend_c = c;
      __syncthreads();
    }

    // ---- strong-Wolfe line search (wolfe_conditions.py:23-239) ----
    float dphi0;
    {
      float r[1] = {0.f};
      for (int i = tid; i < P; i += kBlock) r[0] += d[i] * g[i];
      block_sum<1>(r, scratch, buf); buf ^= 1;
      dphi0 = r[0];
    }
    float a_lo = 0.f, a_hi = 0.f, al = 1.f, f_lo = E, f_hi = E, fa = E, dfa = dphi0;
    bool widen = true, zoom = false;
    const float lim = (-a.c2) * dphi0;
    for (int t = 0; t < a.max_trials; ++t) {
      if (!(widen || zoom)) break;
      if (t > 0) {
        if (widen) { a_hi = al; f_hi = fa; al = 2.0f * al; }
        if (zoom) al = 0.5f * (a_lo + a_hi);
      }
      ba_eval<false, true, true>(L, x, d, al, obs, vis, nullptr, views, vpart, scratch, buf, fa, dfa);
      ++evals;
      ++trials;
      bool fail = fa > E + (a.c1 * al) * dphi0;
      if (zoom) fail = fail || (fa >= f_lo);
      if (t > 0 && widen) fail = fail || (fa >= f_hi);
      const bool curv = a.strong ? (fabsf(dfa) <= lim) : (-1.0f * dfa <= lim);
      const bool up = widen ? (dfa >= 0.f) : (dfa * (a_hi - a_lo) >= 0.f);
      if (zoom) {
        const bool done = !fail && curv;
        const bool flip = !fail && !curv && up;
        const bool setlo = !fail && !curv;
        if (fail || done) { a_hi = al; f_hi = fa; }
        if (flip) { a_hi = a_lo; f_hi = f_lo; }
        if (setlo || done) { a_lo = al; f_lo = fa; }
        if (done) zoom = false;
      } else if (widen) {
        const bool bracket = fail;
        const bool done = !fail && curv;
        const bool flip = !fail && !curv && up;
        if (bracket) { a_lo = a_hi; f_lo = f_hi; }
        if (bracket || done) { a_hi = al; f_hi = fa; }
        if (done || flip) { a_lo = al; f_lo = fa; }
        if (bracket || flip) zoom = true;
        if (bracket || done || flip) widen = false;
      }
      if (a_lo == a_hi) zoom = false;
    }
    const float alpha = a_hi;

    // ---- take the step (bfgs_solver.py:191-199) and test its length (:203-207) ----
    {
      float r[1] = {0.f};
      for (int i = tid; i < P; i += kBlock) {
        const float si = __fmul_rn(alpha, d[i]);
        s_cur[i] = si;
        x[i] = __fadd_rn(x[i], si);
        r[0] += si * si;
      }
      block_sum<1>(r, scratch, buf); buf ^= 1;
      ++steps;
      if (!(sqrtf(r[0]) > a.min_step)) { reason = DAVA_STOP_STEP; break; }
    }
  }

  // ---- outputs ----
  __syncthreads();
  float* xo = a.x_out + (size_t)b * P;
  for (int i = tid; i < P; i += kBlock) xo[i] = x[i];
  if (a.err_out) {
    float e2 = 0.f;
    ba_eval<false, false, false>(L, x, nullptr, 0.f, obs, vis, nullptr, views, vpart, scratch, buf, e2, unused);
    if (tid == 0) a.err_out[b] = e2;
  }
  if (a.status && tid == 0) {
    int32_t* st = a.status + (size_t)b * DAVA_STATUS_WORDS;
    st[0] = steps; st[1] = reason; st[2] = evals; st[3] = trials;
  }
}

// ---- single evaluation kernel (dava_ba_evaluate) ----
struct EvalArgs {
  Layout L;
  int Pv;
  const float* obs;
  const uint8_t* vis;
  const float* x;
  const float* dir;
  const float* alpha;
  float* err;
  float* grad;
  float* slope;
};

template <bool GRAD, bool SLOPE, bool TRIAL>
__global__ __launch_bounds__(kBlock) void ba_evaluate_kernel(EvalArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Layout L = a.L;
  const int P = L.P, M = L.M, N = L.N, Pv = a.Pv;
  const int b = blockIdx.x, tid = threadIdx.x;
  const LdsCarve cv = carve_lds(M, N, Pv);
  float* x = lds + cv.x;
  float* d = lds + cv.d;
  float* g = lds + cv.g0;
  float* obs = lds + cv.obs;
  float* views = lds + cv.views;
  float* vpart = lds + cv.vpart;
  float* scratch = lds + cv.scratch;
  uint8_t* vis = reinterpret_cast<uint8_t*>(lds) + cv.vis_bytes_off;
  for (int i = tid; i < Pv; i += kBlock) {
    x[i] = i < P ? a.x[(size_t)b * P + i] : 0.f;
    d[i] = (a.dir && i < P) ? a.dir[(size_t)b * P + i] : 0.f;
    g[i] = 0.f;
  }
  const int MN = M * N;
  for (int i = tid; i < 2 * MN; i += kBlock) obs[i] = a.obs[(size_t)b * 2 * MN + i];
  for (int i = tid; i < MN; i += kBlock) vis[i] = a.vis[(size_t)b * MN + i] ? 1 : 0;
  __syncthreads();
  const float al = (TRIAL && a.alpha) ? a.alpha[b] : 0.f;
  int buf = 0;
  float E = 0.f, sl = 0.f;
  ba_eval<GRAD, SLOPE, TRIAL>(L, x, d, al, obs, vis, g, views, vpart, scratch, buf, E, sl);
  if (tid == 0) {
    a.err[b] = E;
    if (SLOPE && a.slope) a.slope[b] = sl;
  }
  if (GRAD && a.grad)
    for (int i = tid; i < P; i += kBlock) a.grad[(size_t)b * P + i] = g[i];
}

static int check_scene(const DavaScene* s, bool need_data = true) {
  if (!s) return DAVA_ERR_INVALID_ARGUMENT;
  if (s->batch < 0 || s->num_views < 2 || s->num_points < 1) return DAVA_ERR_INVALID_ARGUMENT;
  const int P = 3 + 3 * s->num_points + 6 * (s->num_views - 1) + (s->distortion ? 5 : 0);
  if (s->num_parameters != P) return DAVA_ERR_INVALID_ARGUMENT;
  if (need_data && s->batch > 0 && (!s->observations || !s->visibility)) return DAVA_ERR_INVALID_ARGUMENT;
  return DAVA_OK;
}

static size_t dense_hessian_bytes(const DavaScene* s) {
  const int P = s->num_parameters;
  return (size_t)s->batch * (size_t)P * (size_t)round_up(P, 32) * sizeof(float);
}

static int lds_bytes_for(const DavaScene* s) {
  return carve_lds(s->num_views, s->num_points, round_up(s->num_parameters, 4)).total_bytes;
}

constexpr int kMaxLds = 160 * 1024;

}  // namespace dava

using namespace dava;

extern "C" size_t dava_ba_solve_workspace_bytes(const DavaScene* scene, const DavaSolverConfig* config) {
  if (check_scene(scene, false) != DAVA_OK || !config) return 0;
  if (config->hessian_mode == DAVA_HESSIAN_DENSE) return dense_hessian_bytes(scene);
  return 0;
}

extern "C" int dava_ba_solve(const DavaScene* scene, const DavaSolverConfig* config, const float* x0,
                             float* x_out, float* error_out, int32_t* status_out, void* workspace,
                             size_t workspace_bytes, void* stream) {
  int st = check_scene(scene);
  if (st != DAVA_OK) return st;
  if (!config || config->iterations < 0 || config->max_line_search_trials < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (config->hessian_mode != DAVA_HESSIAN_DENSE) return DAVA_ERR_UNSUPPORTED;
  if (scene->batch == 0) return DAVA_OK;
  if (!x0 || !x_out) return DAVA_ERR_INVALID_ARGUMENT;
  const int lds = lds_bytes_for(scene);
  if (lds > kMaxLds) return DAVA_ERR_UNSUPPORTED;
  const size_t need = dense_hessian_bytes(scene);
  if (config->iterations > 2 && (!workspace || workspace_bytes < need)) return DAVA_ERR_WORKSPACE;
  SolveArgs a;
  a.L = Layout{scene->num_views, scene->num_points, scene->num_parameters, scene->distortion ? 1 : 0};
  a.B = scene->batch;
  a.Pv = round_up(scene->num_parameters, 4);
  a.Pld = round_up(scene->num_parameters, 32);
  a.obs = scene->observations;
  a.vis = scene->visibility;
  a.x0 = x0;
  a.x_out = x_out;
  a.err_out = error_out;
  a.status = status_out;
  a.hess = static_cast<float*>(workspace);
  a.c1 = config->sufficient_decrease;
  a.c2 = config->curvature;
  a.thr = config->error_threshold;
  a.min_step = config->minimum_step;
  a.iters = config->iterations;
  a.max_trials = config->max_line_search_trials;
  a.strong = config->strong_wolfe;
  a.mode = config->hessian_mode;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(bfgs_ba_solve_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(bfgs_ba_solve_kernel, dim3(scene->batch), dim3(kBlock), lds, s, a);
  return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH;
}

template <bool G, bool S, bool T>
static void launch_eval(const EvalArgs& a, int B, int lds, hipStream_t s) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(ba_evaluate_kernel<G, S, T>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL((ba_evaluate_kernel<G, S, T>), dim3(B), dim3(kBlock), lds, s, a);
}

extern "C" int dava_ba_evaluate(const DavaScene* scene, const float* x, const float* direction, const float* alpha,
                                float* error_out, float* grad_out, float* slope_out, void* stream) {
  int st = check_scene(scene);
  if (st != DAVA_OK) return st;
  if (scene->batch == 0) return DAVA_OK;
  if (!x || !error_out) return DAVA_ERR_INVALID_ARGUMENT;
  if (slope_out && !direction) return DAVA_ERR_INVALID_ARGUMENT;
  const int lds = lds_bytes_for(scene);
  if (lds > kMaxLds) return DAVA_ERR_UNSUPPORTED;
  EvalArgs a;
  a.L = Layout{scene->num_views, scene->num_points, scene->num_parameters, scene->distortion ? 1 : 0};
  a.Pv = round_up(scene->num_parameters, 4);
  a.obs = scene->observations;
  a.vis = scene->visibility;
  a.x = x;
  a.dir = direction;
  a.alpha = alpha;
  a.err = error_out;
  a.grad = grad_out;
  a.slope = slope_out;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool G = grad_out != nullptr, S = slope_out != nullptr, T = direction != nullptr && alpha != nullptr;
  const int B = scene->batch;
  if (G && S && T) launch_eval<true, true, true>(a, B, lds, s);
  else if (G && S) launch_eval<true, true, false>(a, B, lds, s);
  else if (G && T) launch_eval<true, false, true>(a, B, lds, s);
  else if (G) launch_eval<true, false, false>(a, B, lds, s);
  else if (S && T) launch_eval<false, true, true>(a, B, lds, s);
  else if (S) launch_eval<false, true, false>(a, B, lds, s);
  else if (T) launch_eval<false, false, true>(a, B, lds, s);
  else launch_eval<false, false, false>(a, B, lds, s);
  return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH;
}
