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
#include <algorithm>
#include <cstring>
#include <vector>

#include "ba_objective.hpp"
#include "dava_debug.hpp"
#include "dava_tape.hpp"

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
  float* hess_dense;  // HYBRID: B x P x Pld dense matrices after the histories (else null)
  float c1, c2, thr, min_step;
  int iters, max_trials, strong, mode;
  int kcap;       // COMPACT: history capacity (entries)
  int lcap;       // COMPACT, LDS mode: entries 0 .. lcap-1 live in LDS instead of HBM
  float* vecs;    // GV mode: B slices of vstride floats (kVectors x Pv, then rho_j / c_j if scal_slice)
  int vstride;
  int scal_slice;  // GV, wide pass: rho_j, c_j in the workspace slice instead of LDS
  int kcap_lds;    // history entries whose rho_j, c_j (and product coefficients) the LDS image holds
  unsigned long long* phase_cycles;  // DAVA_PHASE_TIMING builds: B x kPhases (else null)
  int* queue;     // work-queue counter (zeroed before the launch), or null: problem = blockIdx.x
  // recording solve (dava_ba_solve_record, dava_tape.hpp): x_k and g_k rows, (alpha, rho, c, gamma)
  float* tape_x;  // (B, K, Pv) or null
  float* tape_g;  // (B, K, Pv)
  float* tape_s;  // (B, tape_T)
  int tape_T;
  int stagger;    // shader cycles per start level (0: none)
  int stagger_levels;  // <= 1: odd workgroups wait `stagger`; L > 1: level (b / 8) mod L waits level x stagger
  float drop_p;   // training-mode drop path probability (0: eval mode)
  unsigned long long drop_seed;
  int second_last;  // training mode's return_second_last: a minimum-step stop keeps x_k
};

// Training mode's drop path (bfgs_solver.py:121-125): problem b keeps updating at iteration k iff
// u(seed, b, k) > p, u uniform on [0, 1) with 24-bit resolution from a counter-based 64-bit mix
// (splitmix64's finaliser over the packed counter): no state, any launch shape or work-queue
// order draws the same schedule.
__device__ __forceinline__ float drop_uniform(unsigned long long seed, int b, int k) {
  unsigned long long z = seed ^ (((unsigned long long)(unsigned)b << 32) | (unsigned)k);
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

struct LdsCarve {
  int x, d, ge, g0, g1, s0, s1, hy0, hy1, hg, obs, views, vpart, scratch, hcoef, hrho, hc, hist, vis_bytes_off,
      total_bytes;
};

constexpr int kVectors = 9;  // x d g g_prev s s_pend Hy Hy_pend Hg

// Waves per solve workgroup: 4 when the problem lives in LDS (two workgroups per CU);
// 8 in global-vector mode, where problems are few and long (C5: B = 256 on 256 CUs) and
// one workgroup per CU would otherwise leave each SIMD a single wave to hide latency with.
__host__ __device__ constexpr int solve_waves(bool gv) { return gv ? 8 : 4; }

// GV mode, COMPACT: the workgroup-wide single history pass keeps at most this many float4
// column groups per thread in registers (P <= 7 * 512 * 4 = 14336); longer rows use two passes.
constexpr int kWideMaxGroups = 7;
// History entries per block reduction in the wide pass for rows of > 2 groups per thread (two
// entries' rows do not fit the registers beside y, g and the sums there).
#ifndef DAVA_GV_ENTRIES
#define DAVA_GV_ENTRIES 1  // (microbenchmark builds only: tools/micro/wide_pass_stream.hip)
#endif
constexpr int kGvEntries = DAVA_GV_ENTRIES;
__host__ __device__ inline bool wide_history_pass(int Pv, int kcap, bool gv) {
  return gv && kcap > 0 && (Pv / 4 + kWave * solve_waves(gv) - 1) / (kWave * solve_waves(gv)) <= kWideMaxGroups;
}
// GV mode, wide pass: where each history entry's rho_j and c_j live.  In LDS (8 B per entry) while the XL
// image (x, d and the objective's gradient, 149 KB at C5) still fits beside them; past that (C5: ~950
// iterations, e.g. the reference's default cap of 1000) in the problem's workspace slice, after its
// kVectors vectors (round_up(kcap, 64) floats each), so that the XL image stays: without it the solve ran
// at 4.80k against 7.22k problems/s at K = 100 (profiles/r05_ab_c5_xl.log).  Measured before the product
// coefficients left the LDS image (when the slice took over at ~320 iterations): K = 400 689 against 539
// problems/s, the reference's defaults 323 against 264, K = 100 unchanged (profiles/r05_ab_c5_scalar_slice.log).
// The pass reads entry j's pair with one uniform load each, issued at the entry's start and needed only
// after its block reduction.
__host__ __device__ inline int gv_scalar_stride(int kcap) { return round_up(kcap, 64); }
__host__ __device__ inline int gv_slice_floats(int Pv, int kcap, bool scalars_in_slice) {
  return kVectors * Pv + (scalars_in_slice ? 2 * gv_scalar_stride(kcap) : 0);
}

// LDS image of one problem.  In global-vector (GV) mode -- large P, where the O(P)
// vectors cannot live on-chip -- the nine vectors sit in a per-problem slice of the
// workspace instead (offsets index that slice) and obs / vis are read in place.
// COMPACT LDS mode may keep the OLDEST lcap history entries on-chip (S row then W row,
// 2 Pv floats per entry): entry j is read by every iteration k > j + 1, so the first
// entries carry the most traffic (lcap = 6 at C3 removes 12% of the history reads).
// GV mode with xl ("x local"): x, d and the objective's gradient output (ge) still fit in
// LDS (3 Pv floats; C5: 149 KB), so the objective -- whose per-(view, point) work reads x
// and d and accumulates point gradients view after view, one dependent access per pair --
// runs on-chip; the other vectors stay in the workspace slice (its x and d slots unused).
__host__ __device__ inline LdsCarve carve_lds(int M, int N, int Pv, int kcap = 0, bool gv = false, int lcap = 0,
                                              bool xl = false, int nw = 0) {
  if (nw <= 0) nw = solve_waves(gv);
  LdsCarve c;
  int off = 0;
  int voff = 0;
  int& o = gv ? voff : off;
  int& ox = gv && !xl ? voff : off;
  c.x = ox; ox += Pv;
  c.d = ox; ox += Pv;
  if (gv && xl) voff += 2 * Pv;
  c.ge = gv && xl ? off : 0;
  off += gv && xl ? Pv : 0;
  c.g0 = o; o += Pv;
  c.g1 = o; o += Pv;
  c.s0 = o; o += Pv;
  c.s1 = o; o += Pv;
  c.hy0 = o; o += Pv;
  c.hy1 = o; o += Pv;
  c.hg = o; o += Pv;
  c.obs = off; off += gv ? 0 : round_up(2 * M * N, 4);
  c.views = off; off += round_up(views_floats(M), 4);
  c.vpart = off; off += round_up(vpart_floats(M, nw), 4);
  c.scratch = off; off += 2 * nw * 32;
  // COMPACT: per-entry product coefficients, for the two-pass products only (compact_products: GV rows
  // past the wide pass, LDS-mode rows of more than 4 float4 groups per lane); the single-pass forms form
  // each entry's coefficients on the fly (r05: 16 B per entry returned to the on-chip history entries /
  // the XL image)
  const bool two_pass = gv ? !wide_history_pass(Pv, kcap, true) : (Pv / 4 + kWave - 1) / kWave > 4;
  c.hcoef = off; off += two_pass ? 4 * kcap : 0;
  c.hrho = off; off += round_up(kcap, 4);
  c.hc = off; off += round_up(kcap, 4);
  c.hist = off; off += gv ? 0 : 2 * lcap * Pv;
  c.vis_bytes_off = off * 4;
  c.total_bytes = c.vis_bytes_off + (gv ? 0 : round_up(M * N, 16));
  return c;
}


__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// LDS-mode fused pass: rows of at most this many float4 groups per lane go through buffer loads (bitwise
// equal; C1, C2: C2 +2.5%, profiles/r03_ab_fused_buffer_loads_small.log; all rows, i.e. 4: C3 -6%,
// profiles/r03_ab_buffer_loads.log).  (The GV wide pass through buffer loads: C5 -2.5 .. +1.8% across
// boxes, not kept.)
constexpr int kFusedBufferLoadsGM = 2;
constexpr int kSweepRows = 4;  // DENSE sweep: matrix rows in flight per lane
// Trial slopes phi'(alpha) of the full trials (the ones that also form the gradient): forward mode (a JVP
// riding on the trial's evaluation) in LDS mode, where the reverse-mode form d . grad measured -1% at C3
// (profiles/r01b_ab_variants.log, `dot`); d . grad in global-vector mode, where it saves the pair sweep's
// tangent registers (C5 +4%, r03 interleaved A/B).  DAVA_TRIAL_DOT_LDS=1: d . grad in LDS mode too (A/B).
#ifndef DAVA_TRIAL_DOT_LDS
#define DAVA_TRIAL_DOT_LDS 0
#endif
constexpr bool kTrialDotLds = DAVA_TRIAL_DOT_LDS != 0;
constexpr bool kTrialDotGv = true;
// Lean trials (r06): a line search's trials from index kLeanFrom on are evaluated for E and the forward-mode
// slope alone -- all the Wolfe tests read (wolfe_conditions.py:116-237) -- without the reverse-mode gradient.
// If the accepted trial was lean, it is evaluated once more in the full trial form (below), so x_{k+1}'s
// objective and gradient are bit for bit what the full-trial path keeps.  The first trials (alpha = 1, accepted
// ~89% of the time at C3) stay full.  DAVA_LEAN_TRIALS (LDS mode) / DAVA_LEAN_TRIALS_GV: the first trial index
// evaluated lean, 0 = none.  LDS mode from the third trial: a search of two trials (reject, accept) would pay
// the lean trial and its full re-evaluation; interleaved A/B (profiles/r06f_lean_index_dot_gvlean_ab.log):
// from the 2nd / 3rd / 4th trial C2 0.514 / 0.514 / 0.505, C2 ray-angle 0.683 / 0.691 / 0.695, C3 0.895 for all
// (no lean trials: C2 0.46).  GV mode keeps full trials: lean from the 2nd / 3rd trial C5 -1.5% / -1.2% (its
// searches are short, and a lean trial's forward-mode tangents cost the packed sweep registers).  First
// trials with d . grad in LDS mode too (DAVA_TRIAL_DOT_LDS=1): C3 -1.1%, C2 -0.5%, not kept.
#ifndef DAVA_LEAN_TRIALS
#define DAVA_LEAN_TRIALS 2
#endif
#ifndef DAVA_LEAN_TRIALS_GV
#define DAVA_LEAN_TRIALS_GV 0
#endif
constexpr int kLeanFromLds = DAVA_LEAN_TRIALS;
constexpr int kLeanFromGv = DAVA_LEAN_TRIALS_GV;
// Runs of known no-move zoom trials iterated as the scalar recurrence they are (r06; bitwise invisible).
#ifndef DAVA_NOMOVE_RUNS
#define DAVA_NOMOVE_RUNS 1
#endif
constexpr bool kNoMoveRuns = DAVA_NOMOVE_RUNS != 0;
constexpr int kSolveWavesPerEU = 2;  // <= 256 VGPRs: two 4-wave workgroups per CU
// Diagnostic builds only (make variant FLAGS=-DDAVA_PHASE_TIMING=1): thread 0 of every
// workgroup accumulates shader-clock cycles per solver phase; dava_ba_solve prints the
// batch averages to stderr after the launch (and synchronises -- never in a product build).
#ifndef DAVA_PHASE_TIMING
#define DAVA_PHASE_TIMING 0
#endif
#if DAVA_PHASE_TIMING
constexpr int kPhases = 7;  // eval at x, history products, direction, trial evals, search logic, step, total
#define DAVA_PHASE(i)                          \
  do {                                         \
    const unsigned long long t1_ = clock64(); \
    ph_acc[i] += t1_ - ph_t0;                  \
    ph_t0 = t1_;                               \
  } while (0)
#else
#define DAVA_PHASE(i) \
  do {                \
  } while (0)
#endif

// Streaming access to the inverse Hessian: every element is read once and written once per BFGS
// iteration, never reused by another workgroup (non-temporal loads and stores measured no better,
// profiles/r01_ab_sweep_variants.log).
__device__ __forceinline__ f4v h_load(const float* p) { return *reinterpret_cast<const f4v*>(p); }
__device__ __forceinline__ void h_store(float* p, f4v v) { *reinterpret_cast<f4v*>(p) = v; }

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
template <int NW, bool PIPE>
__device__ __forceinline__ void dense_sweep(const Layout& L, int Pld, float* __restrict__ H, bool materialized, float gamma0,
                            const float* ps, const float* phy, float prho, float pc, const float* g,
                            const float* gp, float* hy_out, float* hg_out) {
  constexpr int U = kSweepRows;
  const int P = L.P;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int G = (P + 3) / 4;                      // float4 column groups
  const int Gw = (G + NW - 1) / NW;       // groups per wave
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
      if (act) h_store(col + (size_t)r * Pld, h);
    };
    auto synth = [&](int r) {  // row r of gamma0 * I restricted to this lane's 4 columns
      f4v h;
      h[0] = r == j0 ? gamma0 : 0.f; h[1] = r == j0 + 1 ? gamma0 : 0.f;
      h[2] = r == j0 + 2 ? gamma0 : 0.f; h[3] = r == j0 + 3 ? gamma0 : 0.f;
      return h;
    };
    int i = 0;
    // (the buffer descriptor's range is 32-bit: matrices past 2 GiB, P > 23,170, take the loop below)
    if (PIPE && materialized && (size_t)P * Pld * sizeof(float) < (1ull << 31)) {
      // Global-vector mode (one problem per CU, rows of thousands of groups): software-pipelined,
      // two batches of U rows in flight per wave, through buffer loads / stores (a lane past the
      // wave's groups gets an offset past the descriptor's range: its load returns 0 and its store
      // is dropped, no branch).  Without branches around the memory operations the compiler waits
      // vmcnt(8..11) before a row instead of the vmcnt(0) the predicated loads force (a full round
      // trip plus the previous batch's stores per batch).  The batches ahead are clamped to row P - 1
      // (a few redundant loads at the end, never consumed).  Same arithmetic, same order: bitwise.
      // C5 dense +4.9%; the LDS-mode kernels keep the predicated loop below: there (C3, two problems
      // per CU) the same change measured -2.8%, one batch ahead -0.4%, and 8 or 16 rows per batch
      // -0.4 / -2.7% (profiles/r05_ab_dense_sweep_pipe.log, r01_ab_sweep_variants.log).
      const auto rs = make_rsrc(H, (int)((size_t)P * Pld * sizeof(float)));
      const unsigned rowb = (unsigned)Pld * 4u;
      const unsigned base = act ? (unsigned)j0 * 4u : 0x80000000u;
      auto ldrow = [&](int r) {
        return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(base + (unsigned)r * rowb), 0, 0));
      };
      auto strow = [&](int r, f4v h) {
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, h), rs, (int)(base + (unsigned)r * rowb), 0, 0);
      };
      auto update = [&](int r, f4v h, float gi, float gpi, float psi, float phyi) {
        const float yi = gi - gpi;
        const float sri = __fmul_rn(psi, prho), hyi = phyi;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          h[k] = rank2(h[k], sri, sj[k], pc, hj[k], hyi, srj[k]);
          ay[k] += h[k] * yi;
          ag[k] += h[k] * gi;
        }
        strow(r, h);
      };
      static_assert(U == 4, "the row scalars are read as float4");
      auto consume = [&](int r0, const f4v* h) {
        const float4 g4 = ld4(g + r0), gp4 = ld4(gp + r0), ps4 = ld4(ps + r0), phy4 = ld4(phy + r0);
        update(r0, h[0], g4.x, gp4.x, ps4.x, phy4.x);
        update(r0 + 1, h[1], g4.y, gp4.y, ps4.y, phy4.y);
        update(r0 + 2, h[2], g4.z, gp4.z, ps4.z, phy4.z);
        update(r0 + 3, h[3], g4.w, gp4.w, ps4.w, phy4.w);
      };
      auto tail = [&](int r0, const f4v* h) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (r0 + u < P) update(r0 + u, h[u], g[r0 + u], gp[r0 + u], ps[r0 + u], phy[r0 + u]);
      };
      // two batches in flight, rotated without register copies (a copy would wait for the loads)
      f4v A[U], Bq[U];
#pragma unroll
      for (int u = 0; u < U; ++u) A[u] = ldrow(min(u, P - 1));
#pragma unroll
      for (int u = 0; u < U; ++u) Bq[u] = ldrow(min(U + u, P - 1));
      for (; i + 2 * U <= P; i += 2 * U) {
        consume(i, A);
#pragma unroll
        for (int u = 0; u < U; ++u) A[u] = ldrow(min(i + 2 * U + u, P - 1));
        consume(i + U, Bq);
#pragma unroll
        for (int u = 0; u < U; ++u) Bq[u] = ldrow(min(i + 3 * U + u, P - 1));
      }
      if (i + U <= P) {
        consume(i, A);
        tail(i + U, Bq);
      } else {
        tail(i, A);
      }
    } else if (materialized) {
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

// HYBRID: COMPACT until the history is full (kcap = 1024 entries), then the dense matrix.  A problem
// still running at iteration kcap + 1 folds its history into H once,
//   H_ij = gamma0 delta_ij + sum_e [ s_ei (c_e rho_e s_ej - rho_e w_ej) - w_ei (rho_e s_ej) ]
// (the rank-2 terms U_e the history stands for, compact_products), and continues with dense_sweep.  The
// iteration cap alone never pays for the dense matrix: with the reference's stopping rules problems stop
// long before 1025 iterations, in the compact phase.  Same mapping as dense_sweep (lane = float4 column
// group, the wave's share of the groups), kFoldRows rows per pass in registers, every history entry streamed
// once per pass.  Entries e < lcap are the LDS-resident ones (LH: S row then W row).  The fold is a sum in
// entry order, not the reference's sequence of rank-2 updates: the same matrix up to rounding, as COMPACT
// itself.  Its cost is P / kFoldRows passes over the whole history, and per entry and pass 2 kFoldRows row
// values every lane needs: loaded once, coalesced, by 2 kFoldRows lanes and broadcast through SGPRs
// (v_readlane; kFoldReadlane) rather than as wave-uniform vector loads.  K = 1,100 fixed (every problem folds;
// interleaved, bitwise equal, profiles/r06j_fold_rows_readlane_ab.log): 8 rows with uniform loads (r05) C3
// 8.33 s, C5 41.9 s (the fold ~34 s of it); 16 / 32 rows with uniform loads C5 19.3 / 47.0 s; readlane 16 / 32
// rows C5 **17.3** / 14.4 s, C3 **7.64** / 7.17 s.  16 rows: at 32 (128 accumulators) the LDS-mode ray-angle
// hybrid kernel -- already at 256 VGPRs with ~300 SGPRs spilled -- returned wrong results
// (test_hybrid_switch_ray_angle_matches_oracle, rel 0.83; 16 and 8 rows pass,
// profiles/r06l_fold_variants_hybrid_ray_test.log).  (One column per lane, 32 rows, uniform loads: C5 67.7 s,
// profiles/r06i_fold_column_lanes_rejected.log.)
constexpr int kHybrid = 2;  // kernel MODE (internal; callers ask for DAVA_HESSIAN_COMPACT)
#ifndef DAVA_FOLD_ROWS
#define DAVA_FOLD_ROWS 16
#endif
constexpr int kFoldRows = DAVA_FOLD_ROWS;
#ifndef DAVA_FOLD_READLANE
#define DAVA_FOLD_READLANE 1
#endif
constexpr bool kFoldReadlane = DAVA_FOLD_READLANE != 0;
template <int NW>
__device__ void fold_history(int P, int Pv, int Pld, int nh, const float* __restrict__ S, const float* __restrict__ W,
                             const float* LH, int lcap, const float* hrho, const float* hc, float gamma0,
                             float* __restrict__ H) {
  constexpr int R = kFoldRows;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int G = (P + 3) / 4;
  const int Gw = (G + NW - 1) / NW;
  const int g_end = min(G, (wave + 1) * Gw);
  for (int gb = wave * Gw; gb < g_end; gb += kWave) {
    const int grp = gb + lane;
    const bool act = grp < g_end;
    const int j0 = grp * 4;
    for (int i0 = 0; i0 < P; i0 += R) {
      float h[R][4];
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) h[r][q] = i0 + r == j0 + q ? gamma0 : 0.f;
      for (int e = 0; e < nh; ++e) {
        const float* sr = e < lcap ? LH + (size_t)2 * e * Pv : S + (size_t)e * Pv;
        const float* wr = e < lcap ? sr + Pv : W + (size_t)e * Pv;
        const float rho = hrho[e], crho = hc[e] * rho;
        float u[4] = {0, 0, 0, 0}, v[4] = {0, 0, 0, 0};
        if (act) {
          const float4 s4 = ld4(sr + j0), w4 = ld4(wr + j0);
          const float sj[4] = {s4.x, s4.y, s4.z, s4.w}, wj[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            u[q] = crho * sj[q] - rho * wj[q];
            v[q] = rho * sj[q];
          }
        }
        if constexpr (kFoldReadlane) {
          // the pass's 2R row values in one coalesced load (lane r: s_e[i0 + r], lane R + r: w_e[i0 + r]), then
          // broadcast to every lane through SGPRs (v_readlane) instead of 2R wave-uniform vector loads
          static_assert(2 * R <= kWave, "one row value per lane");
          float rv = 0.f;
          if (lane < 2 * R) {
            const int rr = lane < R ? lane : lane - R;
            rv = (lane < R ? sr : wr)[min(i0 + rr, P - 1)];
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const float si = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rv), r));
            const float wi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rv), R + r));
#pragma unroll
            for (int q = 0; q < 4; ++q) h[r][q] += si * u[q] - wi * v[q];
          }
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int i = min(i0 + r, P - 1);  // (rows past P are computed and dropped)
            const float si = sr[i], wi = wr[i];
#pragma unroll
            for (int q = 0; q < 4; ++q) h[r][q] += si * u[q] - wi * v[q];
          }
        }
      }
      if (act)
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (i0 + r < P) {
            f4v o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = j0 + q < P ? h[r][q] : 0.f;
            h_store(H + (size_t)(i0 + r) * Pld + j0, o);
          }
    }
  }
}

// COMPACT mode: the inverse Hessian is never formed.  The exact BFGS history
//   H_k = gamma0 I + sum_j U_j,   U_j v = c_j rho_j (s_j.v) s_j - rho_j (w_j.v) s_j - rho_j (s_j.v) w_j
// (w_j = H_{j-1} y_j, the same rank-2 terms the reference adds to its dense H,
// bfgs_solver.py:263-303) is kept in HBM as rows S[j], W[j] of Pv floats, so
// a product H v costs 2 passes over 2 nh P floats instead of a P^2 sweep.
// Pass 1: 4 dots per entry (s.y, w.y, s.g, w.g) -> coefficients in LDS.
// Pass 2: a = H y and b = H g as coefficient-weighted sums of the rows.
template <int U, int NW>  // U: column groups of both rows in flight per lane in pass 1
__device__ __forceinline__ void compact_products(int P, int Pv, int nh, const float* __restrict__ S, const float* __restrict__ W,
                                 float* coef, const float* hrho, const float* hc, float gamma0, const float* g,
                                 const float* gp, float* a_out, float* b_out) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // scalar: row addresses wave-uniform
  const int G = (P + 3) / 4;
  for (int j = wave; j < nh; j += NW) {
    const float* sr = S + (size_t)j * Pv;
    const float* wr = W + (size_t)j * Pv;
    float sy = 0.f, wy = 0.f, sg = 0.f, wg = 0.f;
    auto dots = [&](int q, const f4v& s4, const f4v& w4) {
      const float4 g4 = ld4(g + 4 * q), p4 = ld4(gp + 4 * q);
      const float y0 = g4.x - p4.x, y1 = g4.y - p4.y, y2 = g4.z - p4.z, y3 = g4.w - p4.w;
      sy += s4[0] * y0 + s4[1] * y1 + s4[2] * y2 + s4[3] * y3;
      wy += w4[0] * y0 + w4[1] * y1 + w4[2] * y2 + w4[3] * y3;
      sg += s4[0] * g4.x + s4[1] * g4.y + s4[2] * g4.z + s4[3] * g4.w;
      wg += w4[0] * g4.x + w4[1] * g4.y + w4[2] * g4.z + w4[3] * g4.w;
    };
    int q = lane;
    for (; q + (U - 1) * kWave < G; q += U * kWave) {
      f4v s4[U], w4[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        s4[u] = *reinterpret_cast<const f4v*>(sr + 4 * (q + u * kWave));
        w4[u] = *reinterpret_cast<const f4v*>(wr + 4 * (q + u * kWave));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) dots(q + u * kWave, s4[u], w4[u]);
    }
    for (; q < G; q += kWave)
      dots(q, *reinterpret_cast<const f4v*>(sr + 4 * q), *reinterpret_cast<const f4v*>(wr + 4 * q));
    sy = wave_sum(sy); wy = wave_sum(wy); sg = wave_sum(sg); wg = wave_sum(wg);
    if (lane == 0) {
      const float rho = hrho[j], cr = hc[j] * rho;
      coef[4 * j + 0] = cr * sy - rho * wy;
      coef[4 * j + 1] = -rho * sy;
      coef[4 * j + 2] = cr * sg - rho * wg;
      coef[4 * j + 3] = -rho * sg;
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < G; q += (kWave * NW)) {
    const float4 g4 = ld4(g + 4 * q), p4 = ld4(gp + 4 * q);
    f4v y4 = {g4.x - p4.x, g4.y - p4.y, g4.z - p4.z, g4.w - p4.w};
    f4v gg = {g4.x, g4.y, g4.z, g4.w};
    f4v a4 = gamma0 * y4, b4 = gamma0 * gg;
    const float* sr = S + 4 * q;
    const float* wr = W + 4 * q;
    int j = 0;
    for (; j + 4 <= nh; j += 4) {
      f4v s4[4], w4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s4[u] = *reinterpret_cast<const f4v*>(sr + (size_t)(j + u) * Pv);
        w4[u] = *reinterpret_cast<const f4v*>(wr + (size_t)(j + u) * Pv);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 cf = ld4(coef + 4 * (j + u));
        a4 += cf.x * s4[u] + cf.y * w4[u];
        b4 += cf.z * s4[u] + cf.w * w4[u];
      }
    }
    for (; j < nh; ++j) {
      const f4v s4 = *reinterpret_cast<const f4v*>(sr + (size_t)j * Pv);
      const f4v w4 = *reinterpret_cast<const f4v*>(wr + (size_t)j * Pv);
      const float4 cf = ld4(coef + 4 * j);
      a4 += cf.x * s4 + cf.y * w4;
      b4 += cf.z * s4 + cf.w * w4;
    }
    st4(a_out + 4 * q, make_float4(a4[0], a4[1], a4[2], a4[3]));
    st4(b_out + 4 * q, make_float4(b4[0], b4[1], b4[2], b4[3]));
  }
}

// COMPACT mode, GV (long rows, 8-wave workgroup): one pass over the history, workgroup-wide.
// Thread t owns float4 column groups t, t + 512, ... (GT of them) and keeps its columns of
// y, g and of the two running sums in registers.  E entries per round (2 while GT <= 4, else
// 1 so that s, w, y, g and the sums fit in 256 VGPRs): every thread loads its columns of the
// entries' s and w rows, forms its partial dots with y and g, one block reduction gives the
// 4E dots to every thread in the same order, and each thread adds the entries'
// contributions to its own columns of H y and H g.  Rows cross HBM once per iteration (the
// two-pass variant reads them twice).
template <int GT, int NW>
__device__ __forceinline__ void compact_products_wide(int P, int Pv, int nh, const float* __restrict__ S,
                                                      const float* __restrict__ W, const float* hrho, const float* hc,
                                                      float gamma0, const float* g, const float* gp, float* a_out,
                                                      float* b_out, float* scratch, int& buf) {
  constexpr int BLOCK = kWave * NW;
  constexpr int E = GT <= 2 ? 2 : kGvEntries;
  const int tid = threadIdx.x;
  const int G = (P + 3) / 4;
  const f4v z = f4v{0, 0, 0, 0};
  f4v y[GT], gg[GT], pa[GT], pb[GT];
#pragma unroll
  for (int u = 0; u < GT; ++u) {
    const int q = tid + u * BLOCK;
    y[u] = gg[u] = pa[u] = pb[u] = z;
    if (q < G) {
      gg[u] = *reinterpret_cast<const f4v*>(g + 4 * q);
      y[u] = gg[u] - *reinterpret_cast<const f4v*>(gp + 4 * q);
    }
  }
  auto dot4 = [](f4v a, f4v b) { const f4v t = a * b; return (t[0] + t[1]) + (t[2] + t[3]); };
  for (int j = 0; j < nh; j += E) {
    const int ne = min(E, nh - j);  // uniform
    f4v s4[E][GT], w4[E][GT];
    float d[4 * E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
#pragma unroll
      for (int u = 0; u < GT; ++u) {
        const int q = tid + u * BLOCK;
        if (u < GT - 1 && (E == 1 || e < ne)) {  // groups 0 .. GT-2 lie inside the row for every thread
          s4[e][u] = *reinterpret_cast<const f4v*>(S + (size_t)(j + e) * Pv + 4 * q);
          w4[e][u] = *reinterpret_cast<const f4v*>(W + (size_t)(j + e) * Pv + 4 * q);
          continue;
        }
        s4[e][u] = w4[e][u] = z;
        if (e < ne && q < G) {
          s4[e][u] = *reinterpret_cast<const f4v*>(S + (size_t)(j + e) * Pv + 4 * q);
          w4[e][u] = *reinterpret_cast<const f4v*>(W + (size_t)(j + e) * Pv + 4 * q);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      d[4 * e] = d[4 * e + 1] = d[4 * e + 2] = d[4 * e + 3] = 0.0f;
#pragma unroll
      for (int u = 0; u < GT; ++u) {
        d[4 * e] += dot4(s4[e][u], y[u]);
        d[4 * e + 1] += dot4(w4[e][u], y[u]);
        d[4 * e + 2] += dot4(s4[e][u], gg[u]);
        d[4 * e + 3] += dot4(w4[e][u], gg[u]);
      }
    }
    block_sum<4 * E, NW>(d, scratch, buf);
    buf ^= 1;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (e < ne) {
        const float rho = hrho[j + e], cr = hc[j + e] * rho;
        const float ay = cr * d[4 * e] - rho * d[4 * e + 1], by = -rho * d[4 * e];
        const float ag = cr * d[4 * e + 2] - rho * d[4 * e + 3], bg = -rho * d[4 * e + 2];
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          pa[u] += ay * s4[e][u] + by * w4[e][u];
          pb[u] += ag * s4[e][u] + bg * w4[e][u];
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < GT; ++u) {
    const int q = tid + u * BLOCK;
    if (q < G) {
      *reinterpret_cast<f4v*>(a_out + 4 * q) = pa[u] + gamma0 * y[u];
      *reinterpret_cast<f4v*>(b_out + 4 * q) = pb[u] + gamma0 * gg[u];
    }
  }
}

// GV mode, COMPACT, iteration k >= 2: the workgroup-wide history pass of compact_products_wide and
// everything up to the line search in ONE sweep over this thread's float4 column groups, from
// registers: H'y and H'g stay in registers (never written to the workspace), s_{k-1} is loaded
// once, the four curvature dots go through one block reduction, then d = -H_k g (same per-element
// formula as the generic tail), phi'(0)'s partial d.g, and the history append (W row <- H'y,
// S row <- s) -- instead of four more passes over workspace vectors (C5: the direction phase was
// 9% of the solve, profiles/r02_phase_cycles_c5.log).  Returns this thread's d.g partial.
// Per entry the four dots are packed 2-wide FMA chains over this thread's groups (v_pk_fma_f32,
// as the LDS-mode pass does) and the contributions to H'y, H'g packed FMAs: at C5 (GT = 7) ~250
// VALU ops per entry and wave instead of ~420.  (Rejected, interleaved A/B,
// profiles/r03_ab_c5_park_yg_lds.log: parking y and g in the dead LDS gradient / direction slots to
// free registers for two entries per reduction -- bitwise equal, but the per-entry LDS re-reads and
// the spills cost 14% with one entry and 19% with two.  Forming only H'g from the history and
// H'y = H'g + d_prev: two entries per reduction, +0.5..0.9% at C5 but a different rounding that moved
// a C2 problem 2.1e-5 from the oracle, profiles/r03_ab_hy_from_d.log.  r05, in the microbenchmark
// tools/micro/wide_pass_stream.hip: each wave owning a contiguous segment of every row instead of the
// strided groups t, t + BLOCK, ... -- 4.68 vs 4.76 us per entry staged, 4.74 vs 4.71 in registers at
// B = 256, another rounding; not adopted, profiles/r05_micro_wide_pass_ownership.log.)
template <int GT, int NW, bool STAGED = false, int ROWSLOTS = 2>
__device__ __forceinline__ float wide_direction(int P, int Pv, int nh, const float* __restrict__ S,
                                                const float* __restrict__ W, float* hrho, float* hc, float gamma0,
                                                const float* g, const float* gp, const float* s_cur, float* d,
                                                float* s_row, float* w_row, float* scratch, int& buf, int entry,
                                                float* tape_rho, float* tape_c, float* stage = nullptr,
                                                size_t row_stride = 0) {
  constexpr int BLOCK = kWave * NW;
  constexpr int E = GT <= 2 ? 2 : kGvEntries;
  const size_t RSd = row_stride ? row_stride : (size_t)Pv;  // floats from one history row to the next
  const int tid = threadIdx.x;
  const int G = (P + 3) / 4;
  const f4v z = f4v{0, 0, 0, 0};
  f4v y[GT], gg[GT], pa[GT], pb[GT];
#pragma unroll
  for (int u = 0; u < GT; ++u) {
    const int q = tid + u * BLOCK;
    y[u] = gg[u] = pa[u] = pb[u] = z;
    if (q < G) {
      gg[u] = *reinterpret_cast<const f4v*>(g + 4 * q);
      y[u] = gg[u] - *reinterpret_cast<const f4v*>(gp + 4 * q);
    }
  }
  // STAGED (XL images: stage = the dead LDS slots of d and the objective's gradient, 2 Pv floats): every
  // entry's rows come HBM -> LDS by global_load_lds (no registers in flight), issued for entry j + 1 as
  // soon as this thread has read entry j's groups back, so the copy runs under entry j's dots, block
  // reduction and accumulation.  Each thread copies and reads back only its own float4 groups (the copy's
  // lane-linear LDS layout is this pass's column ownership), so the staging buffer needs no barrier; the
  // copy is issued from inline asm so that the compiler's wait accounting does not stall the LDS traffic
  // of the reduction behind it, and its completion is waited for explicitly (vmcnt(0)) before the read.
  // The same rows, dots and sums in the same order: bitwise the register path's result
  // (profiles/r04_dma_stream_bitwise.log); C5 +4.5% (profiles/r04_ab_c5_dma_stream_rotmat.log).  M0 (the
  // copy's LDS base) is saved and restored around each copy, so the compiler's view of it stays true.
  constexpr bool staged = STAGED && E == 1;
  if constexpr (staged) {
    {
      typedef __attribute__((address_space(3))) float lds_float;
      const int wave = tid / kWave;
      const unsigned stage_off = __builtin_amdgcn_readfirstlane(
          (unsigned)(uintptr_t)((lds_float*)stage) + 16u * (unsigned)(wave * kWave));
      const unsigned lane_off = 16u * (unsigned)(tid % kWave);  // this lane's 16 B within a wave's group
      // copies address the rows as a wave-uniform 64-bit base (SGPRs) plus this thread's 32-bit byte
      // offset 16 (tid + u BLOCK), so a copy costs one VGPR, not a 64-bit address per group
      auto uniform_ptr64 = [](const float* p) {  // wave-uniform 64-bit address, in SGPRs
        const unsigned long long v = (unsigned long long)(uintptr_t)p;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
        return ((unsigned long long)hi << 32) | lo;
      };
      const unsigned w_bytes = __builtin_amdgcn_readfirstlane(4u * (unsigned)Pv);
      const unsigned voff = 16u * (unsigned)tid;  // one VGPR for every group: the group's step is in the base
      // The stage holds ROWSLOTS rows (Pv floats each; the solve's XL image has room for 2, one entry): the
      // rows stream as S_0, W_0, S_1, W_1, ..., row r into slot r % ROWSLOTS, each issued as soon as the row
      // ROWSLOTS before it (same slot) has been read back.  ROWSLOTS = 2 is one entry: entry j + 1 copied
      // while entry j is consumed.
      const int nrows = 2 * nh;
      auto copy_row = [&](int r) {  // row r (entry r / 2, S or W) -> slot r % ROWSLOTS, this thread's groups
        const float* row = ((r & 1) ? W : S) + (size_t)(r >> 1) * RSd;
        const unsigned slot_off = __builtin_amdgcn_readfirstlane(4u * (unsigned)Pv * (unsigned)(r % ROWSLOTS));
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          const int q = tid + u * BLOCK;
          const unsigned long long row_u = uniform_ptr64(row + 4 * u * BLOCK);
          const unsigned ds = __builtin_amdgcn_readfirstlane(stage_off + slot_off + 16u * (unsigned)(u * BLOCK));
          if (q < G) {
            unsigned saved;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(saved)
                : "v"(voff), "s"(row_u), "s"(ds)
                : "memory");
          }
        }
      };
      (void)lane_off;
      (void)w_bytes;
#pragma unroll
      for (int r = 0; r < ROWSLOTS; ++r)
        if (r < nrows) copy_row(r);
      // (the last group's copies are issued only by waves with lanes in it)
      const bool hl = __builtin_amdgcn_readfirstlane(tid / kWave) * kWave + (GT - 1) * BLOCK < G;
      for (int j = 0; j < nh; ++j) {
        // rows 2j and 2j + 1 must have landed; rows issued after them may stay in flight
        if (ROWSLOTS > 2 && 2 * j + 2 < nrows) {
          if (hl) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GT * (ROWSLOTS - 2)) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((GT - 1) * (ROWSLOTS - 2)) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's copies of entry j have landed
        }
        const float* st_s = stage + Pv * ((2 * j) % ROWSLOTS) + 4 * tid;  // this thread's groups: + 4 u BLOCK
        const float* st_w = stage + Pv * ((2 * j + 1) % ROWSLOTS) + 4 * tid;
        f4v s4[GT], w4[GT];
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          const int q = tid + u * BLOCK;
          s4[u] = w4[u] = z;
          if (u < GT - 1 || q < G) {
            s4[u] = *reinterpret_cast<const f4v*>(st_s + 4 * u * BLOCK);
            w4[u] = *reinterpret_cast<const f4v*>(st_w + 4 * u * BLOCK);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read back before the next copies overwrite it
        if (2 * j + ROWSLOTS < nrows) copy_row(2 * j + ROWSLOTS);
        if (2 * j + 1 + ROWSLOTS < nrows) copy_row(2 * j + 1 + ROWSLOTS);
        f2v sy2 = {0.f, 0.f}, wy2 = {0.f, 0.f}, sg2 = {0.f, 0.f}, wg2 = {0.f, 0.f};
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          sy2 = pk_fma(s4[u].lo, y[u].lo, sy2); sy2 = pk_fma(s4[u].hi, y[u].hi, sy2);
          wy2 = pk_fma(w4[u].lo, y[u].lo, wy2); wy2 = pk_fma(w4[u].hi, y[u].hi, wy2);
          sg2 = pk_fma(s4[u].lo, gg[u].lo, sg2); sg2 = pk_fma(s4[u].hi, gg[u].hi, sg2);
          wg2 = pk_fma(w4[u].lo, gg[u].lo, wg2); wg2 = pk_fma(w4[u].hi, gg[u].hi, wg2);
        }
        float dd[4] = {sy2.x + sy2.y, wy2.x + wy2.y, sg2.x + sg2.y, wg2.x + wg2.y};
#if DAVA_MICRO_NOSYNC  // (tools/micro/wide_pass_stream.hip only: the wave's own partial dots, no barrier -- timing)
        wave_sums<4>(dd);
#else
        block_sum<4, NW, true>(dd, scratch, buf);
        buf ^= 1;
#endif
        const float rho = hrho[j], cr = hc[j] * rho;
        const float ay = fmaf(cr, dd[0], -(rho * dd[1])), by = -rho * dd[0];
        const float ag = fmaf(cr, dd[2], -(rho * dd[3])), bg = -rho * dd[2];
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          pa[u] = pk_fma4(by, w4[u], pk_fma4(ay, s4[u], pa[u]));
          pb[u] = pk_fma4(bg, w4[u], pk_fma4(ag, s4[u], pb[u]));
        }
      }
    }
  }
  for (int j = 0; j < (staged ? 0 : nh); j += E) {  // (the register path)
    const int ne = min(E, nh - j);  // uniform
    f4v s4[E][GT], w4[E][GT];
    float dd[4 * E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
#pragma unroll
      for (int u = 0; u < GT; ++u) {
        const int q = tid + u * BLOCK;
        if (u < GT - 1 && (E == 1 || e < ne)) {  // groups 0 .. GT-2 lie inside the row for every thread
          s4[e][u] = *reinterpret_cast<const f4v*>(S + (size_t)(j + e) * RSd + 4 * q);
          w4[e][u] = *reinterpret_cast<const f4v*>(W + (size_t)(j + e) * RSd + 4 * q);
          continue;
        }
        s4[e][u] = w4[e][u] = z;
        if (e < ne && q < G) {
          s4[e][u] = *reinterpret_cast<const f4v*>(S + (size_t)(j + e) * RSd + 4 * q);
          w4[e][u] = *reinterpret_cast<const f4v*>(W + (size_t)(j + e) * RSd + 4 * q);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      f2v sy2 = {0.f, 0.f}, wy2 = {0.f, 0.f}, sg2 = {0.f, 0.f}, wg2 = {0.f, 0.f};
#pragma unroll
      for (int u = 0; u < GT; ++u) {
        sy2 = pk_fma(s4[e][u].lo, y[u].lo, sy2); sy2 = pk_fma(s4[e][u].hi, y[u].hi, sy2);
        wy2 = pk_fma(w4[e][u].lo, y[u].lo, wy2); wy2 = pk_fma(w4[e][u].hi, y[u].hi, wy2);
        sg2 = pk_fma(s4[e][u].lo, gg[u].lo, sg2); sg2 = pk_fma(s4[e][u].hi, gg[u].hi, sg2);
        wg2 = pk_fma(w4[e][u].lo, gg[u].lo, wg2); wg2 = pk_fma(w4[e][u].hi, gg[u].hi, wg2);
      }
      dd[4 * e] = sy2.x + sy2.y;
      dd[4 * e + 1] = wy2.x + wy2.y;
      dd[4 * e + 2] = sg2.x + sg2.y;
      dd[4 * e + 3] = wg2.x + wg2.y;
    }
    block_sum<4 * E, NW>(dd, scratch, buf);
    buf ^= 1;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (e < ne) {
        const float rho = hrho[j + e], cr = hc[j + e] * rho;
        const float ay = fmaf(cr, dd[4 * e], -(rho * dd[4 * e + 1])), by = -rho * dd[4 * e];
        const float ag = fmaf(cr, dd[4 * e + 2], -(rho * dd[4 * e + 3])), bg = -rho * dd[4 * e + 2];
#pragma unroll
        for (int u = 0; u < GT; ++u) {
          pa[u] = pk_fma4(by, w4[e][u], pk_fma4(ay, s4[e][u], pa[u]));
          pb[u] = pk_fma4(bg, w4[e][u], pk_fma4(ag, s4[e][u], pb[u]));
        }
      }
    }
  }
  // H'y, H'g in registers; s_{k-1}; the curvature dots (s.y, H'y.y, s.g, H'y.g)
  f4v sv[GT];
  float r[4] = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < GT; ++u) {
    const int q = tid + u * BLOCK;
    const f4v yu = y[u], gu = gg[u];
    pa[u] += gamma0 * yu;
    pb[u] += gamma0 * gu;
    sv[u] = q < G ? *reinterpret_cast<const f4v*>(s_cur + 4 * q) : z;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r[0] += sv[u][e] * yu[e]; r[1] += pa[u][e] * yu[e];
      r[2] += sv[u][e] * gu[e]; r[3] += pa[u][e] * gu[e];
    }
  }
  block_sum<4, NW>(r, scratch, buf);
  buf ^= 1;
  const float rho = r[0] <= 0.f ? 0.f : 1.0f / r[0];  // inverse_curvature (func_inverse_curvature.py:24-28)
  const float c = 1.0f + rho * r[1];
  const float sg = r[2], hyg = r[3];
  const float rsg = rho * sg;
  float dg = 0.f;
#pragma unroll
  for (int u = 0; u < GT; ++u) {
    const int q = tid + u * BLOCK;
    if (q < G) {
      const f4v gu = gg[u];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * q + e;
        if (i < P) {
          const float sri = sv[u][e] * rho;
          const float di = -1.0f * (pb[u][e] + sri * (c * sg) - sri * hyg - pa[u][e] * rsg);
          d[i] = di;
          dg += di * gu[e];
        } else if constexpr (staged) {
          // the staged copies filled whole groups of d's slot with the last entry's W-row pads: the
          // pads [P, Pv) of d are zero again before the objective reads x + alpha d in float4 groups
          d[i] = 0.f;
        }
      }
      *reinterpret_cast<f4v*>(s_row + 4 * q) = sv[u];  // history entry `entry` = (s, H'y, rho, c)
      *reinterpret_cast<f4v*>(w_row + 4 * q) = pa[u];
    }
  }
  if (tid == 0) {
    hrho[entry] = rho;
    hc[entry] = c;
    if (tape_rho) { *tape_rho = rho; *tape_c = c; }
  }
  return dg;
}

// COMPACT mode, single pass (P <= 1024, i.e. at most GM <= 4 float4 groups per lane):
// the coefficients of entry j depend only on entry j's own dots, so one wave
// loads the two rows of an entry into registers, reduces its 4 dots in-wave
// (no barrier), and immediately accumulates the entry's contribution to
// H y and H g -- every history row crosses HBM once per iteration.  Entries
// are dealt round-robin to the 4 waves; the per-wave partial sums are then
// added in a fixed tree ((w0 + w2) + (w1 + w3)) through 4 spare LDS vectors,
// so the result is deterministic.  a_out / b_out / spare0..3 are Pv-float LDS vectors.
// Entries j < lcap are read from the LDS-resident history LH (S row at LH + 2 j Pv, W row
// Pv floats later) -- the same values in the same per-wave order, so the result is
// bitwise the same as with every entry in HBM.
// Wave priorities (s_setprio): the two workgroups on a CU put one wave on each SIMD, and
// VALU issue between them goes by priority, then age.  A wave streaming its history (HBM-
// latency-bound, few VALU ops per byte) drops to 0 so the partner's objective evaluation or
// line-search step (VALU/LDS-latency-bound, the critical path) issues first: C3 +1.0%
// (interleaved A/B, profiles/r01c_ab_wave_priority.log; levels 1..3 within noise of
// each other).  Re-measured on the r04 kernel (profiles/r04_ab_c2_history.log): the drop still
// pays for the short rows of four problems per CU (C2: without it -2%) but no longer for C3's
// rows of four groups (without it +1.3%), so only rows of <= 2 groups per lane drop.
constexpr int kBasePrio = 2;
constexpr int kHistPrio = 0;
template <int GM>
constexpr bool kHistDropsPrio = GM <= 2;
// EF: history entries in flight per wave (each holds 2 GM float4 rows in registers).  More
// entries in flight = more bytes outstanding per wave, which is what the history stream of a
// problem with few waves (or few problems per CU) is bound by.  (Interleaved A/B,
// profiles/r02_ab_entries_in_flight.log: 3 / 5 for short rows and 3 for long rows are slower or
// within noise -- 3 costs C3 8%.)
// Rejected, r03: LDS-DMA staging of 1-3 more entries per wave by global_load_lds_dwordx4 (no VGPRs),
// in the LDS the resident entries use -- bitwise equal, but C2 -2..-5% and C1 (B = 8192) -3..-5%
// (profiles/r03_ab_c2_lds_dma_staging.log).  Rejected, r02: refilling each entry slot as soon as it
// is consumed (a register ring) -- at the 256-VGPR cap the spills (scratch ops 26 -> 201) cost C3 33%,
// C2 13% (profiles/r02_ab_history_ring.log).
template <int GM>
constexpr bool kBatchAllEntries = GM <= 2;  // compact_products_fused: on-chip entries in batches too
template <int GM>
__host__ __device__ constexpr int fused_inflight() {
  return GM <= 2 ? 4 : 2;  // rows of <= 2 float4 groups per lane (P <= 512: C1, C2) : 3-4 groups (C3)
}
template <int GM, int NW>
__device__ __forceinline__ void compact_products_fused(int P, int Pv, int nh, const float* __restrict__ S,
                                       const float* __restrict__ W, const float* LH, int lcap,
                                       const float* hrho, const float* hc,
                                       float gamma0, const float* g, const float* gp, float* a_out, float* b_out,
                                       float* spare0, float* spare1, float* spare2, float* spare3) {
  static_assert(NW == 1 || NW == 2 || NW == 4, "the cross-wave combine is written for 1, 2 or 4 waves");
  constexpr int EF = fused_inflight<GM>();
  const int lane = threadIdx.x & (kWave - 1);
  // the wave index as a scalar: the entry index j (and so each row's buffer descriptor) is then
  // provably wave-uniform; from threadIdx.x / 64 the compiler cannot tell, keeps the descriptor in
  // VGPRs and wraps every buffer load in a waterfall loop (readfirstlane x 4, compares, exec juggling)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int G = (P + 3) / 4;
  f4v pa[GM], pb[GM];
  bool ok[GM];
#pragma unroll
  for (int m = 0; m < GM; ++m) {
    // (exec-masked for every group: telling the compiler that groups 0 .. GM-2 are full -- they are,
    // GM = ceil(G / 64) -- dropped 14 instructions per 4-entry batch and cost C3 2.3%, C2 0.9%,
    // interleaved A/B profiles/r04_ab_full_groups_and_phase_scan.log)
    ok[m] = lane + kWave * m < G;
    pa[m] = f4v{0, 0, 0, 0};
    pb[m] = f4v{0, 0, 0, 0};
  }
  // y and g stay in LDS (re-read per entry: cheap ds_read_b128, saves 8 GM VGPRs)
  auto gvec = [&](int m) {
    const float4 t = ld4(g + 4 * (lane + kWave * m));
    return f4v{t.x, t.y, t.z, t.w};
  };
  auto yvec = [&](int m) {
    const int q = lane + kWave * m;
    const float4 t = ld4(g + 4 * q), u = ld4(gp + 4 * q);
    return f4v{t.x - u.x, t.y - u.y, t.z - u.z, t.w - u.w};
  };
  // One entry: its four dots with y and g (per lane: packed 2-wide FMA chains, v_pk_fma_f32),
  // one transposed wave reduction of the four (wave_sum4: uniform results), then the entry's
  // contribution to H y and H g as packed FMAs.  ~90 VALU ops per entry at GM = 4 (the round-1
  // form, per-element products + one wave_sum per dot: ~210).
  auto consume = [&](int j, const f4v (&s4)[GM], const f4v (&w4)[GM]) {
    f2v sy2 = {0.f, 0.f}, wy2 = {0.f, 0.f}, sg2 = {0.f, 0.f}, wg2 = {0.f, 0.f};
#pragma unroll
    for (int m = 0; m < GM; ++m) {
      const f4v y = yvec(m), gm = gvec(m);
      sy2 = pk_fma(s4[m].lo, y.lo, sy2); sy2 = pk_fma(s4[m].hi, y.hi, sy2);
      wy2 = pk_fma(w4[m].lo, y.lo, wy2); wy2 = pk_fma(w4[m].hi, y.hi, wy2);
      sg2 = pk_fma(s4[m].lo, gm.lo, sg2); sg2 = pk_fma(s4[m].hi, gm.hi, sg2);
      wg2 = pk_fma(w4[m].lo, gm.lo, wg2); wg2 = pk_fma(w4[m].hi, gm.hi, wg2);
    }
    const float4 t = wave_sum4(sy2.x + sy2.y, wy2.x + wy2.y, sg2.x + sg2.y, wg2.x + wg2.y);
    const float sy = t.x, wy = t.y, sg = t.z, wg = t.w;
    // coefficients with the FMA written out: both call sites (LDS- and HBM-resident entries) must
    // round them identically, and left to itself the compiler contracted cr sy - rho wy into an
    // FMA at one site and not the other (hip's __fmul_rn / __fsub_rn do not stop contraction)
    const float rho = hrho[j], cr = hc[j] * rho;
    const float ay = fmaf(cr, sy, -(rho * wy)), by = -rho * sy;
    const float ag = fmaf(cr, sg, -(rho * wg)), bg = -rho * sg;
#pragma unroll
    for (int m = 0; m < GM; ++m) {
      pa[m] = pk_fma4(by, w4[m], pk_fma4(ay, s4[m], pa[m]));
      pb[m] = pk_fma4(bg, w4[m], pk_fma4(ag, s4[m], pb[m]));
    }
  };
  // buffer loads (rows of <= kFusedBufferLoadsGM groups per lane): a descriptor per row (range =
  // the row), lane offsets loop-invariant, the groups past P read zeros through the range check
  // instead of an exec-mask branch (bitwise equal)
  constexpr bool kBufferLoads = GM <= kFusedBufferLoadsGM;
  const float* Su = uniform_ptr(S);
  const float* Wu = uniform_ptr(W);
  auto load = [&](int j, f4v (&s4)[GM], f4v (&w4)[GM]) {
    if constexpr (kBufferLoads) {
      const auto rs = make_rsrc(Su + (size_t)j * Pv, 4 * Pv);
      const auto rw = make_rsrc(Wu + (size_t)j * Pv, 4 * Pv);
#pragma unroll
      for (int m = 0; m < GM; ++m) {
        s4[m] = buf_ld4(rs, 16 * (lane + kWave * m));
        w4[m] = buf_ld4(rw, 16 * (lane + kWave * m));
      }
    } else {
      const float* sr = S + (size_t)j * Pv;
      const float* wr = W + (size_t)j * Pv;
#pragma unroll
      for (int m = 0; m < GM; ++m) {
        const int q = lane + kWave * m;
        s4[m] = ok[m] ? *reinterpret_cast<const f4v*>(sr + 4 * q) : f4v{0, 0, 0, 0};
        w4[m] = ok[m] ? *reinterpret_cast<const f4v*>(wr + 4 * q) : f4v{0, 0, 0, 0};
      }
    }
  };
  if constexpr (kHistDropsPrio<GM>) __builtin_amdgcn_s_setprio(kHistPrio);
  int j = wave;
  if constexpr (kBatchAllEntries<GM>) {
  // Rows of <= 2 groups (C1, C2): the on-chip entries and the HBM remainder go through batches too (up to
  // EF entries loaded, then consumed in order), so their consume chains (dots, wave reduction,
  // coefficients, accumulation) interleave instead of running one entry at a time.  Same entries in the
  // same order: bitwise the one-at-a-time form (profiles/r05_ab_batch_serial.log: 1024 / 1024 C2 and
  // 2048 / 2048 C3 rows equal; C1 shape +1.2%, C2 at B = 256 +1.1%, C2 at B = 1024 +-0; rows of 4 groups,
  // C3: -0.7%, so they keep the one-at-a-time form).
  auto lds_load = [&](int jj, f4v (&s4)[GM], f4v (&w4)[GM]) {
    const float* sr = LH + (size_t)2 * jj * Pv;
    const float* wr = sr + Pv;
#pragma unroll
    for (int m = 0; m < GM; ++m) {
      const int q = lane + kWave * m;
      s4[m] = ok[m] ? *reinterpret_cast<const f4v*>(sr + 4 * q) : f4v{0, 0, 0, 0};
      w4[m] = ok[m] ? *reinterpret_cast<const f4v*>(wr + 4 * q) : f4v{0, 0, 0, 0};
    }
  };
  auto batch = [&](auto count, int jj, auto&& loader) {
    constexpr int C = decltype(count)::value;
    f4v s[C][GM], w[C][GM];
#pragma unroll
    for (int e = 0; e < C; ++e) loader(jj + e * NW, s[e], w[e]);
#pragma unroll
    for (int e = 0; e < C; ++e) consume(jj + e * NW, s[e], w[e]);
  };
  auto batch_of = [&](int cnt, int jj, auto&& loader) {  // cnt: 1 .. EF, wave-uniform
    if (cnt >= 4 && EF >= 4) batch(std::integral_constant<int, (EF >= 4 ? 4 : 1)>{}, jj, loader);
    else if (cnt == 3 && EF >= 3) batch(std::integral_constant<int, (EF >= 3 ? 3 : 1)>{}, jj, loader);
    else if (cnt >= 2) batch(std::integral_constant<int, 2>{}, jj, loader);
    else batch(std::integral_constant<int, 1>{}, jj, loader);
  };
  for (const int nl = min(lcap, nh); j < nl;) {
    const int cnt = min(EF, (nl - j + NW - 1) / NW);
    batch_of(cnt, j, lds_load);
    j += cnt * NW;
  }
  for (; j + (EF - 1) * NW < nh; j += EF * NW) batch(std::integral_constant<int, EF>{}, j, load);
  if (j < nh) batch_of((nh - j + NW - 1) / NW, j, load);
  } else {
  // on-chip entries first (wave-uniform).  (Rejected, r05, profiles/r05_ab_c2_stagger_prefetch.log,
  // profiles/r05_ab_c3_prefetch.log: issuing the first HBM batch before consuming these, so its latency
  // runs under them -- bitwise the same sums, C2 +0.1%, C3 -0.5%, 26 VGPRs spilled.)
  for (const int nl = min(lcap, nh); j < nl; j += NW) {
    f4v s0[GM], w0[GM];
    const float* sr = LH + (size_t)2 * j * Pv;
    const float* wr = sr + Pv;
#pragma unroll
    for (int m = 0; m < GM; ++m) {
      const int q = lane + kWave * m;
      s0[m] = ok[m] ? *reinterpret_cast<const f4v*>(sr + 4 * q) : f4v{0, 0, 0, 0};
      w0[m] = ok[m] ? *reinterpret_cast<const f4v*>(wr + 4 * q) : f4v{0, 0, 0, 0};
    }
    consume(j, s0, w0);
  }
  // EF entries of this wave in flight: all loads issued before any is consumed.  (Rejected, r04,
  // profiles/r04_ab_variants_c2.log: two register batches, the next batch's loads issued before this
  // one is consumed -- C2 -2..-8%.)
  for (; j + (EF - 1) * NW < nh; j += EF * NW) {
    f4v s[EF][GM], w[EF][GM];
#pragma unroll
    for (int e = 0; e < EF; ++e) load(j + e * NW, s[e], w[e]);
#pragma unroll
    for (int e = 0; e < EF; ++e) consume(j + e * NW, s[e], w[e]);
  }
  for (; j < nh; j += NW) {  // the rest, one entry in flight
    f4v s0[GM], w0[GM];
    load(j, s0, w0);
    consume(j, s0, w0);
  }
  }
  if constexpr (kHistDropsPrio<GM>) __builtin_amdgcn_s_setprio(kBasePrio);
  // deterministic cross-wave sum: ((w0 + w2) + (w1 + w3)) + gamma0 * (y | g)  (NW = 4),
  // (w0 + w1) + gamma0 * (y | g)  (NW = 2), w0 + gamma0 * (y | g)  (NW = 1).  With NW > 1 the last
  // adds are left to the caller's block-wide pass after its barrier (same operations, same order):
  // (w0 + w2) | w0 in spare0/1 and (w1 + w3) | w1 in spare2/3.
  auto put = [&](float* A, float* B) {
#pragma unroll
    for (int m = 0; m < GM; ++m)
      if (ok[m]) {
        const int q = lane + kWave * m;
        *reinterpret_cast<f4v*>(A + 4 * q) = pa[m];
        *reinterpret_cast<f4v*>(B + 4 * q) = pb[m];
      }
  };
  auto add = [&](const float* A, const float* B) {
#pragma unroll
    for (int m = 0; m < GM; ++m)
      if (ok[m]) {
        const int q = lane + kWave * m;
        pa[m] += *reinterpret_cast<const f4v*>(A + 4 * q);
        pb[m] += *reinterpret_cast<const f4v*>(B + 4 * q);
      }
  };
  if constexpr (NW == 1) {  // + gamma0 (y | g), into the outputs
#pragma unroll
    for (int m = 0; m < GM; ++m)
      if (ok[m]) {
        pa[m] += gamma0 * yvec(m);
        pb[m] += gamma0 * gvec(m);
      }
    put(a_out, b_out);
    return;
  }
  if constexpr (NW == 2) {
    if (wave == 0) put(spare0, spare1);
    if (wave == 1) put(spare2, spare3);
    return;
  }
  if (wave == 2) put(spare0, spare1);
  if (wave == 3) put(spare2, spare3);
  __syncthreads();
  if (wave == 0) { add(spare0, spare1); put(spare0, spare1); }
  if (wave == 1) { add(spare2, spare3); put(spare2, spare3); }
}

// XL: GV mode with x, d and the objective's gradient in LDS.  PPT > 0: the objective keeps
// each thread's (<= PPT) points in registers across the view sweep (ba_eval).
// NW: waves per workgroup -- 8 in GV mode; 4 (default) or 2 in LDS mode (two-wave workgroups put
// twice as many small problems on a CU at once, DESIGN.md 3.1 Launch).
// SLICE: the GV wide pass's rho_j, c_j in the workspace slice (gv_scalar_stride), a kernel of its own:
// chosen at run time inside one kernel, the two forms cost both 1-10% to register allocation
// (profiles/r05_ab_c5_scalar_slice.log).  (The LDS image's scalar capacity stays a run-time argument,
// kcap_lds: with the constant 0 in the SLICE kernels this compiler rejects the kernel with an illegal
// V_CMP_NE_U32 on src_shared_base.)
template <int MODE, bool GV, int RES, bool XL, int PPT, int NW, bool SLICE = false>
__global__ __launch_bounds__(kWave * NW, kSolveWavesPerEU) void bfgs_ba_solve_kernel(SolveArgs a) {
  static_assert(!XL || GV, "XL is a global-vector-mode variant");
  static_assert(!SLICE || (GV && MODE != DAVA_HESSIAN_DENSE), "SLICE is a global-vector history variant");
  static_assert(GV ? NW == solve_waves(true) : (NW == 1 || NW == 2 || NW == 4), "LDS mode runs 1-, 2- or 4-wave workgroups");
  constexpr int BLOCK = kWave * NW;
  constexpr bool kTrialDot = GV ? kTrialDotGv : kTrialDotLds;
  constexpr int kLeanFrom = GV ? kLeanFromGv : kLeanFromLds;
  constexpr bool kLean = kLeanFrom > 0;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __builtin_amdgcn_s_setprio(kBasePrio);
  const Layout L = a.L;
  const int P = L.P, M = L.M, N = L.N;
  const int Pv = a.Pv;
  const int tid = threadIdx.x;
  // Work queue (a.queue != null): the grid holds as many workgroups as are resident at once and
  // each takes the next problem when it finishes one, so a problem that stops early or runs a
  // long line search never leaves its slot idle.  Without a queue: problem = blockIdx.x.
  __shared__ int queued_problem;
  // Staggered start (a.stagger > 0: every problem of the launch is resident at once): the odd
  // workgroups -- dealt round-robin, so the odd XCDs -- start a.stagger shader cycles (~8 us) late.
  // Problems that start together stay in phase for the whole solve, so every CU streams history
  // rows at the same time (HBM-bound) and evaluates the objective at the same time (VALU-bound);
  // offsetting half the chip by part of an iteration lets one half's stream run while the other
  // half evaluates.  C2 (B = 1024): +6% on two boxes, +0.4% on a third; C3 (16 problems per slot)
  // gets no stagger
  // (profiles/r02_ab_stagger.log).  Results are unchanged (timing only).
  // Spread start (a.stagger_levels = L > 1; GV launches, one long problem per CU): within each XCD
  // (workgroups are dealt round-robin, so b / 8 numbers them inside their XCD) the problems start at
  // L evenly spaced offsets.  Every problem alternates an HBM-bound history stream with a VALU-bound
  // objective evaluation; started together, all CUs stream at once and then all compute at once.
  // (Rejected, r05, profiles/r05_ab_c2_stagger_prefetch.log: levels by (b >> 8) mod L, i.e. the
  // problems sharing one CU started a quarter or half of an iteration apart -- C2 within +-1%.)
  const int level = a.stagger_levels > 1 ? (int)((blockIdx.x >> 3) % (unsigned)a.stagger_levels) : (blockIdx.x & 1);
  if (a.stagger > 0 && level > 0) {
    const unsigned long long t0 = clock64();
    const unsigned long long wait = (unsigned long long)a.stagger * (unsigned long long)level;
    while (clock64() - t0 < wait) __builtin_amdgcn_s_sleep(8);
  }
  for (int b = blockIdx.x;;) {
    if (a.queue) {
      __syncthreads();  // every thread is done with the previous problem's LDS image
      if (tid == 0) queued_problem = atomicAdd(a.queue, 1);
      __syncthreads();
      b = queued_problem;
      if (b >= a.B) break;
    }
    constexpr bool kHistory = MODE != DAVA_HESSIAN_DENSE;  // COMPACT, or HYBRID's compact phase
    const int lcap = kHistory && !GV ? a.lcap : 0;
    constexpr bool gvs = SLICE;  // rho_j, c_j in the workspace slice
    const LdsCarve cv = carve_lds(M, N, Pv, kHistory ? a.kcap_lds : 0, GV, lcap, XL, NW);
    float* LH = lds + cv.hist;  // LDS-resident history entries 0 .. lcap-1
    float* vb0 = GV ? a.vecs + (size_t)b * a.vstride : lds;
    float* x = (GV && !XL ? vb0 : lds) + cv.x;
    float* d = (GV && !XL ? vb0 : lds) + cv.d;
    float* ge = lds + cv.ge;  // XL: the objective's gradient output, copied to g / gp after each evaluation
    // the objective's gradient target and its publication to the workspace vector `dst`
    auto grad_buf = [&](float* dst) { return XL ? ge : dst; };
    auto publish = [&](float* dst) {
      if constexpr (XL) {
        for (int i = tid; i < P; i += BLOCK) dst[i] = ge[i];
        __syncthreads();
      }
    };
    float* g = vb0 + cv.g0;
    float* gp = vb0 + cv.g1;
    float* hcoef = lds + cv.hcoef;
    float* hrho = gvs ? vb0 + kVectors * Pv : lds + cv.hrho;
    float* hc = gvs ? hrho + gv_scalar_stride(a.kcap) : lds + cv.hc;
    float* s_cur = vb0 + cv.s0;
    float* s_pend = vb0 + cv.s1;
    float* hy_new = vb0 + cv.hy0;
    float* hy_pend = vb0 + cv.hy1;
    float* hg = vb0 + cv.hg;
    float* views = lds + cv.views;
    float* vpart = lds + cv.vpart;
    float* scratch = lds + cv.scratch;
    const int MN = M * N;
    const float* obs = GV ? a.obs + (size_t)b * 2 * MN : lds + cv.obs;
    const uint8_t* vis = GV ? a.vis + (size_t)b * MN : reinterpret_cast<uint8_t*>(lds) + cv.vis_bytes_off;

    // ---- stage the problem into LDS (zero the vector pads) ----
    const float* x0 = a.x0 + (size_t)b * P;
    for (int i = tid; i < Pv; i += BLOCK) {
      x[i] = i < P ? x0[i] : 0.f;
      d[i] = g[i] = gp[i] = s_cur[i] = s_pend[i] = hy_new[i] = hy_pend[i] = hg[i] = 0.f;
    }
    if (!GV) {
      float* o = lds + cv.obs;
      uint8_t* v = reinterpret_cast<uint8_t*>(lds) + cv.vis_bytes_off;
      const float* ob = a.obs + (size_t)b * 2 * MN;
      for (int i = tid; i < 2 * MN; i += BLOCK) o[i] = ob[i];
      const uint8_t* vbb = a.vis + (size_t)b * MN;
      for (int i = tid; i < MN; i += BLOCK) v[i] = vbb[i] ? 1 : 0;
    }
    __syncthreads();

    float* H = nullptr;   // DENSE (and HYBRID's dense phase): this problem's P x Pld inverse Hessian
    float* SH = nullptr;  // COMPACT: history rows S[kcap][Pv], W[kcap][Pv]
    float* WH = nullptr;
    if (MODE == DAVA_HESSIAN_DENSE) {
      H = a.hess ? a.hess + (size_t)b * P * a.Pld : nullptr;
    } else if (a.hess) {
      SH = a.hess + (size_t)b * 2 * a.kcap * Pv;
      WH = SH + (size_t)a.kcap * Pv;
      if (MODE == kHybrid) H = a.hess_dense + (size_t)b * P * a.Pld;
    }
    int buf = 0;
    bool materialized = false;
    float gamma0 = 1.f, pend_rho = 0.f, pend_c = 1.f;
    int steps = 0, reason = DAVA_STOP_ITERATIONS, evals = 0, trials = 0;
    float E = 0.f, unused = 0.f;

    // When the line search accepts the step it evaluated last, that trial (which also
    // formed the full gradient) IS the evaluation at x_{k+1} = x_k + alpha d: same point,
    // bit for bit, so the next iteration's objective + gradient are taken from it.
    bool have_next = false;
    float E_next = 0.f;
  #if DAVA_PHASE_TIMING
    unsigned long long ph_acc[kPhases] = {0, 0, 0, 0, 0, 0, 0};
    const unsigned long long ph_start = clock64();
    unsigned long long ph_t0 = ph_start;
  #endif
    // training mode: the drop path stops this problem at the top of iteration kend (a.iters: never).
    // Drawn once here and used as the loop's bound, so the solve loop carries nothing extra (a
    // per-iteration test cost C3 6% through register allocation, profiles/r02_ab_drop_check.log).
    int kend = a.iters;
    if (a.drop_p > 0.f) {
      kend = 0;
      while (kend < a.iters && drop_uniform(a.drop_seed, b, kend) > a.drop_p) ++kend;
    }
    int k = 0;
    for (; k < kend; ++k) {
      { float* t = g; g = gp; gp = t; }  // gp <- previous gradient; g <- (trial) gradient buffer
      if (a.tape_x) {  // recording: x_k (the same threads wrote x[i] when the last step was taken)
        float* r = a.tape_x + ((size_t)b * a.iters + k) * Pv;
        for (int i = tid; i < Pv; i += BLOCK) r[i] = x[i];  // (pads are zero)
      }
      if (have_next) {
        E = E_next;
      } else {
        ba_eval<true, false, false, false, false, RES, float, NW, PPT, GV>(L, x, nullptr, 0.f, obs, vis, grad_buf(g), views, vpart,
                                                                  scratch, buf, E, unused);
        publish(g);
        ++evals;
      }
      DAVA_PHASE(0);
      if (a.tape_g) {  // recording: g_k
        float* r = a.tape_g + ((size_t)b * a.iters + k) * Pv;
        for (int i = tid; i < Pv; i += BLOCK) r[i] = g[i];
      }
      if (!(E > a.thr)) { reason = DAVA_STOP_ERROR; break; }

      // phi'(0) = d . g is accumulated where d is formed (same per-thread order as a separate
      // pass over d); its block reduction below is also the barrier that publishes d
      float dg = 0.f;
      if (k == 0) {
        // first step: no inverse Hessian yet, d = -g (bfgs_solver.py:152-155)
        for (int i = tid; i < P; i += BLOCK) {
          const float di = -1.0f * g[i];
          d[i] = di;
          dg += di * g[i];
        }
      } else {
        float r[4] = {0, 0, 0, 0};
        float rho = 0.f, c = 1.f, sg = 0.f, hyg = 0.f;
        bool deferred = false;  // the fused pass left its last cross-wave add to the pass below
        bool tail_done = false;  // GV: wide_direction formed d and appended the history entry itself
        if (k == 1) {
          // H_0 = gamma I, gamma from N&W eq. 6.20 (bfgs_solver.py:159-167, 217-233)
          for (int i = tid; i < P; i += BLOCK) {
            const float gi = g[i], yi = gi - gp[i], si = s_cur[i];
            r[0] += si * yi; r[1] += yi * yi; r[2] += si * gi; r[3] += yi * gi;
          }
          block_sum<4, NW>(r, scratch, buf); buf ^= 1;
          const float gamma = clamp_min(r[0] / clamp_min(r[1], 1e-5f), 1e-4f);
          gamma0 = gamma;
          if (a.tape_s && tid == 0) a.tape_s[(size_t)b * a.tape_T + 3 * a.iters] = gamma;
          rho = r[0] <= 0.f ? 0.f : 1.0f / r[0];
          c = 1.0f + rho * (gamma * r[1]);
          sg = r[2];
          hyg = gamma * r[3];
          for (int i = tid; i < P; i += BLOCK) {
            const float gi = g[i], yi = gi - gp[i];
            hy_new[i] = gamma * yi;
            hg[i] = gamma * gi;
          }
          // (no barrier needed: each thread reads back only its own hy_new / hg below)
        } else {
          if constexpr (MODE == DAVA_HESSIAN_DENSE) {
            dense_sweep<NW, GV>(L, a.Pld, H, materialized, gamma0, s_pend, hy_pend, pend_rho, pend_c, g, gp, hy_new, hg);
            materialized = true;
          } else if (MODE == kHybrid && k - 1 >= a.kcap) {
            // the history is full: fold it into H (once), then sweep H as DENSE does.  The fold is
            // H' itself, so this first sweep applies no pending update (zero rows, rho 0: exact).
            if (!materialized) {
              for (int i = tid; i < Pv; i += BLOCK) s_pend[i] = hy_pend[i] = 0.f;
              fold_history<NW>(P, Pv, a.Pld, a.kcap, SH, WH, LH, lcap, hrho, hc, gamma0, H);
              pend_rho = 0.f;
              pend_c = 1.f;
              __syncthreads();
            }
            dense_sweep<NW, GV>(L, a.Pld, H, true, gamma0, s_pend, hy_pend, pend_rho, pend_c, g, gp, hy_new, hg);
            materialized = true;
          } else {
            const int G4 = (P + 3) / 4;
            const int GM = (G4 + kWave - 1) / kWave;
            deferred = !GV && NW > 1 && GM <= 4;
            if constexpr (GV) {  // workgroup-wide single pass, else two passes
              const int GT = (G4 + kWave * NW - 1) / (kWave * NW);
              const int nh = k - 1;
              float* tr = a.tape_s ? a.tape_s + (size_t)b * a.tape_T + a.iters + k - 1 : nullptr;
              float* tcp = tr ? tr + a.iters : nullptr;
              float* srow = SH + (size_t)(k - 1) * Pv;
              float* wrow = WH + (size_t)(k - 1) * Pv;
              const bool fuse = wide_history_pass(Pv, a.kcap, GV) && k - 1 < a.kcap;
              if (fuse) {
                tail_done = true;
                if (GT <= 1) dg = wide_direction<1, NW, XL>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, s_cur, d, srow, wrow, scratch, buf, k - 1, tr, tcp, XL ? lds + cv.d : nullptr);
                else if (GT == 2) dg = wide_direction<2, NW, XL>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, s_cur, d, srow, wrow, scratch, buf, k - 1, tr, tcp, XL ? lds + cv.d : nullptr);
                else if (GT == 3) dg = wide_direction<3, NW, XL>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, s_cur, d, srow, wrow, scratch, buf, k - 1, tr, tcp, XL ? lds + cv.d : nullptr);
                else if (GT == 4) dg = wide_direction<4, NW, XL>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, s_cur, d, srow, wrow, scratch, buf, k - 1, tr, tcp, XL ? lds + cv.d : nullptr);
                else if (GT == 5) dg = wide_direction<5, NW, XL>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, s_cur, d, srow, wrow, scratch, buf, k - 1, tr, tcp, XL ? lds + cv.d : nullptr);
                else if (GT == 6) dg = wide_direction<6, NW, XL>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, s_cur, d, srow, wrow, scratch, buf, k - 1, tr, tcp, XL ? lds + cv.d : nullptr);
                else dg = wide_direction<7, NW, XL>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, s_cur, d, srow, wrow, scratch, buf, k - 1, tr, tcp, XL ? lds + cv.d : nullptr);
              } else if (!wide_history_pass(Pv, a.kcap, GV))
                compact_products<GV ? 8 : 1, NW>(P, Pv, nh, SH, WH, hcoef, hrho, hc, gamma0, g, gp, hy_new, hg);
              else if (GT <= 1) compact_products_wide<1, NW>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, hy_new, hg, scratch, buf);
              else if (GT == 2) compact_products_wide<2, NW>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, hy_new, hg, scratch, buf);
              else if (GT == 3) compact_products_wide<3, NW>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, hy_new, hg, scratch, buf);
              else if (GT == 4) compact_products_wide<4, NW>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, hy_new, hg, scratch, buf);
              else if (GT == 5) compact_products_wide<5, NW>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, hy_new, hg, scratch, buf);
              else if (GT == 6) compact_products_wide<6, NW>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, hy_new, hg, scratch, buf);
              else compact_products_wide<7, NW>(P, Pv, nh, SH, WH, hrho, hc, gamma0, g, gp, hy_new, hg, scratch, buf);
            } else
            if (GM <= 1) compact_products_fused<1, NW>(P, Pv, k - 1, SH, WH, LH, lcap, hrho, hc, gamma0, g, gp, hy_new, hg, s_pend, hy_pend, d, hg);
            else if (GM == 2) compact_products_fused<2, NW>(P, Pv, k - 1, SH, WH, LH, lcap, hrho, hc, gamma0, g, gp, hy_new, hg, s_pend, hy_pend, d, hg);
            else if (GM == 3) compact_products_fused<3, NW>(P, Pv, k - 1, SH, WH, LH, lcap, hrho, hc, gamma0, g, gp, hy_new, hg, s_pend, hy_pend, d, hg);
            else if (GM == 4) compact_products_fused<4, NW>(P, Pv, k - 1, SH, WH, LH, lcap, hrho, hc, gamma0, g, gp, hy_new, hg, s_pend, hy_pend, d, hg);
            else
            // GV mode (very long rows, few resident waves): 8 column groups in flight per lane;
            // the LDS-mode kernel keeps the lean loop (its register budget is the fused pass's)
            compact_products<GV ? 8 : 1, NW>(P, Pv, k - 1, SH, WH, hcoef, hrho, hc, gamma0, g, gp, hy_new, hg);
          }
          if (!tail_done) {
          __syncthreads();
          DAVA_PHASE(1);
          if (deferred) {  // finish the fused pass's cross-wave sum here, all threads at once
            for (int i = tid; i < P; i += BLOCK) {
              const float gi = g[i], yi = gi - gp[i], si = s_cur[i];
              float hi, gh;
              hi = s_pend[i] + d[i];
              gh = hy_pend[i] + hg[i];
              hi += gamma0 * yi;
              gh += gamma0 * gi;
              hy_new[i] = hi;
              hg[i] = gh;
              r[0] += si * yi; r[1] += hi * yi; r[2] += si * gi; r[3] += hi * gi;
            }
          } else
          for (int i = tid; i < P; i += BLOCK) {
            const float gi = g[i], yi = gi - gp[i], si = s_cur[i], hi = hy_new[i];
            r[0] += si * yi; r[1] += hi * yi; r[2] += si * gi; r[3] += hi * gi;
          }
          block_sum<4, NW>(r, scratch, buf); buf ^= 1;
          rho = r[0] <= 0.f ? 0.f : 1.0f / r[0];  // inverse_curvature (func_inverse_curvature.py:24-28)
          c = 1.0f + rho * r[1];
          sg = r[2];
          hyg = r[3];
          }
        }
        // d = -H_k g,  H_k = H' + c (rho s) s^T - (rho s) (H'y)^T - (H'y) (rho s)^T
        const float rsg = rho * sg;
        if (!tail_done)
        for (int i = tid; i < P; i += BLOCK) {
          const float sri = s_cur[i] * rho;
          const float di = -1.0f * (hg[i] + sri * (c * sg) - sri * hyg - hy_new[i] * rsg);
          d[i] = di;
          dg += di * g[i];
        }
        if (MODE == DAVA_HESSIAN_DENSE || (MODE == kHybrid && k - 1 >= a.kcap)) {
          // the new update becomes the pending one; recycle the old buffers
          { float* t = s_pend; s_pend = s_cur; s_cur = t; }
          { float* t = hy_pend; hy_pend = hy_new; hy_new = t; }
          pend_rho = rho;
          pend_c = c;
        } else if (k - 1 < a.kcap && !tail_done) {
          // append U_k = (s, H y, rho, c) to the history (entry k-1), on-chip if it is one of the first lcap
          if (k - 1 < lcap) {
            float* sr = LH + (size_t)2 * (k - 1) * Pv;
            for (int i = tid; i < Pv; i += BLOCK) { sr[i] = s_cur[i]; sr[Pv + i] = hy_new[i]; }
            if (a.tape_x) {  // recording: the tape keeps every entry (the reads stay on chip)
              float* tsr = SH + (size_t)(k - 1) * Pv;
              float* twr = WH + (size_t)(k - 1) * Pv;
              for (int i = tid; i < Pv; i += BLOCK) { tsr[i] = s_cur[i]; twr[i] = hy_new[i]; }
            }
          } else {
            float* sr = SH + (size_t)(k - 1) * Pv;
            float* wr = WH + (size_t)(k - 1) * Pv;
            for (int i = tid; i < Pv; i += BLOCK) { sr[i] = s_cur[i]; wr[i] = hy_new[i]; }
          }
          if (tid == 0) {
            hrho[k - 1] = rho;
            hc[k - 1] = c;
            if (a.tape_s) {
              a.tape_s[(size_t)b * a.tape_T + a.iters + k - 1] = rho;
              a.tape_s[(size_t)b * a.tape_T + 2 * a.iters + k - 1] = c;
            }
          }
        }
      }

      // ---- strong-Wolfe line search (wolfe_conditions.py:23-239) ----
      float dphi0;
      {
        float r[1] = {dg};
        block_sum<1, NW>(r, scratch, buf); buf ^= 1;
        dphi0 = r[0];
      }
      DAVA_PHASE(2);
      float a_lo = 0.f, a_hi = 0.f, al = 1.f, f_lo = E, f_hi = E, fa = E, dfa = dphi0;
      float last_al = 0.f, last_fa = 0.f;
      // Largest alpha seen whose trial point rounded back to x.  Rounding is monotone
      // (0 <= a' <= a => |fl(a' d_i)| <= |fl(a d_i)| and fl(x_i + .) stays x_i), so every smaller
      // trial is a no-move point too and needs neither evaluation nor the check: at fp32
      // stagnation a bisection towards 0 runs ~150 such trials per line search (C2's slowest
      // problems: thousands per solve).
      float nomove_al = -1.0f;
      bool widen = true, zoom = false, evaluated = false, last_same = false;
      bool last_grad = false;  // the last evaluated trial formed its gradient (reusable at x_{k+1})
      // trial gradients go into gp's buffer (g_prev is dead once d is formed)
      const float lim = (-a.c2) * dphi0;
      for (int t = 0; t < a.max_trials; ++t) {
        if (!(widen || zoom)) break;
        if (t > 0) {
          if (widen) { a_hi = al; f_hi = fa; al = 2.0f * al; }
          if (zoom) al = 0.5f * (a_lo + a_hi);
        }
        DAVA_PHASE(4);
        // Trial points that round back to x exactly (tiny alpha, e.g. bisecting an uphill
        // direction at fp32 stagnation) need no evaluation: the reference's closure would
        // return f(x) and, via autograd w.r.t. alpha, (d * g).sum() -- exactly f0 and
        // phi'(0).  The check rides on the objective's first reduction (CHECK).  Otherwise
        // E and the full gradient at the trial point are formed (kept for reuse as the
        // next iterate's gradient) and phi'(alpha) = d . grad (DOT) -- for the first trial;
        // later ones form E and phi'(alpha) only (kLean).
        const bool known_same = al <= nomove_al;  // uniform
        if (kNoMoveRuns && known_same && zoom && E >= f_lo) {
          // A run of known no-move trials in the zoom phase: each trial point is x itself (f = E, phi' =
          // phi'(0)), and with E >= f_lo every one fails the sufficient-decrease test, so a_hi <- alpha and
          // the next bisection point is tried.  That is a scalar recurrence: iterate it here, without the
          // trial machinery, until the interval closes, the next point needs an evaluation (above
          // nomove_al) or the trial budget ends -- the same states and counts as the general path below,
          // trial by trial (uniform; C2's slowest problems run thousands of these per solve).
          for (;;) {
            a_hi = al;
            f_hi = E;
            ++trials;
            if (a_lo == a_hi) { zoom = false; break; }
            if (t + 1 >= a.max_trials) break;
            const float nx = 0.5f * (a_lo + a_hi);
            if (!(nx <= nomove_al)) break;
            al = nx;
            ++t;
          }
          evaluated = true;
          last_same = true;
          last_al = al;
          last_fa = fa = E;
          dfa = dphi0;
          continue;
        }
        const bool lean = kLean && t >= kLeanFrom;  // uniform
        bool moved = false;
        if (!known_same) {
          if (lean)
            moved = ba_eval<false, true, true, false, true, RES, float, NW, PPT, GV>(
                L, x, d, al, obs, vis, nullptr, views, vpart, scratch, buf, fa, dfa);
          else
            moved = ba_eval<true, !kTrialDot, true, kTrialDot, true, RES, float, NW, PPT, GV>(
                L, x, d, al, obs, vis, grad_buf(gp), views, vpart, scratch, buf, fa, dfa);
        }
        if (moved) {
          ++evals;
          last_same = false;
          last_grad = !lean;
          if (kLean && lean && !(isfinite(fa) && isfinite(dfa))) {
            // overflowed lean trial: the rule below needs the reverse-mode gradient (rare): the full trial form
            ba_eval<true, !kTrialDot, true, kTrialDot, false, RES, float, NW, PPT, GV>(
                L, x, d, al, obs, vis, grad_buf(gp), views, vpart, scratch, buf, fa, dfa);
            ++evals;
            last_grad = true;
          }
          // Overflowed trial (fp32 at a wild step): the reference's phi'(alpha) is autograd w.r.t.
          // alpha, i.e. (grad E(x + alpha d) * d).sum() (wolfe_conditions.py:134-143) -- NaN as
          // soon as the reverse-mode gradient holds a NaN or infinities of both signs, where the
          // forward-mode tangent may come out as +-Inf.  The NaN-blind Wolfe comparisons branch on
          // that class (a -Inf slope passes `phi' (a_hi - a_lo) >= 0` when a_hi < a_lo, NaN does
          // not), so here the slope is re-formed from the trial's reverse-mode gradient.  Finite
          // trials keep the forward-mode slope bit for bit.  Uniform branch (fa, dfa are
          // block-reduced); ba_eval<GRAD> ends with a barrier, so the gradient is complete.
          if (!(isfinite(fa) && isfinite(dfa))) {
            const float* gt = grad_buf(gp);
            float r[1] = {0.f};
            for (int i = tid; i < P; i += BLOCK) r[0] += gt[i] * d[i];
            block_sum<1, NW>(r, scratch, buf); buf ^= 1;
            dfa = r[0];
          }
        } else {
          fa = E;
          dfa = dphi0;
          last_same = true;
          if (!known_same) nomove_al = al;
        }
        DAVA_PHASE(3);
        ++trials;
        evaluated = true;
        last_al = al;
        last_fa = fa;
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
      if (a.tape_s && tid == 0) a.tape_s[(size_t)b * a.tape_T + k] = alpha;
      if constexpr (kLean) {
        if (evaluated && last_al == alpha && !last_same && !last_grad) {  // uniform
          // The accepted trial was lean: evaluate it again in the full trial form (the same point, formed
          // the same way, the same instantiation as a first trial), so x_{k+1}'s objective and gradient are
          // bit for bit those the full-trial path keeps -- the trajectory does not depend on which trial of
          // the search was accepted.  Rejected trials (the zoom tails of C2's slowest problems) stay lean.
          float f2, s2;
          ba_eval<true, !kTrialDot, true, kTrialDot, true, RES, float, NW, PPT, GV>(
              L, x, d, alpha, obs, vis, grad_buf(gp), views, vpart, scratch, buf, f2, s2);
          ++evals;
          last_fa = f2;
          last_grad = true;
        }
      }
      have_next = evaluated && last_al == alpha && (last_same || last_grad);
      E_next = last_fa;
      if (have_next && last_same) {  // x_{k+1} == x_k bitwise: its gradient is g itself
        for (int i = tid; i < P; i += BLOCK) gp[i] = g[i];
      } else if (have_next) {
        publish(gp);  // XL: only the trial that is kept needs its gradient in the workspace
      }
      DAVA_PHASE(4);

      // ---- take the step (bfgs_solver.py:191-199) and test its length (:203-207) ----
      {
        float r[1] = {0.f};
        if (a.second_last) {  // x moves only once the step has passed the test (uniform branch)
          for (int i = tid; i < P; i += BLOCK) {
            const float si = __fmul_rn(alpha, d[i]);
            s_cur[i] = si;
            r[0] += si * si;
          }
        } else {
          for (int i = tid; i < P; i += BLOCK) {
            const float si = __fmul_rn(alpha, d[i]);
            s_cur[i] = si;
            x[i] = __fadd_rn(x[i], si);
            r[0] += si * si;
          }
        }
        block_sum<1, NW>(r, scratch, buf); buf ^= 1;
        ++steps;
        DAVA_PHASE(5);
        if (!(sqrtf(r[0]) > a.min_step)) { reason = DAVA_STOP_STEP; break; }
        if (a.second_last) {  // the same additions, after the test (bfgs_solver.py:208-212)
          for (int i = tid; i < P; i += BLOCK) x[i] = __fadd_rn(x[i], s_cur[i]);
          __syncthreads();
        }
      }
    }
    if (k == kend && kend < a.iters) reason = DAVA_STOP_DROP;  // uniform
  #if DAVA_PHASE_TIMING
    ph_acc[kPhases - 1] = clock64() - ph_start;
    if (tid == 0 && a.phase_cycles)
      for (int i = 0; i < kPhases; ++i) a.phase_cycles[(size_t)b * kPhases + i] = ph_acc[i];
  #endif

    // ---- outputs ----
    __syncthreads();
    float* xo = a.x_out + (size_t)b * P;
    for (int i = tid; i < P; i += BLOCK) xo[i] = x[i];
    if (a.err_out) {
      float e2 = 0.f;
      ba_eval<false, false, false, false, false, RES, float, NW, PPT, GV>(L, x, nullptr, 0.f, obs, vis, nullptr, views, vpart, scratch, buf,
                                                     e2, unused);
      if (tid == 0) a.err_out[b] = e2;
    }
    if (a.status && tid == 0) {
      int32_t* st = a.status + (size_t)b * DAVA_STATUS_WORDS;
      st[0] = steps; st[1] = reason; st[2] = evals; st[3] = trials;
    }
    if (!a.queue) break;
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

// The evaluation the solve runs per line-search trial, as one launch (dava_ba_evaluate), with the solve's
// own layout per mode so that it measures -- and, as the generic path's closure, runs -- the same sweep:
//   LDS mode (P fits on-chip): x, d, gradient, observations and visibility staged in LDS, NW = 4 waves,
//     PPT = 1 when every point has a thread (C1-C3: each thread's point in registers across the views);
//   GV + XL (C5: 8 waves, one problem per CU): x, d and the gradient in LDS (3 Pv floats), observations
//     and visibility read in place, the packed pair sweep (two points per step) -- the in-solve trial;
//   GV without XL (an image past the LDS): x, d and the gradient in place in HBM.
// (Before r05 the GV form ran 4 waves with the vectors in HBM: at C5 VALUBusy 40% and 4.2x the
// algorithmic bytes from the per-view read-modify-write of the point gradients, profiles/r05_eval_*.)
template <bool GRAD, bool SLOPE, bool TRIAL, bool GV, int RES, bool XL = false, int NW = kWaves, int PPT = 0>
__global__ __launch_bounds__(kWave * NW) void ba_evaluate_kernel(EvalArgs a) {
  static_assert(!XL || GV, "XL is a global-vector-mode variant");
  constexpr int BLOCK = kWave * NW;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Layout L = a.L;
  const int P = L.P, M = L.M, N = L.N, Pv = a.Pv;
  const int b = blockIdx.x, tid = threadIdx.x;
  const LdsCarve cv = carve_lds(M, N, Pv, 0, GV, 0, XL, NW);
  const int MN = M * N;
  float* views = lds + cv.views;
  float* vpart = lds + cv.vpart;
  float* scratch = lds + cv.scratch;
  const float* x;
  const float* d;
  float* g;
  const float* obs;
  const uint8_t* vis;
  if (GV && !XL) {  // an image past the LDS: work on the caller's buffers in place
    x = a.x + (size_t)b * P;
    d = a.dir ? a.dir + (size_t)b * P : nullptr;
    g = a.grad ? a.grad + (size_t)b * P : nullptr;
    obs = a.obs + (size_t)b * 2 * MN;
    vis = a.vis + (size_t)b * MN;
  } else {
    float* xl = lds + cv.x;
    float* dl = lds + cv.d;
    float* gl = lds + (XL ? cv.ge : cv.g0);
    for (int i = tid; i < Pv; i += BLOCK) {
      xl[i] = i < P ? a.x[(size_t)b * P + i] : 0.f;
      dl[i] = (a.dir && i < P) ? a.dir[(size_t)b * P + i] : 0.f;
      gl[i] = 0.f;
    }
    if constexpr (GV) {  // XL: the scene stays in HBM, read in place as the solve does
      obs = a.obs + (size_t)b * 2 * MN;
      vis = a.vis + (size_t)b * MN;
    } else {
      float* ol = lds + cv.obs;
      uint8_t* vl = reinterpret_cast<uint8_t*>(lds) + cv.vis_bytes_off;
      for (int i = tid; i < 2 * MN; i += BLOCK) ol[i] = a.obs[(size_t)b * 2 * MN + i];
      for (int i = tid; i < MN; i += BLOCK) vl[i] = a.vis[(size_t)b * MN + i] ? 1 : 0;
      obs = ol; vis = vl;
    }
    x = xl; d = dl; g = gl;
  }
  __syncthreads();
  const float al = (TRIAL && a.alpha) ? a.alpha[b] : 0.f;
  int buf = 0;
  float E = 0.f, sl = 0.f;
  ba_eval<GRAD, SLOPE, TRIAL, false, false, RES, float, NW, PPT, GV>(L, x, d, al, obs, vis, g, views, vpart, scratch,
                                                                     buf, E, sl);
  if (tid == 0) {
    a.err[b] = E;
    if (SLOPE && a.slope) a.slope[b] = sl;
  }
  if (GRAD && a.grad && (!GV || XL))
    for (int i = tid; i < P; i += BLOCK) a.grad[(size_t)b * P + i] = g[i];
}

// ---- host API (everything below): left out of the microbenchmarks that include this file for its device
// passes alone (tools/micro/*.hip define DAVA_DEVICE_PASSES_ONLY), so they do not instantiate every solve kernel
#ifndef DAVA_DEVICE_PASSES_ONLY
static int check_scene(const DavaScene* s, bool need_data = true) {
  if (!s) return DAVA_ERR_INVALID_ARGUMENT;
  if (s->batch < 0 || s->num_views < 2 || s->num_points < 1) return DAVA_ERR_INVALID_ARGUMENT;
  const int P = 3 + 3 * s->num_points + 6 * (s->num_views - 1) + (s->distortion ? 5 : 0);
  if (s->num_parameters != P) return DAVA_ERR_INVALID_ARGUMENT;
  if (need_data && s->batch > 0 && (!s->observations || !s->visibility)) return DAVA_ERR_INVALID_ARGUMENT;
  if (s->residual != DAVA_RESIDUAL_SQUARED_REPROJECTION && s->residual != DAVA_RESIDUAL_RAY_ANGLE)
    return DAVA_ERR_INVALID_ARGUMENT;
  if (s->residual == DAVA_RESIDUAL_RAY_ANGLE && s->distortion) return DAVA_ERR_UNSUPPORTED;
  return DAVA_OK;
}

static size_t dense_hessian_bytes(const DavaScene* s) {
  const int P = s->num_parameters;
  return (size_t)s->batch * (size_t)P * (size_t)round_up(P, 32) * sizeof(float);
}

constexpr int kMaxLds = 160 * 1024;
constexpr int kSliceMinGroups = 6;
// GV mode, wide pass: rho_j, c_j move to the workspace slice when that keeps the XL image on-chip
// (see gv_scalar_stride)
static bool gv_scalars_slice(const DavaScene* s, int kcap) {
  const int Pv = round_up(s->num_parameters, 4);
  if (!wide_history_pass(Pv, kcap, true)) return false;
  // only rows of >= 6 float4 groups per thread have the slice form instantiated (wide_direction SLICE):
  // narrower rows leave room for the scalars beside their XL image at any cap
  if ((Pv / 4 + kWave * solve_waves(true) - 1) / (kWave * solve_waves(true)) < kSliceMinGroups) return false;
  if (debug_knob(kDbgGvScalarSlice) >= 0) return debug_knob(kDbgGvScalarSlice) > 0;  // tests
  const int M = s->num_views, N = s->num_points, nw = solve_waves(true);
  return carve_lds(M, N, Pv, kcap, true, 0, true, nw).total_bytes > kMaxLds &&
         carve_lds(M, N, Pv, 0, true, 0, true, nw).total_bytes <= kMaxLds;
}
static int lds_bytes_for(const DavaScene* s, int kcap = 0, bool gv = false, int lcap = 0, bool xl = false,
                         int nw = 0) {
  const int Pv = round_up(s->num_parameters, 4);
  const int kl = gv && xl && gv_scalars_slice(s, kcap) ? 0 : kcap;  // (the slice form exists with XL only)
  return carve_lds(s->num_views, s->num_points, Pv, kl, gv, lcap, xl, nw).total_bytes;
}

// Waves per LDS-mode workgroup (GV mode: always 8).  The register budget (256 VGPRs) holds two
// waves per SIMD, eight per CU, whatever the split, so the choice is how many waves share one
// problem: two waves while a history row is at most 2 x 64 float4 column groups (P <= 512), else
// four, so small problems do not pay for barriers and cross-wave sums over idle waves
// (interleaved A/B, profiles/r02_ab_waves.log: C2 +19%, 8192 two-view 64-point problems +49%,
// C3 -17% at two).  One wave per problem measured another +9% on the 64-point shape but put one
// K = 100 run-to-stagnation problem 3e-5 from the oracle (30x the reference's own 1-ulp
// sensitivity), so it stays opt-in.  DENSE keeps 4.  The kDbgSolveWaves override (1 | 2 | 4) is for
// A/B runs and tests.
static int lds_mode_waves(const DavaScene* s, int mode) {
  const long long w = debug_knob(kDbgSolveWaves);
  if (w == 1 || w == 2 || w == 4) return (int)w;
  if (mode != DAVA_HESSIAN_COMPACT) return 4;
  const int groups = (round_up(s->num_parameters, 4) / 4 + kWave - 1) / kWave;  // per-lane float4 groups at 1 wave
  return groups <= 2 ? 2 : 4;
}
static int solve_waves_for(const DavaScene* s, bool gv, int mode) {
  return gv ? solve_waves(true) : lds_mode_waves(s, mode);
}

// Global-vector mode when the all-in-LDS image would cost more than two workgroups
// per CU (e.g. C5: P = 12381 -> 446 KB of vectors per problem).
constexpr int kLdsModeBudget = 72 * 1024;
static bool use_gv(const DavaScene* s, int kcap = 0) {
  return debug_flag(kDbgForceGV) || lds_bytes_for(s, kcap, false) > kLdsModeBudget;
}
// GV mode: run the objective on LDS copies of x and d (carve_lds `xl`) whenever they fit
// beside the rest of the image.  The kDbgGVNoXL override forces the in-workspace variant (tests).
static bool use_xl(const DavaScene* s, int kcap, bool gv) {
  if (!gv || debug_flag(kDbgGVNoXL)) return false;
  return lds_bytes_for(s, kcap, true, 0, true) <= kMaxLds;
}
// the launch keeps rho_j, c_j in the workspace slice (bfgs_ba_solve_kernel SLICE)
static bool gv_slice_used(const DavaScene* s, int kcap) {
  return use_xl(s, kcap, true) && gv_scalars_slice(s, kcap);
}
static size_t gv_vector_bytes(const DavaScene* s, int kcap) {
  return (size_t)s->batch * (size_t)gv_slice_floats(round_up(s->num_parameters, 4), kcap, gv_slice_used(s, kcap)) *
         sizeof(float);
}

// History entries the COMPACT mode keeps: one per iteration k = 1 .. iterations-1, at most
// kMaxCompactEntries; a longer solve is HYBRID (fold_history: the dense matrix after the history fills).
// The kDbgCompactSwitch override lowers the capacity (tests: the switch at K = 30 instead of 1025).
constexpr int kMaxCompactEntries = 1024;
static int compact_capacity(const DavaSolverConfig* c) {
  const int need = c->iterations > 1 ? c->iterations - 1 : 1;
  const long long sw = debug_knob(kDbgCompactSwitch);
  const int cap = sw >= 1 && sw < kMaxCompactEntries ? (int)sw : kMaxCompactEntries;
  return min(need, cap);
}
static bool hybrid_solve(const DavaSolverConfig* c) {
  return c->hessian_mode == DAVA_HESSIAN_COMPACT && c->iterations - 1 > compact_capacity(c);
}

static size_t compact_history_bytes(const DavaScene* s, const DavaSolverConfig* c) {
  return (size_t)s->batch * 2 * (size_t)compact_capacity(c) * (size_t)round_up(s->num_parameters, 4) * sizeof(float);
}

// COMPACT, LDS mode, single-pass products: how many of the oldest history entries to keep
// on-chip.  Default: whatever fits beside the problem image without lowering the number of
// workgroups a CU holds at the register limit (4 SIMDs x kSolveWavesPerEU waves / nw:
// two 4-wave workgroups of 80 KiB, or four 2-wave workgroups of 40 KiB); the kDbgLdsHistory override
// sets the count (A/B and tests; 0 = all in HBM; values past one workgroup's LDS are clamped).
static int lds_history_entries(const DavaScene* s, int kcap, bool gv, int nw) {
  const int Pv = round_up(s->num_parameters, 4);
  if (gv || kcap <= 0 || (Pv / 4 + kWave - 1) / kWave > 4) return 0;
  const int base = lds_bytes_for(s, kcap, false, 0, false, nw);
  const int per = 2 * Pv * (int)sizeof(float);
  int per_cu = 4 * kSolveWavesPerEU / nw;  // workgroups per CU at the register limit
  if (debug_knob(kDbgWgPerCu) > 0) per_cu = (int)debug_knob(kDbgWgPerCu);  // A/B: LDS budget = 160 KB / this
  int n = (kMaxLds / per_cu - base) / per;
  // rows of <= 2 groups per lane consume the on-chip entries in batches, entries dealt round-robin to the
  // waves: a multiple of the waves keeps the waves' batches equal (C2 at K = 100: 7 entries measured -1.2%
  // against 6; the C1 shape 18 against 17 also -1.2%, so for these short rows an on-chip entry past the
  // first few is worth little either way, profiles/r05_ab_lds_coefficients.log)
  if ((Pv / 4 + kWave - 1) / kWave <= 2) n -= n % nw;
  if (debug_knob(kDbgLdsHistory) >= 0) n = (int)debug_knob(kDbgLdsHistory);
  n = min(n, (kMaxLds - base) / per);
  return max(0, min(n, kcap));
}

}  // namespace dava

using namespace dava;

// ---- debug overrides (dava_debug.hpp): set only through the two calls below, never from the environment ----
namespace dava {
static long long g_debug_knobs[kDbgKnobs] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
static const char* const kDebugKnobNames[kDbgKnobs] = {
    "FORCE_GV", "GV_NO_XL", "SOLVE_WAVES", "WG_PER_CU", "LDS_HISTORY", "STAGGER", "STAGGER_LEVELS",
    "NO_PPT", "NO_QUEUE", "ADJ_GV_WAVES", "ADJ_FORCE_GV", "ADJ_LDS_ENTRIES", "ADJ_GD_HBM",
    "COMPACT_SWITCH", "GV_SCALAR_SLICE", "ADJ_SC_GLOBAL"};
long long debug_knob(int k) { return k >= 0 && k < kDbgKnobs ? g_debug_knobs[k] : -1; }
}  // namespace dava

extern "C" int dava_debug_set_override(const char* name, int64_t value) {
  if (!name) return DAVA_ERR_INVALID_ARGUMENT;
  for (int k = 0; k < kDbgKnobs; ++k)
    if (strcmp(name, kDebugKnobNames[k]) == 0) {
      g_debug_knobs[k] = value < 0 ? -1 : value;
      return DAVA_OK;
    }
  return DAVA_ERR_INVALID_ARGUMENT;
}

extern "C" void dava_debug_clear_overrides(void) {
  for (int k = 0; k < kDbgKnobs; ++k) g_debug_knobs[k] = -1;
}

// Bytes of the solve's state (vectors in GV mode + inverse-Hessian state); the work-queue
// counter follows at that offset, in the last kQueueBytes of the workspace.
constexpr size_t kQueueBytes = 256;
static size_t solve_state_bytes(const DavaScene* scene, const DavaSolverConfig* config) {
  const int kcap = config->hessian_mode == DAVA_HESSIAN_COMPACT ? compact_capacity(config) : 0;
  const size_t vec = use_gv(scene, kcap) ? gv_vector_bytes(scene, kcap) : 0;
  if (config->hessian_mode == DAVA_HESSIAN_DENSE) return vec + dense_hessian_bytes(scene);
  // HYBRID: the dense matrices follow the histories (SolveArgs::hess_dense)
  return vec + compact_history_bytes(scene, config) + (hybrid_solve(config) ? dense_hessian_bytes(scene) : 0);
}

extern "C" size_t dava_ba_solve_workspace_bytes(const DavaScene* scene, const DavaSolverConfig* config) {
  if (check_scene(scene, false) != DAVA_OK || !config) return 0;
  if (config->hessian_mode != DAVA_HESSIAN_DENSE && config->hessian_mode != DAVA_HESSIAN_COMPACT) return 0;
  return solve_state_bytes(scene, config) + kQueueBytes;
}

extern "C" int dava_ba_solve_plan(const DavaScene* scene, const DavaSolverConfig* config, DavaSolvePlan* plan) {
  const int st = check_scene(scene, false);
  if (st != DAVA_OK) return st;
  if (!config || !plan || config->iterations < 0) return DAVA_ERR_INVALID_ARGUMENT;
  const int mode = config->hessian_mode;
  if (mode != DAVA_HESSIAN_DENSE && mode != DAVA_HESSIAN_COMPACT) return DAVA_ERR_INVALID_ARGUMENT;
  const int kcap = mode == DAVA_HESSIAN_COMPACT ? compact_capacity(config) : 0;
  const bool gv = use_gv(scene, kcap);
  const int nw = solve_waves_for(scene, gv, mode);
  const int lcap = mode == DAVA_HESSIAN_COMPACT ? lds_history_entries(scene, kcap, gv, nw) : 0;
  plan->global_vectors = gv ? 1 : 0;
  plan->workgroup_threads = kWave * nw;
  plan->lds_bytes = lds_bytes_for(scene, kcap, gv, lcap, use_xl(scene, kcap, gv), nw);
  plan->lds_history_entries = lcap;
  return plan->lds_bytes > kMaxLds ? DAVA_ERR_UNSUPPORTED : DAVA_OK;
}

constexpr int kStaggerCycles = 20000;  // ~8 us at the shader clock; one C2 iteration is ~47 us

template <int MODE, bool GV, int RES, bool XL, int PPT, int NW, bool SLICE = false>
static void launch_solve_ppt(const SolveArgs& a, int B, int lds, hipStream_t s) {
  const auto kernel = bfgs_ba_solve_kernel<MODE, GV, RES, XL, PPT, NW, SLICE>;
  constexpr int threads = kWave * NW;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  int grid = B;
  SolveArgs args = a;
  int slots = 0;  // workgroups resident at once (host queries only; nothing synchronises)
  {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) == hipSuccess && per_cu > 0 &&
        cus > 0)
      slots = per_cu * cus;
  }
  // stagger only a launch whose problems all run at once (one round, B <= slots)
  args.stagger = slots > 0 && B <= slots && B > 1 ? kStaggerCycles : 0;
  args.stagger_levels = 1;
  if (debug_knob(kDbgStagger) >= 0) args.stagger = (int)debug_knob(kDbgStagger);  // A/B (cycles)
  if (debug_knob(kDbgStaggerLevels) >= 1) args.stagger_levels = (int)debug_knob(kDbgStaggerLevels);
  if (args.queue) {  // one workgroup per resident slot
    if (slots > 0) grid = min(B, slots);
    // The hardware already refills a slot as soon as its workgroup retires, but only from its
    // own XCD's share of the grid (workgroups are dealt round-robin over the 8 XCDs): the
    // queue pays where per-problem work is uneven -- stopping rules active, or few problems
    // per slot so one long line search decides an XCD's finish (C2: +10%, C3 to convergence:
    // +4.5%).  With fixed K and >= 8 problems per slot (C3: 16) it measured -1%: plain grid.
    const bool fixed_k = !(args.thr >= 0.f) && !(args.min_step >= 0.f);
    if (grid == B || (fixed_k && B >= 8 * grid)) {
      args.queue = nullptr;
      grid = B;
    }
  }
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), lds, s, args);
}

// Points per thread held in registers by the objective: one for the LDS-mode kernels (C1-C3:
// N <= 256; C3 +12% over re-reading x, d and the gradient from LDS per view).  Larger N, GV
// mode and the kDbgNoPPT override take the re-reading variant: eight points per thread at C5 spill
// (1 KB of scratch per lane) and ran 42% slower.
// One-wave workgroups (one problem per wave) hold two points per lane (N <= 128).
template <bool GV, bool XL, int NW>
constexpr int kRegisterPoints = GV ? 0 : (NW == 1 ? 2 : 1);

template <int MODE, bool GV, int RES, bool XL, int NW, bool SLICE = false>
static void launch_solve_nw(const SolveArgs& a, int B, int lds, hipStream_t s) {
  constexpr int R = kRegisterPoints<GV, XL, NW>;
  if constexpr (SLICE)  // (GV: no points in registers)
    launch_solve_ppt<MODE, GV, RES, XL, 0, NW, SLICE>(a, B, lds, s);
  else if (R > 0 && a.L.N <= R * kWave * NW && !debug_flag(kDbgNoPPT))
    launch_solve_ppt<MODE, GV, RES, XL, R, NW>(a, B, lds, s);
  else
    launch_solve_ppt<MODE, GV, RES, XL, 0, NW>(a, B, lds, s);
}

template <int MODE, bool GV, int RES, bool XL, bool SLICE = false>
static void launch_solve_res(const SolveArgs& a, int B, int lds, hipStream_t s, int nw) {
  if constexpr (GV) launch_solve_nw<MODE, GV, RES, XL, solve_waves(true), SLICE>(a, B, lds, s);
  else if (nw == 1) launch_solve_nw<MODE, GV, RES, XL, 1>(a, B, lds, s);
  else if (nw == 2) launch_solve_nw<MODE, GV, RES, XL, 2>(a, B, lds, s);
  else launch_solve_nw<MODE, GV, RES, XL, 4>(a, B, lds, s);
}

template <int MODE, bool GV, bool XL = false, bool SLICE = false>
static void launch_solve(const SolveArgs& a, int B, int lds, hipStream_t s, int residual, int nw) {
  if (residual == DAVA_RESIDUAL_RAY_ANGLE) launch_solve_res<MODE, GV, DAVA_RESIDUAL_RAY_ANGLE, XL, SLICE>(a, B, lds, s, nw);
  else launch_solve_res<MODE, GV, DAVA_RESIDUAL_SQUARED_REPROJECTION, XL, SLICE>(a, B, lds, s, nw);
}

// A recording solve (the tape of dava_tape.hpp) needs COMPACT mode and P <= 14336: the adjoint kernel
// runs P <= 1024 with its O(P) vectors in LDS and larger P (the forward's global-vector mode, e.g. C5)
// with them in its workspace, both over rows of at most 14 float4 groups per thread.  A GV-mode
// recording also needs the forward's wide single-pass history products (the ones that write the tape).
constexpr int kTapeMaxParameters = 14336;
static bool tape_supported(const DavaScene* scene, const DavaSolverConfig* config) {
  if (config->hessian_mode != DAVA_HESSIAN_COMPACT || config->iterations < 1) return false;
  const int kcap = compact_capacity(config);
  if (hybrid_solve(config) || scene->num_parameters > kTapeMaxParameters) return false;
  const bool gv = use_gv(scene, kcap);
  return !gv || wide_history_pass(round_up(scene->num_parameters, 4), kcap, true);
}
static TapeLayout solve_tape_layout(const DavaScene* scene, const DavaSolverConfig* config) {
  const int kcap = compact_capacity(config);
  const int Pv = round_up(scene->num_parameters, 4);
  return tape_layout(scene->batch, scene->num_parameters, config->iterations, use_gv(scene, kcap) ? gv_slice_floats(Pv, kcap, gv_slice_used(scene, kcap)) : 0);
}

static int solve_impl(const DavaScene* scene, const DavaSolverConfig* config, const float* x0, float* x_out,
                      float* error_out, int32_t* status_out, void* workspace, size_t workspace_bytes, bool record,
                      void* stream) {
  int st = check_scene(scene);
  if (st != DAVA_OK) return st;
  if (!config || config->iterations < 0 || config->max_line_search_trials < 0) return DAVA_ERR_INVALID_ARGUMENT;
  if (!(config->drop_path_p >= 0.f && config->drop_path_p <= 1.f)) return DAVA_ERR_INVALID_ARGUMENT;
  const int mode = config->hessian_mode;
  if (mode != DAVA_HESSIAN_DENSE && mode != DAVA_HESSIAN_COMPACT) return DAVA_ERR_INVALID_ARGUMENT;
  if (record && !tape_supported(scene, config)) return DAVA_ERR_UNSUPPORTED;
  if (scene->batch == 0) return DAVA_OK;
  if (!x0 || !x_out) return DAVA_ERR_INVALID_ARGUMENT;
  const int kcap = mode == DAVA_HESSIAN_COMPACT ? compact_capacity(config) : 0;
  const bool hybrid = hybrid_solve(config);
  const bool gv = use_gv(scene, kcap);
  const bool xl = use_xl(scene, kcap, gv);
  const int nw = solve_waves_for(scene, gv, mode);
  // recording keeps every history entry in HBM (the adjoint reads them back; bitwise the same run)
  const int lcap = mode == DAVA_HESSIAN_COMPACT ? lds_history_entries(scene, kcap, gv, nw) : 0;
  const int lds = lds_bytes_for(scene, kcap, gv, lcap, xl, nw);
  if (lds > kMaxLds) return DAVA_ERR_UNSUPPORTED;
  const size_t vec = gv ? gv_vector_bytes(scene, kcap) : 0;
  const TapeLayout tl = solve_tape_layout(scene, config);
  const size_t need = record ? tl.queue_byte : solve_state_bytes(scene, config);
  const bool uses_ws = record || gv || (mode == DAVA_HESSIAN_DENSE ? config->iterations > 2 : config->iterations > 1);
  if (uses_ws && (!workspace || workspace_bytes < need)) return DAVA_ERR_WORKSPACE;
  // the work queue needs its counter in the workspace's tail (dava_ba_solve_workspace_bytes
  // includes it); a workspace sized without it runs one workgroup per problem instead
  const bool queue = workspace && workspace_bytes >= need + kQueueBytes && !debug_flag(kDbgNoQueue);
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
  a.vecs = gv ? static_cast<float*>(workspace) : nullptr;
  a.scal_slice = xl && gv_scalars_slice(scene, kcap) ? 1 : 0;
  a.vstride = gv_slice_floats(round_up(scene->num_parameters, 4), kcap, a.scal_slice != 0);
  a.kcap_lds = a.scal_slice ? 0 : kcap;
  a.hess = workspace ? reinterpret_cast<float*>(static_cast<char*>(workspace) + vec) : nullptr;
  a.hess_dense = hybrid && a.hess ? a.hess + compact_history_bytes(scene, config) / sizeof(float) : nullptr;
  a.c1 = config->sufficient_decrease;
  a.c2 = config->curvature;
  a.thr = config->error_threshold;
  a.min_step = config->minimum_step;
  a.iters = config->iterations;
  a.max_trials = config->max_line_search_trials;
  a.strong = config->strong_wolfe;
  a.mode = mode;
  a.kcap = kcap;
  a.lcap = lcap;
  a.phase_cycles = nullptr;
  a.stagger = 0;
  a.stagger_levels = 1;
  a.drop_p = config->drop_path_p;
  a.drop_seed = ((unsigned long long)config->drop_seed_hi << 32) | config->drop_seed_lo;
  a.second_last = config->return_second_last ? 1 : 0;
  a.queue = queue ? reinterpret_cast<int*>(static_cast<char*>(workspace) + need) : nullptr;
  a.tape_x = a.tape_g = a.tape_s = nullptr;
  a.tape_T = tl.T;
  if (record) {
    float* t = static_cast<float*>(workspace);
    a.hess = t + tl.hist;
    a.tape_x = t + tl.x;
    a.tape_g = t + tl.g;
    a.tape_s = t + tl.scal;
    a.vecs = gv ? t + tl.vecs : nullptr;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  // (a recording zeroes its whole queue tail: the tape tensor handed back includes it)
  if (record && workspace_bytes >= need + kQueueBytes) {
    if (hipMemsetAsync(static_cast<char*>(workspace) + need, 0, kQueueBytes, s) != hipSuccess) return DAVA_ERR_LAUNCH;
  } else if (queue && hipMemsetAsync(a.queue, 0, sizeof(int), s) != hipSuccess) {
    return DAVA_ERR_LAUNCH;
  }
  // the tape's scalar rows have slots no solve writes (rho / c of step K, padding): zero them so a
  // tape is a deterministic function of the inputs, byte for byte (B x T floats, small)
  if (record && hipMemsetAsync(a.tape_s, 0, (size_t)scene->batch * tl.T * sizeof(float), s) != hipSuccess)
    return DAVA_ERR_LAUNCH;
#if DAVA_PHASE_TIMING
  const size_t ph_bytes = (size_t)scene->batch * kPhases * sizeof(unsigned long long);
  if (hipMalloc(&a.phase_cycles, ph_bytes) != hipSuccess) return DAVA_ERR_LAUNCH;
  (void)hipMemsetAsync(a.phase_cycles, 0, ph_bytes, s);
  {
    const unsigned long long zero[kEvalSections] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_eval_cycles), zero, sizeof(zero));
  }
#endif
  if (mode == DAVA_HESSIAN_DENSE) {
    if (xl) launch_solve<DAVA_HESSIAN_DENSE, true, true>(a, scene->batch, lds, s, scene->residual, nw);
    else if (gv) launch_solve<DAVA_HESSIAN_DENSE, true>(a, scene->batch, lds, s, scene->residual, nw);
    else launch_solve<DAVA_HESSIAN_DENSE, false>(a, scene->batch, lds, s, scene->residual, nw);
  } else if (hybrid) {
    if (xl && a.scal_slice) launch_solve<kHybrid, true, true, true>(a, scene->batch, lds, s, scene->residual, nw);
    else if (xl) launch_solve<kHybrid, true, true>(a, scene->batch, lds, s, scene->residual, nw);
    else if (gv) launch_solve<kHybrid, true>(a, scene->batch, lds, s, scene->residual, nw);
    else launch_solve<kHybrid, false>(a, scene->batch, lds, s, scene->residual, nw);
  } else {
    if (xl && a.scal_slice) launch_solve<DAVA_HESSIAN_COMPACT, true, true, true>(a, scene->batch, lds, s, scene->residual, nw);
    else if (xl) launch_solve<DAVA_HESSIAN_COMPACT, true, true>(a, scene->batch, lds, s, scene->residual, nw);
    else if (gv) launch_solve<DAVA_HESSIAN_COMPACT, true>(a, scene->batch, lds, s, scene->residual, nw);
    else launch_solve<DAVA_HESSIAN_COMPACT, false>(a, scene->batch, lds, s, scene->residual, nw);
  }
  const bool launched = hipGetLastError() == hipSuccess;
#if DAVA_PHASE_TIMING
  {
    unsigned long long* h = static_cast<unsigned long long*>(malloc(ph_bytes));
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h, a.phase_cycles, ph_bytes, hipMemcpyDeviceToHost);
    (void)hipFree(a.phase_cycles);
    static const char* names[kPhases] = {"eval_at_x", "history", "direction", "trial_evals", "search_logic", "step",
                                         "total"};
    double avg[kPhases] = {0};
    for (int b = 0; b < scene->batch; ++b)
      for (int i = 0; i < kPhases; ++i) avg[i] += (double)h[(size_t)b * kPhases + i] / scene->batch;
    fprintf(stderr, "[dava phase cycles / problem]");
    for (int i = 0; i < kPhases; ++i) fprintf(stderr, " %s=%.0f (%.1f%%)", names[i], avg[i], 100.0 * avg[i] / avg[kPhases - 1]);
    fprintf(stderr, "\n");
    // per-problem distribution (a launch lasts as long as its slowest problems): p50 / p99 / max per phase
    {
      std::vector<unsigned long long> col(scene->batch);
      fprintf(stderr, "[dava phase cycles distribution]");
      for (int i = 0; i < kPhases; ++i) {
        for (int b = 0; b < scene->batch; ++b) col[b] = h[(size_t)b * kPhases + i];
        std::sort(col.begin(), col.end());
        const size_t n = col.size();
        fprintf(stderr, " %s=p50:%llu,p99:%llu,max:%llu", names[i], col[n / 2], col[std::min(n - 1, (size_t)(0.99 * n))],
                col[n - 1]);
      }
      fprintf(stderr, "\n");
    }
    unsigned long long ev[kEvalSections] = {};
    (void)hipMemcpyFromSymbol(ev, HIP_SYMBOL(g_eval_cycles), sizeof(ev));
    static const char* enames[kEvalSections] = {"view_constants", "point_sums", "setup", "pair_sweep", "final_sums",
                                                "gradient_assembly"};
    fprintf(stderr, "[dava objective cycles / problem]");
    for (int i = 0; i < kEvalSections; ++i) fprintf(stderr, " %s=%.0f", enames[i], (double)ev[i] / scene->batch);
    fprintf(stderr, "\n");
    free(h);
  }
#endif
  return launched ? DAVA_OK : DAVA_ERR_LAUNCH;
}

extern "C" int dava_ba_solve(const DavaScene* scene, const DavaSolverConfig* config, const float* x0,
                             float* x_out, float* error_out, int32_t* status_out, void* workspace,
                             size_t workspace_bytes, void* stream) {
  return solve_impl(scene, config, x0, x_out, error_out, status_out, workspace, workspace_bytes, false, stream);
}

extern "C" size_t dava_ba_solve_tape_bytes(const DavaScene* scene, const DavaSolverConfig* config) {
  if (check_scene(scene, false) != DAVA_OK || !config || !tape_supported(scene, config)) return 0;
  return solve_tape_layout(scene, config).total_bytes;
}

extern "C" int dava_ba_solve_record(const DavaScene* scene, const DavaSolverConfig* config, const float* x0,
                                    float* x_out, float* error_out, int32_t* status_out, void* tape,
                                    size_t tape_bytes, void* stream) {
  if (!status_out && scene && scene->batch > 0) return DAVA_ERR_INVALID_ARGUMENT;  // the adjoint needs the steps
  return solve_impl(scene, config, x0, x_out, error_out, status_out, tape, tape_bytes, true, stream);
}

template <bool G, bool S, bool T, bool GV, int RES, bool XL, int NW, int PPT>
static void launch_eval_form(const EvalArgs& a, int B, int lds, hipStream_t s) {
  const auto kernel = ba_evaluate_kernel<G, S, T, GV, RES, XL, NW, PPT>;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(kernel, dim3(B), dim3(kWave * NW), lds, s, a);
}

// form: 0 = LDS mode, PPT 0 | 1 = LDS mode, a point per thread in registers | 2 = GV + XL (8 waves) |
// 3 = GV in place (8 waves)
template <bool G, bool S, bool T, int RES>
static void launch_eval_res(const EvalArgs& a, int B, int lds, hipStream_t s, int form) {
  constexpr int GVW = solve_waves(true);
  if (form == 3) launch_eval_form<G, S, T, true, RES, false, GVW, 0>(a, B, lds, s);
  else if (form == 2) launch_eval_form<G, S, T, true, RES, true, GVW, 0>(a, B, lds, s);
  else if (form == 1) launch_eval_form<G, S, T, false, RES, false, kWaves, 1>(a, B, lds, s);
  else launch_eval_form<G, S, T, false, RES, false, kWaves, 0>(a, B, lds, s);
}

template <bool G, bool S, bool T>
static void launch_eval(const EvalArgs& a, int B, int lds, hipStream_t s, int form, int res) {
  if (res == DAVA_RESIDUAL_RAY_ANGLE) launch_eval_res<G, S, T, DAVA_RESIDUAL_RAY_ANGLE>(a, B, lds, s, form);
  else launch_eval_res<G, S, T, DAVA_RESIDUAL_SQUARED_REPROJECTION>(a, B, lds, s, form);
}

extern "C" int dava_ba_evaluate(const DavaScene* scene, const float* x, const float* direction, const float* alpha,
                                float* error_out, float* grad_out, float* slope_out, void* stream) {
  int st = check_scene(scene);
  if (st != DAVA_OK) return st;
  if (scene->batch == 0) return DAVA_OK;
  if (!x || !error_out) return DAVA_ERR_INVALID_ARGUMENT;
  if (slope_out && !direction) return DAVA_ERR_INVALID_ARGUMENT;
  const bool gv = use_gv(scene);
  const int gvw = solve_waves(true);
  const bool xl = gv && !debug_flag(kDbgGVNoXL) && lds_bytes_for(scene, 0, true, 0, true, gvw) <= kMaxLds;
  const int form = gv ? (xl ? 2 : 3) : (scene->num_points <= kBlock && !debug_flag(kDbgNoPPT) ? 1 : 0);
  const int lds = gv ? lds_bytes_for(scene, 0, true, 0, xl, gvw) : lds_bytes_for(scene, 0, false);
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
  if (G && S && T) launch_eval<true, true, true>(a, B, lds, s, form, scene->residual);
  else if (G && S) launch_eval<true, true, false>(a, B, lds, s, form, scene->residual);
  else if (G && T) launch_eval<true, false, true>(a, B, lds, s, form, scene->residual);
  else if (G) launch_eval<true, false, false>(a, B, lds, s, form, scene->residual);
  else if (S && T) launch_eval<false, true, true>(a, B, lds, s, form, scene->residual);
  else if (S) launch_eval<false, true, false>(a, B, lds, s, form, scene->residual);
  else if (T) launch_eval<false, false, true>(a, B, lds, s, form, scene->residual);
  else launch_eval<false, false, false>(a, B, lds, s, form, scene->residual);
  return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH;
}

#else
}  // namespace dava
#endif  // DAVA_DEVICE_PASSES_ONLY
