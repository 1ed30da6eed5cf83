/*
 * dava_ba.h -- C ABI of the MI355X (gfx950) batched BFGS bundle-adjustment solver.
 *
 * This is the drop-in boundary for the one hot path of
 * jskinn/deep-attention-visual-odometry that this project replaces: the
 * `autograd_solvers/` BFGS loop + strong-Wolfe line search evaluated on a
 * multi-view pinhole (+ Brown-Conrady) reprojection objective.  The reference
 * is pure PyTorch (no FFI exists there); each entry point below names the
 * reference interface it replaces.  The Python mirror of the reference API
 * (deep_attention_visual_odometry_amd.autograd_solvers) binds these symbols
 * through ctypes; INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer (HBM) unless stated otherwise.
 *    Struct arguments themselves are host memory.
 *  - `stream` is a hipStream_t (NULL = default stream); all work is
 *    enqueued asynchronously on it, nothing synchronises the host, and no
 *    entry point allocates memory (caller supplies the workspace), so every
 *    call is graph-capturable.
 *  - Functional ownership, like the reference (`bfgs_solver.py:197`):
 *    inputs are never written; outputs may not alias inputs unless stated.
 *  - Return value: DAVA_OK or a DAVA_ERR_* code; nothing throws across the ABI.
 *    dava_status_string() turns a code into text.
 *  - fp32 throughout the fused solver (the reference's dtype for the BA path);
 *    the generic BFGS building blocks come in _f32 and _f64 flavours because
 *    the reference's own unit tests drive them in float64.
 */
#ifndef DAVA_BA_H
#define DAVA_BA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DAVA_ABI_VERSION 4

enum DavaStatus {
  DAVA_OK = 0,
  DAVA_ERR_INVALID_ARGUMENT = 1, /* bad sizes / null pointers / P mismatch  */
  DAVA_ERR_WORKSPACE = 2,        /* workspace missing or too small          */
  DAVA_ERR_LAUNCH = 3,           /* HIP launch failure                      */
  DAVA_ERR_UNSUPPORTED = 4       /* shape outside what this build supports  */
};

/* Representation of the inverse Hessian inside the fused solver. */
enum DavaHessianMode {
  DAVA_HESSIAN_DENSE = 0,  /* dense P x P fp32 per problem in HBM (the reference's data structure) */
  DAVA_HESSIAN_COMPACT = 1 /* exact rank-2 update history (s_j, H_{j-1} y_j): same math, O(kP) bytes;
                            * past 1024 updates (iterations > 1025) a problem that is still running
                            * folds its history into the dense matrix once and continues DENSE */
};

/* Why a problem stopped (bfgs_solver.py:143-145, :203-207). */
enum DavaStopReason {
  DAVA_STOP_ITERATIONS = 0, /* ran `iterations` steps                 */
  DAVA_STOP_ERROR = 1,      /* error <= error_threshold (or NaN)      */
  DAVA_STOP_STEP = 2,       /* ||step|| <= minimum_step (or NaN)      */
  DAVA_STOP_DROP = 3        /* training-mode drop path (drop_path_p)  */
};

/* Per-(view, point) residual summed into the objective.
 *  SQUARED_REPROJECTION: vis * |pi(X) - obs|^2  -- the benchmark objective.
 *  RAY_ANGLE: vis * angle(ray(obs), p) with ray(obs) = (u - cx, v - cy, elu(f) + 1) and p the
 *    camera-relative point: the error CalibrationNetwork minimises (calibration_network.py:58-67,
 *    geometry/homogeneous_projection.py:21-44, geometry/projective_plane_angle_distance.py:20-64).
 *    Pinhole only (distortion must be 0).                                                      */
enum DavaResidual {
  DAVA_RESIDUAL_SQUARED_REPROJECTION = 0,
  DAVA_RESIDUAL_RAY_ANGLE = 1
};

/* A batch of independent calibration problems.
 * Parameter layout per problem (calibration_pinhole_camera_model.py:33-75):
 *   [f, cx, cy | X_0..X_{N-1} (xyz) | t_1..t_{M-1} | w_1..w_{M-1} | k1 k2 k3 p1 p2 (if distortion)]
 * num_parameters must equal 3 + 3N + 6(M-1) + 5*distortion.                     */
typedef struct DavaScene {
  int32_t batch;               /* B >= 0                               */
  int32_t num_views;           /* M >= 2                               */
  int32_t num_points;          /* N >= 1                               */
  int32_t distortion;          /* 0 = pinhole, 1 = + Brown-Conrady     */
  int32_t num_parameters;      /* P                                    */
  const float* observations;   /* (B, M, N, 2) fp32                    */
  const uint8_t* visibility;   /* (B, M, N) 0/1                        */
  int32_t residual;            /* DavaResidual                         */
} DavaScene;

/* Mirrors the eval-mode BFGSSolver constructor (bfgs_solver.py:49-78). */
typedef struct DavaSolverConfig {
  float sufficient_decrease;      /* c1, default 1e-4                          */
  float curvature;                /* c2, default 0.9                           */
  float error_threshold;          /* default 1e-4                              */
  float minimum_step;             /* default 1e-8                              */
  int32_t iterations;             /* default 1000                              */
  int32_t max_line_search_trials; /* 1000 in wolfe_conditions.py:116           */
  int32_t strong_wolfe;           /* 1 (bfgs_solver.py:189)                    */
  int32_t hessian_mode;           /* DavaHessianMode                           */
  /* Training mode's drop path (bfgs_solver.py:121-125): at the top of every iteration a problem
   * keeps updating only if a uniform draw in [0, 1) exceeds drop_path_p, else it stops for good
   * (DAVA_STOP_DROP).  Draws are counter-based (seed, problem, iteration): the same seed gives the
   * same schedule on any launch shape.  0 = eval mode (the default).                           */
  float drop_path_p;
  uint32_t drop_seed_lo, drop_seed_hi;
  /* Training mode's return_second_last (bfgs_solver.py:196-212): a problem that stops by the
   * minimum-step rule returns the parameters BEFORE its last step (x_k, not x_{k+1}); every other
   * stop returns the current ones, as without it.  0 = off (the default).  The reference's own
   * masked_scatter also moves rows between problems when a problem stops this way while a later
   * problem of the batch continues; the caller detects that case from the status words (the Python
   * module then runs the reference's loop instead).                                */
  int32_t return_second_last;
} DavaSolverConfig;

/* Per-problem status written by dava_ba_solve: int32 (B, 4) =
 * {steps taken, DavaStopReason, objective evaluations, line-search trials}. */
#define DAVA_STATUS_WORDS 4

/* Bytes of device workspace dava_ba_solve needs for this scene/config: the solve's state
 * (inverse-Hessian representation; O(P) vectors for large P) followed by a 256-byte
 * work-queue counter.  A workspace of this size lets the launch run one workgroup per
 * resident slot, each taking the next problem when it finishes one (problems that stop
 * early free their slot); a workspace without the counter's 256 bytes still works, one
 * workgroup per problem. */
size_t dava_ba_solve_workspace_bytes(const DavaScene* scene, const DavaSolverConfig* config);

/* How dava_ba_solve runs a scene/config (host-only query, no device needed): lets a caller
 * account for the HBM traffic of the launch (benchmarks, roofline) without re-deriving it. */
typedef struct DavaSolvePlan {
  int32_t global_vectors;      /* 1: the O(P) state lives in the workspace (large P), 0: in LDS  */
  int32_t workgroup_threads;   /* threads of the one workgroup that solves a problem            */
  int32_t lds_bytes;           /* dynamic LDS per workgroup                                     */
  int32_t lds_history_entries; /* COMPACT: the oldest history entries kept on-chip, never in HBM */
} DavaSolvePlan;
int dava_ba_solve_plan(const DavaScene* scene, const DavaSolverConfig* config, DavaSolvePlan* plan_out);

/* The whole eval-mode solve, one launch.
 * Replaces BFGSSolver.forward(parameters, error_function)
 * (autograd_solvers/bfgs_solver.py:80-215) with error_function = the objective
 * over `scene` (its `residual`), including line_search_wolfe_conditions
 * (autograd_solvers/line_search/wolfe_conditions.py:23-239, strong=True).
 *   x0        (B, P) fp32 initial guess
 *   x_out     (B, P) fp32 result (may alias x0)
 *   error_out (B)    fp32 objective at x_out, or NULL
 *   status_out(B, 4) int32, or NULL                                         */
int dava_ba_solve(const DavaScene* scene, const DavaSolverConfig* config, const float* x0, float* x_out,
                  float* error_out, int32_t* status_out, void* workspace, size_t workspace_bytes,
                  void* stream);

/* ---- differentiating THROUGH the fused solve (the reference's create_graph mode,
 * bfgs_solver.py:85, :133-135, :213-215: every iteration's gradient kept in the graph, the
 * line search's step size a constant) without a dense (B, P, P) inverse Hessian per iteration.
 * A recording solve keeps a tape in HBM (x_k, g_k, the compact history rows, step sizes; see
 * csrc/dava_tape.hpp); the adjoint replays it backwards, one workgroup per problem.
 * COMPACT mode only, iterations <= 1025 and P <= 14336: shapes whose O(P) state fits the LDS
 * (C1-C3) keep it there, larger ones (the forward's global-vector mode, e.g. C5 with P = 12381)
 * keep it in the adjoint's workspace.  Otherwise the size queries return 0 and the calls
 * DAVA_ERR_UNSUPPORTED. */

/* Bytes of the tape (including the work-queue counter's 256 bytes), or 0 if unsupported. */
size_t dava_ba_solve_tape_bytes(const DavaScene* scene, const DavaSolverConfig* config);

/* dava_ba_solve (bitwise the same x_out, error_out and status_out) that also writes the tape.
 * status_out is required (the adjoint reads the steps each problem took). */
int dava_ba_solve_record(const DavaScene* scene, const DavaSolverConfig* config, const float* x0, float* x_out,
                         float* error_out, int32_t* status_out, void* tape, size_t tape_bytes, void* stream);

/* Device workspace of dava_ba_solve_backward, or 0 if unsupported. */
size_t dava_ba_solve_backward_workspace_bytes(const DavaScene* scene, const DavaSolverConfig* config);

/* History entries (s_j, w_j) the adjoint keeps in LDS for its whole reverse sweep (the oldest
 * ones, as many as one workgroup's LDS leaves room for, at most iterations - 1).  The library
 * reads no environment; only the test/A-B override dava_debug_set_override("ADJ_LDS_ENTRIES", n)
 * caps it.  Informational: for byte models. */
int dava_ba_solve_backward_lds_entries(const DavaScene* scene, const DavaSolverConfig* config);

/* Vector-Jacobian product of the recorded solve: given x_out_grad = dL/dx_out (B, P), writes
 *   x0_grad            (B, P)        dL/dx0
 *   observations_grad  (B, M, N, 2)  dL/dobs (or NULL)
 * scene/config/status must be those of the recording call, the tape unmodified. */
int dava_ba_solve_backward(const DavaScene* scene, const DavaSolverConfig* config, const void* tape,
                           size_t tape_bytes, const int32_t* status, const float* x_out_grad, float* x0_grad,
                           float* observations_grad, void* workspace, size_t workspace_bytes, void* stream);

/* One objective evaluation per problem at x + alpha[b] * direction.
 * Replaces one call of the reference-composed error function plus
 * torch.autograd.grad (bfgs_solver.py:131-135 / wolfe_conditions.py:134-143):
 *   direction (B, P) or NULL (then alpha is ignored and the point is x)
 *   alpha     (B)    or NULL (= 0)
 *   error_out (B)    E
 *   grad_out  (B, P) dE/dx at the point, or NULL
 *   slope_out (B)    d . dE/dx at the point (forward mode), or NULL (needs direction) */
int dava_ba_evaluate(const DavaScene* scene, const float* x, const float* direction, const float* alpha,
                     float* error_out, float* grad_out, float* slope_out, void* stream);

/* Second derivatives of the objective, for differentiating THROUGH a solve whose error
 * function is a fused objective (the reference's create_graph double backward,
 * bfgs_solver.py:133-135).  Per problem, at x with direction v (per problem, NULL = 0):
 *   error_out (B)         E
 *   grad_out  (B, P)      dE/dx
 *   hv_out    (B, P)      (d^2E/dx^2) v
 *   obs_grad_out (B,M,N,2)  dE/dobs
 *   obs_hv_out   (B,M,N,2)  (d^2E/dobs dx) v
 * Every output may be NULL.  Forward-over-reverse of the same objective code (dual numbers).
 * Shapes whose dual LDS image exceeds 160 KiB return DAVA_ERR_UNSUPPORTED.                 */
int dava_ba_second_order(const DavaScene* scene, const float* x, const float* direction, float* error_out,
                         float* grad_out, float* hv_out, float* obs_grad_out, float* obs_hv_out, void* stream);
/* The same with an observation direction u (B, M, N, 2) as well (NULL = 0; r06, additive to ABI 4): the
 * observations carry tangent u, so
 *   hv_out     = (d^2E/dx^2) v + (d^2E/dx dobs) u
 *   obs_hv_out = (d^2E/dobs dx) v + (d^2E/dobs^2) u
 * -- what differentiating dE/dobs again needs (PyTorch double backward of the fused objectives). */
int dava_ba_second_order_obs(const DavaScene* scene, const float* x, const float* direction, const float* obs_direction,
                             float* error_out, float* grad_out, float* hv_out, float* obs_grad_out, float* obs_hv_out,
                             void* stream);

/* ---- generic BFGS building blocks (drive an arbitrary error closure) ----
 * batch = number of problems (all leading dims flattened), n = P.          */

/* BFGSSolver.update_inverse_hessian (bfgs_solver.py:235-303): h, h_out (batch,n,n); s, y (batch,n). */
int dava_bfgs_update_inverse_hessian_f32(int64_t batch, int64_t n, const float* h, const float* s,
                                         const float* y, float* h_out, void* stream);
int dava_bfgs_update_inverse_hessian_f64(int64_t batch, int64_t n, const double* h, const double* s,
                                         const double* y, double* h_out, void* stream);

/* BFGSSolver.scale_initial_inverse_hessian (bfgs_solver.py:217-233): scale_out (batch). */
int dava_bfgs_initial_scale_f32(int64_t batch, int64_t n, const float* s, const float* y, float* scale_out,
                                void* stream);
int dava_bfgs_initial_scale_f64(int64_t batch, int64_t n, const double* s, const double* y,
                                double* scale_out, void* stream);

/* h_out = scale[b] * h (batch,n,n): the k==1 rescale (bfgs_solver.py:159-167). May alias. */
int dava_bfgs_scale_matrix_f32(int64_t batch, int64_t n, const float* scale, const float* h, float* h_out,
                               void* stream);
int dava_bfgs_scale_matrix_f64(int64_t batch, int64_t n, const double* scale, const double* h,
                               double* h_out, void* stream);

/* d_out = -H g (bfgs_solver.py:173-176). */
int dava_bfgs_search_direction_f32(int64_t batch, int64_t n, const float* h, const float* g, float* d_out,
                                   void* stream);
int dava_bfgs_search_direction_f64(int64_t batch, int64_t n, const double* h, const double* g,
                                   double* d_out, void* stream);

/* The generic loop's update + direction WITHOUT the dense matrix (bfgs_solver.py:157-180, the
 * reference's gather / update / scatter of a (B, P, P) inverse Hessian): the inverse Hessian is kept
 * as compact history rows, exact BFGS in product form (the fused solve's COMPACT mode).
 *   S, W   (B_all, capacity, row_stride) history rows s_j and w_j = H_{j-1} y_j of every problem;
 *   rho, c (B_all, capacity); gamma (B_all): per-problem scalars (gamma written when count == 0);
 *   problem_index (n_active) int64: the history slot of each active row of g, y, s, d_out (n_active, n);
 *   count: entries stored so far (the same for every active problem: the loop's step index - 1).
 * For each active problem: H' = gamma I + the `count` stored rank-2 terms; appends entry `count`
 * = (s, H'y, 1/(s.y) or 0 if s.y <= 0, 1 + rho y.H'y) and writes d_out = -H g for
 * H = H' + the new term.  Needs count < capacity and row_stride >= n. */
int dava_bfgs_compact_direction_f32(int64_t n_active, int64_t n, int64_t row_stride, int64_t capacity,
                                    int64_t count, const int64_t* problem_index, const float* g, const float* y,
                                    const float* s, float* S, float* W, float* rho, float* c, float* gamma,
                                    float* d_out, void* stream);
int dava_bfgs_compact_direction_f64(int64_t n_active, int64_t n, int64_t row_stride, int64_t capacity,
                                    int64_t count, const int64_t* problem_index, const double* g, const double* y,
                                    const double* s, double* S, double* W, double* rho, double* c,
                                    double* gamma, double* d_out, void* stream);

/* Strong/weak Wolfe line-search state machine (wolfe_conditions.py:23-239),
 * batched, for an error function evaluated by the caller between calls.
 * state (batch, 9): {a_lo, a_hi, a, f_lo, f_hi, f_a, dphi_a, f0, dphi0}
 * flags (batch, 2) uint8: {widening, zooming}
 *   init:    dphi0 = direction . g0, a = 1, brackets 0, errors f0; widening.
 *   propose: (trial > 0) widening: a_hi = a, f_hi = f_a, a *= 2;
 *            zooming: a = (a_lo + a_hi) / 2.
 *   update:  after the caller wrote f(a) into column 5 and phi'(a) into
 *            column 6 for the active rows, apply N&W 3.5/3.6.
 * The search result is column 1 (a_hi).                                    */
int dava_wolfe_init_f32(int64_t batch, int64_t n, const float* direction, const float* f0, const float* g0,
                        float* state, uint8_t* flags, void* stream);
int dava_wolfe_init_f64(int64_t batch, int64_t n, const double* direction, const double* f0,
                        const double* g0, double* state, uint8_t* flags, void* stream);
int dava_wolfe_propose_f32(int64_t batch, float* state, const uint8_t* flags, void* stream);
int dava_wolfe_propose_f64(int64_t batch, double* state, const uint8_t* flags, void* stream);
int dava_wolfe_update_f32(int64_t batch, int32_t trial, float c1, float c2, int32_t strong, float* state,
                          uint8_t* flags, void* stream);
int dava_wolfe_update_f64(int64_t batch, int32_t trial, double c1, double c2, int32_t strong, double* state,
                          uint8_t* flags, void* stream);

/* ---- reverse mode of the building blocks (differentiating THROUGH the solve) ----
 * The reference's create_graph mode (bfgs_solver.py:85, :134, :213-215) back-propagates
 * through every op of the loop.  These are the vector-Jacobian products of the ops above;
 * grad_out is dL/d(output), every grad_* output may be NULL (not formed).  All (batch,n,n)
 * matrices are row-major and general (H is not assumed symmetric).                      */

/* VJP of update_inverse_hessian, including InverseCurvature's custom backward
 * (utils/func_inverse_curvature.py:36-51).  n <= 150 KiB / (9 sizeof(T)).               */
int dava_bfgs_update_inverse_hessian_backward_f32(int64_t batch, int64_t n, const float* h, const float* s,
                                                  const float* y, const float* grad_out, float* grad_h,
                                                  float* grad_s, float* grad_y, void* stream);
int dava_bfgs_update_inverse_hessian_backward_f64(int64_t batch, int64_t n, const double* h, const double* s,
                                                  const double* y, const double* grad_out, double* grad_h,
                                                  double* grad_s, double* grad_y, void* stream);

/* VJP of initial_scale (clamp backward passes where the input >= the bound, as torch). */
int dava_bfgs_initial_scale_backward_f32(int64_t batch, int64_t n, const float* s, const float* y,
                                         const float* grad_out, float* grad_s, float* grad_y, void* stream);
int dava_bfgs_initial_scale_backward_f64(int64_t batch, int64_t n, const double* s, const double* y,
                                         const double* grad_out, double* grad_s, double* grad_y, void* stream);

/* VJP of scale_matrix: grad_scale (batch), grad_h (batch,n,n). */
int dava_bfgs_scale_matrix_backward_f32(int64_t batch, int64_t n, const float* scale, const float* h,
                                        const float* grad_out, float* grad_scale, float* grad_h, void* stream);
int dava_bfgs_scale_matrix_backward_f64(int64_t batch, int64_t n, const double* scale, const double* h,
                                        const double* grad_out, double* grad_scale, double* grad_h, void* stream);

/* VJP of search_direction (d = -H g): grad_h = -grad_d g^T, grad_g = -H^T grad_d. */
int dava_bfgs_search_direction_backward_f32(int64_t batch, int64_t n, const float* h, const float* g,
                                            const float* grad_d, float* grad_h, float* grad_g, void* stream);
int dava_bfgs_search_direction_backward_f64(int64_t batch, int64_t n, const double* h, const double* g,
                                            const double* grad_d, double* grad_h, double* grad_g, void* stream);

/* ---- the building blocks above on HOST memory (CPU tensors; csrc/bfgs_host.hip) ----
 * The reference's solver runs wherever its parameters live (bfgs_solver.py:94-117; BASELINE C1 is
 * "BFGS on PyTorch CPU").  Same arguments and semantics as the device entry points of the same name
 * without the `dava_cpu_` prefix, every pointer host memory, no stream, synchronous.           */
int dava_cpu_bfgs_update_inverse_hessian_f32(int64_t batch, int64_t n, const float* h, const float* s,
                                             const float* y, float* h_out);
int dava_cpu_bfgs_update_inverse_hessian_f64(int64_t batch, int64_t n, const double* h, const double* s,
                                             const double* y, double* h_out);
int dava_cpu_bfgs_initial_scale_f32(int64_t batch, int64_t n, const float* s, const float* y, float* scale_out);
int dava_cpu_bfgs_initial_scale_f64(int64_t batch, int64_t n, const double* s, const double* y, double* scale_out);
int dava_cpu_bfgs_scale_matrix_f32(int64_t batch, int64_t n, const float* scale, const float* h, float* h_out);
int dava_cpu_bfgs_scale_matrix_f64(int64_t batch, int64_t n, const double* scale, const double* h, double* h_out);
int dava_cpu_bfgs_search_direction_f32(int64_t batch, int64_t n, const float* h, const float* g, float* d_out);
int dava_cpu_bfgs_search_direction_f64(int64_t batch, int64_t n, const double* h, const double* g, double* d_out);
int dava_cpu_wolfe_init_f32(int64_t batch, int64_t n, const float* direction, const float* f0, const float* g0,
                            float* state, uint8_t* flags);
int dava_cpu_wolfe_init_f64(int64_t batch, int64_t n, const double* direction, const double* f0, const double* g0,
                            double* state, uint8_t* flags);
int dava_cpu_wolfe_propose_f32(int64_t batch, float* state, const uint8_t* flags);
int dava_cpu_wolfe_propose_f64(int64_t batch, double* state, const uint8_t* flags);
int dava_cpu_wolfe_update_f32(int64_t batch, int32_t trial, float c1, float c2, int32_t strong, float* state,
                              uint8_t* flags);
int dava_cpu_wolfe_update_f64(int64_t batch, int32_t trial, double c1, double c2, int32_t strong, double* state,
                              uint8_t* flags);
int dava_cpu_bfgs_update_inverse_hessian_backward_f32(int64_t batch, int64_t n, const float* h, const float* s,
                                                      const float* y, const float* grad_out, float* grad_h,
                                                      float* grad_s, float* grad_y);
int dava_cpu_bfgs_update_inverse_hessian_backward_f64(int64_t batch, int64_t n, const double* h, const double* s,
                                                      const double* y, const double* grad_out, double* grad_h,
                                                      double* grad_s, double* grad_y);
int dava_cpu_bfgs_initial_scale_backward_f32(int64_t batch, int64_t n, const float* s, const float* y,
                                             const float* grad_out, float* grad_s, float* grad_y);
int dava_cpu_bfgs_initial_scale_backward_f64(int64_t batch, int64_t n, const double* s, const double* y,
                                             const double* grad_out, double* grad_s, double* grad_y);
int dava_cpu_bfgs_scale_matrix_backward_f32(int64_t batch, int64_t n, const float* scale, const float* h,
                                            const float* grad_out, float* grad_scale, float* grad_h);
int dava_cpu_bfgs_scale_matrix_backward_f64(int64_t batch, int64_t n, const double* scale, const double* h,
                                            const double* grad_out, double* grad_scale, double* grad_h);
int dava_cpu_bfgs_search_direction_backward_f32(int64_t batch, int64_t n, const float* h, const float* g,
                                                const float* grad_d, float* grad_h, float* grad_g);
int dava_cpu_bfgs_search_direction_backward_f64(int64_t batch, int64_t n, const double* h, const double* g,
                                                const double* grad_d, double* grad_h, double* grad_g);

/* ---- legacy IOptimisableFunction camera model (camera_model/pinhole_camera_model_l1.py) ----
 * Error and/or the reference's hand-written gradient of PinholeCameraModelL1 for
 * batch x estimates independent estimates (one workgroup each).  Per estimate:
 *   focal, cx, cy (1)      translation, lie_vector (views, 3)     world_points (points-2, 3)
 * shared per batch item: true_points (views, points, 2), visibility (views, points) 0/1.
 * inverse_pixel_ratio = 1/|maximum_pixel_ratio|; error_scale = the reference's fp32
 * sqrt(1/(views*points)).  error_out (batch, estimates), gradient_out (batch, estimates, P)
 * with P = 3 + 6 views + 3 points - 7, either may be NULL.  points >= 3.                  */
int dava_l1_camera_evaluate_f32(int64_t batch, int32_t estimates, int32_t views, int32_t points, const float* focal,
                                const float* cx, const float* cy, const float* translation, const float* lie_vector,
                                const float* world_points, const float* true_points, const uint8_t* visibility,
                                float minimum_z_distance, float inverse_pixel_ratio, float max_gradient,
                                float error_scale, float* error_out, float* gradient_out, void* stream);
int dava_l1_camera_evaluate_f64(int64_t batch, int32_t estimates, int32_t views, int32_t points, const double* focal,
                                const double* cx, const double* cy, const double* translation,
                                const double* lie_vector, const double* world_points, const double* true_points,
                                const uint8_t* visibility, double minimum_z_distance, double inverse_pixel_ratio,
                                double max_gradient, double error_scale, double* error_out, double* gradient_out,
                                void* stream);

/* Reverse mode through the model above (the reference's autograd through get_error /
 * get_gradient when enable_error_gradients / enable_grad_gradients allow it,
 * pinhole_camera_model_l1.py:132-285).  For every estimate and every input element
 * d in [0, D), D = 3 + 6 views + 3 (points-2), ordered focal, cx, cy, translation (views, 3),
 * lie_vector (views, 3), world_points (points-2, 3):
 *   input_cotangent_out[b, e, d] = error_cotangent[b, e] d error/d x_d
 *                                + sum_q gradient_cotangent[b, e, q] d gradient_q/d x_d
 * (either cotangent may be NULL).  detach_points != 0 differentiates the gradient with the world
 * and camera-relative points held constant, as the reference's enable_grad_gradients = False
 * does (:185-198).  Branches, clamps and clips take the derivative of the branch taken;
 * sign() is flat.  One workgroup per (b, e, d); deterministic.                              */
int dava_l1_camera_vjp_f32(int64_t batch, int32_t estimates, int32_t views, int32_t points, const float* focal,
                           const float* cx, const float* cy, const float* translation, const float* lie_vector,
                           const float* world_points, const float* true_points, const uint8_t* visibility,
                           float minimum_z_distance, float inverse_pixel_ratio, float max_gradient, float error_scale,
                           const float* error_cotangent, const float* gradient_cotangent, int32_t detach_points,
                           float* input_cotangent_out, void* stream);
int dava_l1_camera_vjp_f64(int64_t batch, int32_t estimates, int32_t views, int32_t points, const double* focal,
                           const double* cx, const double* cy, const double* translation, const double* lie_vector,
                           const double* world_points, const double* true_points, const uint8_t* visibility,
                           double minimum_z_distance, double inverse_pixel_ratio, double max_gradient,
                           double error_scale, const double* error_cotangent, const double* gradient_cotangent,
                           int32_t detach_points, double* input_cotangent_out, void* stream);

/* ---- test and A/B hooks ----
 * The library makes its launch choices itself (LDS or global-vector mode, waves per workgroup,
 * on-chip history entries, work queue, ...) and reads NOTHING from the environment.  Tests and A/B
 * measurements override a choice by name (FORCE_GV, GV_NO_XL, SOLVE_WAVES, WG_PER_CU, LDS_HISTORY,
 * STAGGER, STAGGER_LEVELS, NO_PPT, NO_QUEUE, ADJ_GV_WAVES, ADJ_FORCE_GV, ADJ_LDS_ENTRIES, ADJ_GD_HBM,
 * COMPACT_SWITCH, GV_SCALAR_SLICE, ADJ_SC_GLOBAL; csrc/dava_debug.hpp); value < 0 restores the
 * library's choice.  Process-wide, not thread-safe, host-only.  DAVA_ERR_INVALID_ARGUMENT for an
 * unknown name.                                                                                   */
int dava_debug_set_override(const char* name, int64_t value);
void dava_debug_clear_overrides(void);

/* ---- misc ---- */
const char* dava_status_string(int status);
int dava_abi_version(void);
/* Compiled-in device architecture, e.g. "gfx950". */
const char* dava_device_arch(void);

#ifdef __cplusplus
}
#endif

#endif /* DAVA_BA_H */
