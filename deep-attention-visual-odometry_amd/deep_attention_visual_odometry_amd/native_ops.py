"""Torch-tensor wrappers over the ``torch.ops.dava`` operators (``_ops.py``, one HIP launch each;
no math here).

All tensors must live on a ROCm device; work is enqueued on the current torch stream of that
device.  The generic BFGS building blocks are ``torch.autograd.Function`` s whose forward and
backward are both ``torch.ops.dava`` operators, so ``torch.compile`` traces them (fake kernels
give the shapes) and autograd differentiates through them like the reference's torch code.
"""
from typing import Optional, Tuple

import torch

from . import _native as N
from . import _ops  # noqa: F401  (registers torch.ops.dava.*)
from ._ops import _dt, scene_struct, solver_config


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


def _scene_inputs(x: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor):
    dev = x.device
    obs = _c(observations.detach().to(device=dev, dtype=torch.float32))
    vis = _c(visibility.detach().to(device=dev, dtype=torch.uint8))
    return obs, vis


def _fp32_on_device(x: torch.Tensor, what: str) -> torch.Tensor:
    N.require_device_tensor(x, what)
    if x.dtype != torch.float32:
        raise TypeError("the fused BA kernels compute in float32 (the reference's BA dtype)")
    return _c(x.detach())


def _opt(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None else _c(t.detach().to(torch.float32))


def ba_evaluate(x: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor, num_views: int,
                num_points: int, distortion: bool = False, direction: Optional[torch.Tensor] = None,
                alpha: Optional[torch.Tensor] = None, want_grad: bool = True, want_slope: bool = False,
                residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION,
                ) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
    """E, dE/dx, d.dE/dx at x + alpha*direction for a (B, P) fp32 batch (``torch.ops.dava.ba_evaluate``)."""
    x = _fp32_on_device(x, "x")
    obs, vis = _scene_inputs(x, observations, visibility)
    err, grad, slope = torch.ops.dava.ba_evaluate(x, obs, vis, num_views, num_points, bool(distortion),
                                                  _opt(direction), _opt(alpha), bool(want_grad), bool(want_slope),
                                                  int(residual))
    return err, (grad if want_grad else None), (slope if want_slope else None)


def ba_second_order(x: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor, num_views: int,
                    num_points: int, distortion: bool = False, direction: Optional[torch.Tensor] = None,
                    residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION, want_hv: bool = True,
                    want_obs: bool = True, obs_direction: Optional[torch.Tensor] = None):
    """(E, dE/dx, H v + (d2E/dx dobs) u, dE/dobs, (d2E/dobs dx) v + (d2E/dobs2) u) for a (B, P) fp32 batch
    (``torch.ops.dava.ba_second_order``).  ``direction`` / ``obs_direction`` None mean v = 0 / u = 0 (with both
    None only E, dE/dx and dE/dobs are meaningful)."""
    x = _fp32_on_device(x, "x")
    obs, vis = _scene_inputs(x, observations, visibility)
    if obs_direction is not None:
        obs_direction = _c(obs_direction.detach().to(device=x.device, dtype=torch.float32)).reshape(obs.shape)
    err, grad, hv, obs_grad, obs_hv = torch.ops.dava.ba_second_order(
        x, obs, vis, num_views, num_points, bool(distortion), _opt(direction), int(residual), bool(want_hv),
        bool(want_obs), obs_direction)
    return (err, grad, hv if want_hv else None, obs_grad if want_obs else None,
            obs_hv if (want_obs and want_hv) else None)


def ba_solve(x0: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor, num_views: int,
             num_points: int, distortion: bool, *, sufficient_decrease: float = 1e-4, curvature: float = 0.9,
             error_threshold: float = 1e-4, iterations: int = 1000, minimum_step: float = 1e-8,
             max_line_search_trials: int = 1000, strong: bool = True, hessian_mode: int = N.DAVA_HESSIAN_DENSE,
             want_error: bool = False, want_status: bool = False, workspace: Optional[torch.Tensor] = None,
             residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION, drop_path_p: float = 0.0, drop_seed: int = 0,
             return_second_last: bool = False):
    """One fused launch for the whole batch (``torch.ops.dava.ba_solve``).  Returns (x, error|None, status|None).
    ``drop_path_p`` > 0: training mode's drop path with the counter-based schedule of ``drop_seed``.
    ``return_second_last``: a problem stopped by the minimum-step rule returns x before its last step
    (see :func:`second_last_moves_rows` for the one case the reference does differently)."""
    x0 = _fp32_on_device(x0, "parameters")
    obs, vis = _scene_inputs(x0, observations, visibility)
    x, err, status = torch.ops.dava.ba_solve(
        x0, obs, vis, int(num_views), int(num_points), bool(distortion), float(sufficient_decrease),
        float(curvature), float(error_threshold), int(iterations), float(minimum_step), int(max_line_search_trials),
        bool(strong), int(hessian_mode), int(residual), bool(want_error),
        workspace if workspace is not None else x0.new_empty((0,), dtype=torch.uint8), float(drop_path_p),
        int(drop_seed), bool(return_second_last))
    return x, (err if want_error else None), (status if want_status else None)


def second_last_moves_rows(status: torch.Tensor) -> bool:
    """Would the reference's return_second_last scatter (bfgs_solver.py:196-212) have moved rows between
    problems in this solve?  At iteration k it scatters the step-updated rows of the problems that were
    active in the line search into the problems still active after the minimum-step test, in batch
    order: row i of the first set lands on the i-th problem of the second.  That is the identity exactly
    when every problem stopping by the minimum-step rule at k comes after every problem passing it at k.
    From the status words: a problem that stopped by the rule (DAVA_STOP_STEP) after s steps failed it at
    iteration s - 1; any other problem passed it at iterations 0 .. s - 1 (s - 2 for the rule's own).
    One host sync."""
    st = status.reshape(-1, N.STATUS_WORDS)
    if st.shape[0] < 2:
        return False
    steps, by_rule = st[:, 0].long(), st[:, 1] == N.STOP_STEP
    last_pass = steps - 1 - by_rule.long()  # last iteration at which the problem passed the test
    # largest last_pass among the problems AFTER each one (suffix maximum, exclusive)
    after = torch.flip(torch.cummax(torch.flip(last_pass, [0]), 0).values, [0])
    after = torch.cat([after[1:], after.new_full((1,), -2)])
    return bool((by_rule & (after >= steps - 1)).any().item())


def solve_tape_supported(batch: int, num_views: int, num_points: int, distortion: bool, iterations: int,
                         residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION) -> bool:
    """Host-only: does this shape have the fused adjoint -- a recording forward
    (``dava_ba_solve_tape_bytes`` > 0) AND a backward that can launch on it
    (``dava_ba_solve_backward_workspace_bytes`` > 0)?"""
    lib = N.load_library()
    sc = scene_struct(None, None, num_views, num_points, distortion, max(int(batch), 1), residual)
    cfg = solver_config(1e-4, 0.9, 1e-4, iterations, 1e-8, 1000, True, N.DAVA_HESSIAN_COMPACT)
    return int(lib.dava_ba_solve_tape_bytes(sc, cfg)) > 0 and int(lib.dava_ba_solve_backward_workspace_bytes(sc, cfg)) > 0


class _FusedSolve(torch.autograd.Function):
    """x_out = solve(x0, obs) in one recording launch; its backward is the adjoint kernel
    (csrc/bfgs_adjoint.hip), which replays the tape: the reference's create_graph gradient
    through BFGSSolver.forward (bfgs_solver.py:85, :133-135, :213-215) without a (B, P, P)
    inverse Hessian per iteration.  Not differentiable twice."""

    @staticmethod
    def forward(ctx, x0, observations, visibility, num_views, num_points, distortion, residual, cfg):
        c1, c2, thr, iters, min_step, trials, strong, drop_p, drop_seed, second_last = cfg
        x0c = _fp32_on_device(x0, "parameters")
        obs, vis = _scene_inputs(x0c, observations, visibility)
        x, status, tape = torch.ops.dava.ba_solve_record(
            x0c, obs, vis, int(num_views), int(num_points), bool(distortion), float(c1), float(c2), float(thr),
            int(iters), float(min_step), int(trials), bool(strong), int(residual), float(drop_p), int(drop_seed),
            bool(second_last))
        replay = status
        if second_last:  # a minimum-step stop returned x before its last step: the adjoint replays one fewer
            replay = status.clone()
            replay[:, 0] -= (status[:, 1] == N.STOP_STEP).to(torch.int32)
        ctx.save_for_backward(tape, replay, obs, vis)
        ctx.meta = (int(num_views), int(num_points), bool(distortion), int(iters), int(residual))
        ctx.mark_non_differentiable(status)
        ctx.recorded = torch.cuda.Event()  # the tape is complete once the recording launch is
        ctx.recorded.record(torch.cuda.current_stream(x0c.device))
        return x, status

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, x_grad, _status_grad):
        tape, status, obs, vis = ctx.saved_tensors
        m, n, dist, iters, residual = ctx.meta
        need_x, need_obs = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if x_grad is None:
            return (None,) * 8
        # autograd may run this backward on another stream than the recording launch's: order the
        # adjoint after the tape is written
        torch.cuda.current_stream(tape.device).wait_event(ctx.recorded)
        gx, gobs = torch.ops.dava.ba_solve_backward(_c(x_grad.to(torch.float32)), tape, status, obs, vis, m, n, dist,
                                                    iters, residual, bool(need_obs))
        return (gx if need_x else None, gobs if need_obs else None, None, None, None, None, None, None)


def ba_solve_differentiable(x0: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor, num_views: int,
                            num_points: int, distortion: bool, *, sufficient_decrease: float = 1e-4,
                            curvature: float = 0.9, error_threshold: float = 1e-4, iterations: int = 1000,
                            minimum_step: float = 1e-8, max_line_search_trials: int = 1000, strong: bool = True,
                            residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION, drop_path_p: float = 0.0,
                            drop_seed: int = 0, return_second_last: bool = False):
    """The fused COMPACT solve as an autograd node w.r.t. x0 and the observations.
    Returns (x, status)."""
    cfg = (sufficient_decrease, curvature, error_threshold, iterations, minimum_step, max_line_search_trials, strong,
           drop_path_p, drop_seed, return_second_last)
    return _FusedSolve.apply(x0, observations, visibility, num_views, num_points, distortion, residual, cfg)


def solve_workspace_bytes(batch: int, num_views: int, num_points: int, distortion: bool,
                          hessian_mode: int = N.DAVA_HESSIAN_DENSE, iterations: int = 1000) -> int:
    lib = N.load_library()
    sc = scene_struct(None, None, num_views, num_points, distortion, batch)
    cfg = solver_config(1e-4, 0.9, 1e-4, iterations, 1e-8, 1000, True, hessian_mode)
    return int(lib.dava_ba_solve_workspace_bytes(sc, cfg))


def solve_plan(batch: int, num_views: int, num_points: int, distortion: bool,
               hessian_mode: int = N.DAVA_HESSIAN_DENSE, iterations: int = 1000,
               residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION) -> dict:
    """How ``dava_ba_solve`` runs this shape (host-only query): global-vector mode, workgroup
    size, LDS bytes and the number of history entries kept on-chip (COMPACT)."""
    lib = N.load_library()
    sc = scene_struct(None, None, num_views, num_points, distortion, batch, residual)
    cfg = solver_config(1e-4, 0.9, 1e-4, iterations, 1e-8, 1000, True, hessian_mode)
    plan = N.DavaSolvePlan()
    N.check(lib.dava_ba_solve_plan(sc, cfg, plan), "dava_ba_solve_plan")
    return {name: int(getattr(plan, name)) for name, _ in N.DavaSolvePlan._fields_}


def adjoint_lds_entries(batch: int, num_views: int, num_points: int, distortion: bool, iterations: int,
                        residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION) -> int:
    """History entries the fused solve's adjoint keeps on chip (``dava_ba_solve_backward_lds_entries``);
    0 where the adjoint does not run."""
    sc = scene_struct(None, None, num_views, num_points, distortion, batch, residual)
    cfg = solver_config(1e-4, 0.9, -1.0, iterations, -1.0, 1000, True, N.DAVA_HESSIAN_COMPACT)
    return int(N.load_library().dava_ba_solve_backward_lds_entries(sc, cfg))


# ---- generic BFGS building blocks ----
# Each public op is a torch.autograd.Function whose forward AND backward are torch.ops.dava
# operators (HIP kernels, bfgs_ops.hip / bfgs_grad.hip), so the drop-in solver can be
# differentiated through exactly like the reference (bfgs_solver.py:85, :134, :213-215).

def _device_tensor(t: torch.Tensor, what: str) -> torch.Tensor:
    """A ROCm tensor (HIP kernels) or a CPU tensor (the library's host flavours): the operators dispatch
    on the device."""
    N.require_host_or_device_tensor(t, what)
    _dt(t)
    return t


class _UpdateInverseHessian(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, s, y):
        ctx.save_for_backward(h, s, y)
        n = h.shape[-1]
        out = torch.ops.dava.bfgs_update_inverse_hessian(_c(h.detach()).reshape(-1, n, n),
                                                         _c(s.detach()).reshape(-1, n), _c(y.detach()).reshape(-1, n))
        return out.reshape(h.shape)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        h, s, y = ctx.saved_tensors
        n = h.shape[-1]
        nh, ns, ny = ctx.needs_input_grad
        gh, gs, gy = torch.ops.dava.bfgs_update_inverse_hessian_backward(
            _c(h).reshape(-1, n, n), _c(s).reshape(-1, n), _c(y).reshape(-1, n), _c(grad).reshape(-1, n, n),
            nh, ns, ny)
        return (gh.reshape(h.shape) if nh else None, gs.reshape(s.shape) if ns else None,
                gy.reshape(y.shape) if ny else None)


def update_inverse_hessian(h: torch.Tensor, s: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """``BFGSSolver.update_inverse_hessian`` (bfgs_solver.py:235-303), differentiable."""
    _device_tensor(h, "inverse_hessian")
    return _UpdateInverseHessian.apply(h, s, y)


class _InitialScale(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, y):
        ctx.save_for_backward(s, y)
        n = s.shape[-1]
        out = torch.ops.dava.bfgs_initial_scale(_c(s.detach()).reshape(-1, n), _c(y.detach()).reshape(-1, n))
        return out.reshape(s.shape[:-1] + (1,))

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        s, y = ctx.saved_tensors
        n = s.shape[-1]
        ns, ny = ctx.needs_input_grad
        gs, gy = torch.ops.dava.bfgs_initial_scale_backward(_c(s).reshape(-1, n), _c(y).reshape(-1, n),
                                                            _c(grad).reshape(-1), ns, ny)
        return (gs.reshape(s.shape) if ns else None, gy.reshape(y.shape) if ny else None)


def initial_scale(s: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """(..., 1) like the reference's keepdims result (bfgs_solver.py:217-233), differentiable."""
    _device_tensor(s, "step")
    return _InitialScale.apply(s, y)


class _ScaleMatrix(torch.autograd.Function):
    @staticmethod
    def forward(ctx, scale, h):
        ctx.save_for_backward(scale, h)
        n = h.shape[-1]
        out = torch.ops.dava.bfgs_scale_matrix(_c(scale.detach()).reshape(-1), _c(h.detach()).reshape(-1, n, n))
        return out.reshape(h.shape)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        scale, h = ctx.saved_tensors
        n = h.shape[-1]
        nsc, nh = ctx.needs_input_grad
        gsc, gh = torch.ops.dava.bfgs_scale_matrix_backward(_c(scale).reshape(-1), _c(h).reshape(-1, n, n),
                                                            _c(grad).reshape(-1, n, n), nsc, nh)
        return (gsc.reshape(scale.shape) if nsc else None, gh.reshape(h.shape) if nh else None)


def scale_matrix(scale: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """scale[..., None] * h: the k == 1 rescale of H0 (bfgs_solver.py:159-167), differentiable."""
    _device_tensor(h, "inverse_hessian")
    return _ScaleMatrix.apply(scale, h)


class _SearchDirection(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, g):
        ctx.save_for_backward(h, g)
        n = h.shape[-1]
        out = torch.ops.dava.bfgs_search_direction(_c(h.detach()).reshape(-1, n, n), _c(g.detach()).reshape(-1, n))
        return out.reshape(g.shape)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        h, g = ctx.saved_tensors
        n = h.shape[-1]
        nh, ng = ctx.needs_input_grad
        gh, gg = torch.ops.dava.bfgs_search_direction_backward(_c(h).reshape(-1, n, n), _c(g).reshape(-1, n),
                                                               _c(grad).reshape(-1, n), nh, ng)
        return (gh.reshape(h.shape) if nh else None, gg.reshape(g.shape) if ng else None)


def search_direction(h: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """d = -H g (bfgs_solver.py:173-176), differentiable."""
    _device_tensor(h, "inverse_hessian")
    return _SearchDirection.apply(h, g)


class CompactHistory:
    """The generic loop's inverse Hessian as compact history rows (``dava_bfgs_compact_direction``): per problem
    of the whole batch the rank-2 terms (s_j, w_j = H_{j-1} y_j, rho_j, c_j) and gamma, replacing the reference's
    dense (B, P, P) matrix and its masked gather / scatter (``bfgs_solver.py:157-180``).  Rows grow by doubling
    as the loop runs, so memory is O(k P) per problem at iteration k.  Not differentiable: the loop takes it
    only when no graph is kept (the create_graph mode keeps the dense ops and their VJP kernels)."""

    LDS_LIMIT = 150 * 1024  # csrc/bfgs_ops.hip compact_direction: y, g and 4 coefficients per entry in LDS

    def __init__(self, batch: int, p: int, dtype: torch.dtype, device, max_entries: int, capacity: int = 16):
        self.batch, self.p, self.dtype, self.device = int(batch), int(p), dtype, device
        self.stride = (self.p + 3) // 4 * 4
        self.max_entries = max(int(max_entries), 1)
        self.count = 0
        self.gamma = torch.zeros((self.batch,), dtype=dtype, device=device)
        self._alloc(min(capacity, self.max_entries))

    @classmethod
    def supported(cls, p: int, dtype: torch.dtype, max_entries: int) -> bool:
        if dtype not in (torch.float32, torch.float64):
            return False
        size = 4 if dtype == torch.float32 else 8
        return (2 * ((p + 3) // 4 * 4) + 4 * max(max_entries, 1)) * size <= cls.LDS_LIMIT

    def _alloc(self, cap: int) -> None:
        new = [torch.zeros((self.batch, cap, self.stride), dtype=self.dtype, device=self.device) for _ in range(2)]
        scal = [torch.zeros((self.batch, cap), dtype=self.dtype, device=self.device) for _ in range(2)]
        if self.count:
            for a, b in zip(new + scal, (self.s, self.w, self.rho, self.c)):
                a[:, :self.count] = b[:, :self.count]
        self.s, self.w = new
        self.rho, self.c = scal
        self.capacity = cap

    def direction(self, gradient: torch.Tensor, delta_gradient: torch.Tensor, step: torch.Tensor,
                  problem_index: torch.Tensor) -> torch.Tensor:
        """Append (step, H'y) for the active problems `problem_index` (flat batch indices, int64) and return
        d = -H g for them, H the inverse Hessian after this update."""
        if self.count >= self.max_entries:
            raise RuntimeError(f"compact history full ({self.max_entries} entries)")
        if self.count >= self.capacity:
            self._alloc(min(2 * self.capacity, self.max_entries))
        d = torch.ops.dava.bfgs_compact_direction(_c(gradient.detach()), _c(delta_gradient.detach()),
                                                  _c(step.detach()), _c(problem_index), self.count, self.s, self.w,
                                                  self.rho, self.c, self.gamma)
        self.count += 1
        return d

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.s, self.w, self.rho, self.c, self.gamma))


class WolfeState:
    """Device-resident batched line-search state (columns per include/dava_ba.h)."""
    A_LO, A_HI, A, F_LO, F_HI, F_A, DPHI_A, F0, DPHI0 = range(9)

    def __init__(self, direction: torch.Tensor, f0: torch.Tensor, g0: torch.Tensor):
        _device_tensor(direction, "search_direction")
        n = direction.shape[-1]
        d = _c(direction.detach()).reshape(-1, n)
        g = _c(g0.detach().to(direction.dtype)).reshape(-1, n)
        f = _c(f0.detach().to(direction.dtype)).reshape(-1)
        self.batch = d.shape[0]
        self.device = direction.device
        self.state, self.flags = torch.ops.dava.wolfe_init(d, f, g)

    def active(self) -> torch.Tensor:
        return (self.flags[:, 0] | self.flags[:, 1]).bool()

    def propose(self) -> None:
        torch.ops.dava.wolfe_propose(self.state, self.flags)

    def update(self, trial: int, c1: float, c2: float, strong: bool) -> None:
        torch.ops.dava.wolfe_update(self.state, self.flags, int(trial), float(c1), float(c2), bool(strong))
