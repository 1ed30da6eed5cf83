"""Torch-tensor wrappers over the C ABI (no math here: every call is one HIP launch).

All tensors must live on a ROCm device; work is enqueued on the current
torch stream of that device.
"""
from typing import Optional, Tuple

import torch

from . import _native as N


def _dt(t: torch.Tensor) -> str:
    if t.dtype == torch.float32:
        return "f32"
    if t.dtype == torch.float64:
        return "f64"
    raise TypeError(f"unsupported dtype {t.dtype}: the HIP kernels implement float32 and float64")


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


def scene_struct(observations: torch.Tensor, visibility: torch.Tensor, num_views: int, num_points: int,
                 distortion: bool, batch: int, residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION) -> N.DavaScene:
    p = 3 + 3 * num_points + 6 * (num_views - 1) + (5 if distortion else 0)
    return N.DavaScene(batch, num_views, num_points, 1 if distortion else 0, p,
                       N.ptr(observations), N.ptr(visibility), residual)


def ba_evaluate(x: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor, num_views: int,
                num_points: int, distortion: bool = False, direction: Optional[torch.Tensor] = None,
                alpha: Optional[torch.Tensor] = None, want_grad: bool = True, want_slope: bool = False,
                residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION,
                ) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
    """E, dE/dx, d.dE/dx at x + alpha*direction for a (B, P) fp32 batch."""
    lib = N.load_library()
    N.require_device_tensor(x, "x")
    if x.dtype != torch.float32:
        raise TypeError("the fused BA kernels compute in float32 (the reference's BA dtype)")
    x = _c(x.detach())
    b = x.shape[0]
    obs = _c(observations.detach().to(torch.float32))
    vis = _c(visibility.detach().to(torch.uint8))
    d = _c(direction.detach().to(torch.float32)) if direction is not None else None
    a = _c(alpha.detach().to(torch.float32)) if alpha is not None else None
    err = torch.empty(b, device=x.device, dtype=torch.float32)
    grad = torch.empty_like(x) if want_grad else None
    slope = torch.empty(b, device=x.device, dtype=torch.float32) if want_slope else None
    sc = scene_struct(obs, vis, num_views, num_points, distortion, b, residual)
    with torch.cuda.device(x.device):
        N.check(lib.dava_ba_evaluate(sc, N.ptr(x), N.ptr(d), N.ptr(a), N.ptr(err), N.ptr(grad), N.ptr(slope),
                                     N.stream_of(x.device)), "dava_ba_evaluate")
    return err, grad, slope


def ba_second_order(x: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor, num_views: int,
                    num_points: int, distortion: bool = False, direction: Optional[torch.Tensor] = None,
                    residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION, want_hv: bool = True,
                    want_obs: bool = True):
    """(E, dE/dx, H v, dE/dobs, (d2E/dobs dx) v) for a (B, P) fp32 batch (``dava_ba_second_order``).
    ``direction`` None means v = 0 (then only E, dE/dx and dE/dobs are meaningful)."""
    lib = N.load_library()
    N.require_device_tensor(x, "x")
    if x.dtype != torch.float32:
        raise TypeError("the fused BA kernels compute in float32 (the reference's BA dtype)")
    x = _c(x.detach())
    b = x.shape[0]
    obs = _c(observations.detach().to(torch.float32))
    vis = _c(visibility.detach().to(torch.uint8))
    v = _c(direction.detach().to(torch.float32)) if direction is not None else None
    err = torch.empty(b, device=x.device, dtype=torch.float32)
    grad = torch.empty_like(x)
    hv = torch.empty_like(x) if want_hv else None
    obs_grad = torch.empty_like(obs) if want_obs else None
    obs_hv = torch.empty_like(obs) if (want_obs and want_hv) else None
    sc = scene_struct(obs, vis, num_views, num_points, distortion, b, residual)
    with torch.cuda.device(x.device):
        N.check(lib.dava_ba_second_order(sc, N.ptr(x), N.ptr(v), N.ptr(err), N.ptr(grad), N.ptr(hv), N.ptr(obs_grad),
                                         N.ptr(obs_hv), N.stream_of(x.device)), "dava_ba_second_order")
    return err, grad, hv, obs_grad, obs_hv


def ba_solve(x0: torch.Tensor, observations: torch.Tensor, visibility: torch.Tensor, num_views: int,
             num_points: int, distortion: bool, *, sufficient_decrease: float = 1e-4, curvature: float = 0.9,
             error_threshold: float = 1e-4, iterations: int = 1000, minimum_step: float = 1e-8,
             max_line_search_trials: int = 1000, strong: bool = True, hessian_mode: int = N.DAVA_HESSIAN_DENSE,
             want_error: bool = False, want_status: bool = False, workspace: Optional[torch.Tensor] = None,
             residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION):
    """One fused launch for the whole batch.  Returns (x, error|None, status|None)."""
    lib = N.load_library()
    N.require_device_tensor(x0, "parameters")
    if x0.dtype != torch.float32:
        raise TypeError("the fused BA solver computes in float32 (the reference's BA dtype)")
    x0 = _c(x0.detach())
    b = x0.shape[0]
    dev = x0.device
    obs = _c(observations.detach().to(device=dev, dtype=torch.float32))
    vis = _c(visibility.detach().to(device=dev, dtype=torch.uint8))
    sc = scene_struct(obs, vis, num_views, num_points, distortion, b, residual)
    cfg = N.DavaSolverConfig(float(sufficient_decrease), float(curvature), float(error_threshold),
                             float(minimum_step), int(iterations), int(max_line_search_trials),
                             1 if strong else 0, int(hessian_mode))
    need = int(lib.dava_ba_solve_workspace_bytes(sc, cfg))
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    x_out = torch.empty_like(x0)
    err = torch.empty(b, device=dev, dtype=torch.float32) if want_error else None
    status = torch.empty((b, N.STATUS_WORDS), device=dev, dtype=torch.int32) if want_status else None
    with torch.cuda.device(dev):
        N.check(lib.dava_ba_solve(sc, cfg, N.ptr(x0), N.ptr(x_out), N.ptr(err), N.ptr(status), N.ptr(workspace),
                                  workspace.numel(), N.stream_of(dev)), "dava_ba_solve")
    return x_out, err, status


def solve_workspace_bytes(batch: int, num_views: int, num_points: int, distortion: bool,
                          hessian_mode: int = N.DAVA_HESSIAN_DENSE, iterations: int = 1000) -> int:
    lib = N.load_library()
    sc = scene_struct(None, None, num_views, num_points, distortion, batch)
    cfg = N.DavaSolverConfig(1e-4, 0.9, 1e-4, 1e-8, iterations, 1000, 1, hessian_mode)
    return int(lib.dava_ba_solve_workspace_bytes(sc, cfg))


def solve_plan(batch: int, num_views: int, num_points: int, distortion: bool,
               hessian_mode: int = N.DAVA_HESSIAN_DENSE, iterations: int = 1000,
               residual: int = N.DAVA_RESIDUAL_SQUARED_REPROJECTION) -> dict:
    """How ``dava_ba_solve`` runs this shape (host-only query): global-vector mode, workgroup
    size, LDS bytes and the number of history entries kept on-chip (COMPACT)."""
    lib = N.load_library()
    sc = scene_struct(None, None, num_views, num_points, distortion, batch, residual)
    cfg = N.DavaSolverConfig(1e-4, 0.9, 1e-4, 1e-8, iterations, 1000, 1, hessian_mode)
    plan = N.DavaSolvePlan()
    N.check(lib.dava_ba_solve_plan(sc, cfg, plan), "dava_ba_solve_plan")
    return {name: int(getattr(plan, name)) for name, _ in N.DavaSolvePlan._fields_}


# ---- generic BFGS building blocks ----
# Each public op is a torch.autograd.Function whose forward AND backward are HIP kernels
# (bfgs_ops.hip / bfgs_grad.hip), so the drop-in solver can be differentiated through
# exactly like the reference (bfgs_solver.py:85, :134, :213-215).

def _empty_or_none(needed: bool, like: torch.Tensor) -> Optional[torch.Tensor]:
    return torch.empty_like(like) if needed else None


def _update_forward(h: torch.Tensor, s: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    lib = N.load_library()
    N.require_device_tensor(h, "inverse_hessian")
    n = h.shape[-1]
    lead = h.shape[:-2]
    hb, sb, yb = _c(h.detach()).reshape(-1, n, n), _c(s.detach()).reshape(-1, n), _c(y.detach()).reshape(-1, n)
    out = torch.empty_like(hb)
    with torch.cuda.device(h.device):
        N.check(getattr(lib, f"dava_bfgs_update_inverse_hessian_{_dt(h)}")(
            hb.shape[0], n, N.ptr(hb), N.ptr(sb), N.ptr(yb), N.ptr(out), N.stream_of(h.device)),
            "dava_bfgs_update_inverse_hessian")
    return out.reshape(lead + (n, n))


class _UpdateInverseHessian(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, s, y):
        ctx.save_for_backward(h, s, y)
        return _update_forward(h, s, y)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        h, s, y = ctx.saved_tensors
        n = h.shape[-1]
        hb, sb, yb = _c(h).reshape(-1, n, n), _c(s).reshape(-1, n), _c(y).reshape(-1, n)
        gb = _c(grad).reshape(-1, n, n)
        gh = _empty_or_none(ctx.needs_input_grad[0], hb)
        gs = _empty_or_none(ctx.needs_input_grad[1], sb)
        gy = _empty_or_none(ctx.needs_input_grad[2], yb)
        with torch.cuda.device(h.device):
            N.check(getattr(N.load_library(), f"dava_bfgs_update_inverse_hessian_backward_{_dt(h)}")(
                hb.shape[0], n, N.ptr(hb), N.ptr(sb), N.ptr(yb), N.ptr(gb), N.ptr(gh), N.ptr(gs), N.ptr(gy),
                N.stream_of(h.device)), "dava_bfgs_update_inverse_hessian_backward")
        return (gh.reshape(h.shape) if gh is not None else None, gs.reshape(s.shape) if gs is not None else None,
                gy.reshape(y.shape) if gy is not None else None)


def update_inverse_hessian(h: torch.Tensor, s: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """``BFGSSolver.update_inverse_hessian`` (bfgs_solver.py:235-303), differentiable."""
    return _UpdateInverseHessian.apply(h, s, y)


def _initial_scale_forward(s: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    lib = N.load_library()
    N.require_device_tensor(s, "step")
    n = s.shape[-1]
    sb, yb = _c(s.detach()).reshape(-1, n), _c(y.detach()).reshape(-1, n)
    out = torch.empty(sb.shape[0], device=s.device, dtype=s.dtype)
    with torch.cuda.device(s.device):
        N.check(getattr(lib, f"dava_bfgs_initial_scale_{_dt(s)}")(
            sb.shape[0], n, N.ptr(sb), N.ptr(yb), N.ptr(out), N.stream_of(s.device)), "dava_bfgs_initial_scale")
    return out.reshape(s.shape[:-1] + (1,))


class _InitialScale(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, y):
        ctx.save_for_backward(s, y)
        return _initial_scale_forward(s, y)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        s, y = ctx.saved_tensors
        n = s.shape[-1]
        sb, yb = _c(s).reshape(-1, n), _c(y).reshape(-1, n)
        gb = _c(grad).reshape(-1)
        gs = _empty_or_none(ctx.needs_input_grad[0], sb)
        gy = _empty_or_none(ctx.needs_input_grad[1], yb)
        with torch.cuda.device(s.device):
            N.check(getattr(N.load_library(), f"dava_bfgs_initial_scale_backward_{_dt(s)}")(
                sb.shape[0], n, N.ptr(sb), N.ptr(yb), N.ptr(gb), N.ptr(gs), N.ptr(gy), N.stream_of(s.device)),
                "dava_bfgs_initial_scale_backward")
        return (gs.reshape(s.shape) if gs is not None else None, gy.reshape(y.shape) if gy is not None else None)


def initial_scale(s: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """(..., 1) like the reference's keepdims result (bfgs_solver.py:217-233), differentiable."""
    return _InitialScale.apply(s, y)


def _scale_matrix_forward(scale: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    lib = N.load_library()
    n = h.shape[-1]
    hb = _c(h.detach()).reshape(-1, n, n)
    sc = _c(scale.detach()).reshape(-1)
    out = torch.empty_like(hb)
    with torch.cuda.device(h.device):
        N.check(getattr(lib, f"dava_bfgs_scale_matrix_{_dt(h)}")(
            hb.shape[0], n, N.ptr(sc), N.ptr(hb), N.ptr(out), N.stream_of(h.device)), "dava_bfgs_scale_matrix")
    return out.reshape(h.shape)


class _ScaleMatrix(torch.autograd.Function):
    @staticmethod
    def forward(ctx, scale, h):
        ctx.save_for_backward(scale, h)
        return _scale_matrix_forward(scale, h)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        scale, h = ctx.saved_tensors
        n = h.shape[-1]
        hb, sc, gb = _c(h).reshape(-1, n, n), _c(scale).reshape(-1), _c(grad).reshape(-1, n, n)
        gsc = _empty_or_none(ctx.needs_input_grad[0], sc)
        gh = _empty_or_none(ctx.needs_input_grad[1], hb)
        with torch.cuda.device(h.device):
            N.check(getattr(N.load_library(), f"dava_bfgs_scale_matrix_backward_{_dt(h)}")(
                hb.shape[0], n, N.ptr(sc), N.ptr(hb), N.ptr(gb), N.ptr(gsc), N.ptr(gh), N.stream_of(h.device)),
                "dava_bfgs_scale_matrix_backward")
        return (gsc.reshape(scale.shape) if gsc is not None else None, gh.reshape(h.shape) if gh is not None else None)


def scale_matrix(scale: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """scale[..., None] * h: the k == 1 rescale of H0 (bfgs_solver.py:159-167), differentiable."""
    return _ScaleMatrix.apply(scale, h)


def _search_direction_forward(h: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    lib = N.load_library()
    n = h.shape[-1]
    hb = _c(h.detach()).reshape(-1, n, n)
    gb = _c(g.detach()).reshape(-1, n)
    out = torch.empty_like(gb)
    with torch.cuda.device(h.device):
        N.check(getattr(lib, f"dava_bfgs_search_direction_{_dt(h)}")(
            hb.shape[0], n, N.ptr(hb), N.ptr(gb), N.ptr(out), N.stream_of(h.device)), "dava_bfgs_search_direction")
    return out.reshape(g.shape)


class _SearchDirection(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, g):
        ctx.save_for_backward(h, g)
        return _search_direction_forward(h, g)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        h, g = ctx.saved_tensors
        n = h.shape[-1]
        hb, gv, db = _c(h).reshape(-1, n, n), _c(g).reshape(-1, n), _c(grad).reshape(-1, n)
        gh = _empty_or_none(ctx.needs_input_grad[0], hb)
        gg = _empty_or_none(ctx.needs_input_grad[1], gv)
        with torch.cuda.device(h.device):
            N.check(getattr(N.load_library(), f"dava_bfgs_search_direction_backward_{_dt(h)}")(
                hb.shape[0], n, N.ptr(hb), N.ptr(gv), N.ptr(db), N.ptr(gh), N.ptr(gg), N.stream_of(h.device)),
                "dava_bfgs_search_direction_backward")
        return (gh.reshape(h.shape) if gh is not None else None, gg.reshape(g.shape) if gg is not None else None)


def search_direction(h: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """d = -H g (bfgs_solver.py:173-176), differentiable."""
    return _SearchDirection.apply(h, g)


class WolfeState:
    """Device-resident batched line-search state (columns per include/dava_ba.h)."""
    A_LO, A_HI, A, F_LO, F_HI, F_A, DPHI_A, F0, DPHI0 = range(9)

    def __init__(self, direction: torch.Tensor, f0: torch.Tensor, g0: torch.Tensor):
        self.lib = N.load_library()
        N.require_device_tensor(direction, "search_direction")
        self.dt = _dt(direction)
        n = direction.shape[-1]
        d = _c(direction.detach()).reshape(-1, n)
        g = _c(g0.detach().to(direction.dtype)).reshape(-1, n)
        f = _c(f0.detach().to(direction.dtype)).reshape(-1)
        self.batch = d.shape[0]
        self.device = direction.device
        self.state = torch.empty((self.batch, 9), device=self.device, dtype=direction.dtype)
        self.flags = torch.empty((self.batch, 2), device=self.device, dtype=torch.uint8)
        with torch.cuda.device(self.device):
            N.check(getattr(self.lib, f"dava_wolfe_init_{self.dt}")(
                self.batch, n, N.ptr(d), N.ptr(f), N.ptr(g), N.ptr(self.state), N.ptr(self.flags),
                N.stream_of(self.device)), "dava_wolfe_init")

    def active(self) -> torch.Tensor:
        return (self.flags[:, 0] | self.flags[:, 1]).bool()

    def propose(self) -> None:
        with torch.cuda.device(self.device):
            N.check(getattr(self.lib, f"dava_wolfe_propose_{self.dt}")(
                self.batch, N.ptr(self.state), N.ptr(self.flags), N.stream_of(self.device)), "dava_wolfe_propose")

    def update(self, trial: int, c1: float, c2: float, strong: bool) -> None:
        with torch.cuda.device(self.device):
            N.check(getattr(self.lib, f"dava_wolfe_update_{self.dt}")(
                self.batch, int(trial), float(c1), float(c2), 1 if strong else 0, N.ptr(self.state),
                N.ptr(self.flags), N.stream_of(self.device)), "dava_wolfe_update")
