"""Eval-mode BFGS + strong-Wolfe line search (oracle restatement, test infrastructure only).

Restates, in batched PyTorch-CPU form with the same masking semantics and
the same op order (so results are bitwise equal to the reference, see
``tests/test_oracle_golden.py``):

* ``bfgs_solve``          -- ``autograd_solvers/bfgs_solver.py:80-215`` with
                            ``self.training == False`` (no drop-path, no
                            second-last return).
* ``initial_scale``       -- ``bfgs_solver.py:217-233`` (N&W eq. 6.20).
* ``bfgs_update``         -- ``bfgs_solver.py:235-303`` (N&W eq. 6.17).
* ``wolfe_line_search``   -- ``autograd_solvers/line_search/wolfe_conditions.py:23-239``
                            (N&W algorithms 3.5/3.6, bisection zoom, <= 1000 trials,
                            returns the upper bracket).

It also records per-problem statistics (iterations taken, why each problem
stopped, closure evaluations) so the HIP kernel's status words can be
compared with it.
"""
from dataclasses import dataclass, field
from typing import Callable, Optional

import torch

from .trig import curvature_reciprocal

STOP_ITERATIONS = 0
STOP_ERROR = 1
STOP_STEP = 2


def initial_scale(step: torch.Tensor, delta_gradient: torch.Tensor) -> torch.Tensor:
    denom = delta_gradient.square().sum(dim=-1, keepdims=True).clamp(min=1e-5)
    num = (step * delta_gradient).sum(dim=-1, keepdims=True)
    return (num / denom).clamp(min=1e-4)


def bfgs_update(h: torch.Tensor, step: torch.Tensor, delta_gradient: torch.Tensor) -> torch.Tensor:
    """H+ = H + (1 + rho y'Hy) rho s s' - rho s (y'H) - (H y) rho s'."""
    rho = curvature_reciprocal(step, delta_gradient)
    y_h = torch.matmul(delta_gradient.unsqueeze(-2), h)
    y_rho = delta_gradient * rho
    yhy = (y_h * y_rho.unsqueeze(-2)).sum(dim=-1)
    s_rho = step * rho
    ss = torch.matmul(s_rho.unsqueeze(-1), step.unsqueeze(-2)) * (1.0 + yhy.unsqueeze(-1))
    s_yh = torch.matmul(s_rho.unsqueeze(-1), y_h)
    h_y = torch.matmul(h, delta_gradient.unsqueeze(-1))
    hy_s = torch.matmul(h_y, s_rho.unsqueeze(-2))
    return h + ss - s_yh - hy_s


def wolfe_line_search(
    x: torch.Tensor,
    direction: torch.Tensor,
    f0: torch.Tensor,
    g0: torch.Tensor,
    closure: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
    c1: float = 1e-4,
    c2: float = 0.9,
    strong: bool = False,
    trials: Optional[list] = None,
    trial_log: Optional[list] = None,
) -> torch.Tensor:
    """Returns alpha (shape x.shape[:-1]); see module docstring.  ``trial_log`` (diagnostics)
    receives one dict per call: the base point, direction, f0, phi'(0) and, per trial, the
    active mask, alpha, f(alpha) and phi'(alpha)."""
    x = x.detach()
    direction = direction.detach()
    f0 = f0.detach()
    dphi0 = (direction * g0.detach()).sum(dim=-1)
    shape = x.shape[:-1]
    widen = torch.ones(shape, dtype=torch.bool)
    zoom = torch.zeros(shape, dtype=torch.bool)
    sufficient_fail = torch.zeros(shape, dtype=torch.bool)
    curv_ok = torch.zeros(shape, dtype=torch.bool)
    slope_up = torch.zeros(shape, dtype=torch.bool)
    a_lo = torch.zeros(shape, dtype=x.dtype)
    a_hi = a_lo.clone()
    a = torch.ones(shape, dtype=x.dtype)
    f_lo = f0.clone()
    f_hi = f0.clone()
    f_a = f0.clone()
    dphi_a = dphi0.clone()
    log = None
    if trial_log is not None:
        log = dict(x=x.clone(), direction=direction.clone(), f0=f0.clone(), dphi0=dphi0.clone(), trials=[])
        trial_log.append(log)
    for trial in range(1000):
        active = widen | zoom
        if not active.any():
            break
        if trial > 0:
            a_hi[widen] = a[widen]
            f_hi[widen] = f_a[widen]
            a[widen] = 2.0 * a[widen]
            a[zoom] = 0.5 * (a_lo[zoom] + a_hi[zoom])
        if trials is not None:
            trials.append(active.clone())
        alpha = a[active].clone().unsqueeze(-1).requires_grad_(True)
        with torch.enable_grad():
            fa = closure(x[active] + alpha * direction[active], active)
            (dfa,) = torch.autograd.grad(fa.sum(), alpha)
        f_a[active] = fa.detach()
        dphi_a[active] = dfa.squeeze(-1).detach()
        if log is not None:
            log["trials"].append(dict(active=active.clone(), alpha=a.clone(), f=f_a.clone(), dphi=dphi_a.clone()))

        sufficient_fail[active] = f_a[active] > f0[active] + c1 * a[active] * dphi0[active]
        sufficient_fail[zoom] |= f_a[zoom] >= f_lo[zoom]
        if trial > 0:
            sufficient_fail[widen] |= f_a[widen] >= f_hi[widen]
        if strong:
            curv_ok[active] = dphi_a[active].abs() <= -1.0 * c2 * dphi0[active]
        else:
            curv_ok[active] = -1.0 * dphi_a[active] <= -1.0 * c2 * dphi0[active]
        slope_up[widen] = dphi_a[widen] >= 0.0
        slope_up[zoom] = dphi_a[zoom] * (a_hi[zoom] - a_lo[zoom]) >= 0.0

        # zoom phase (N&W 3.6)
        z_hi = zoom & sufficient_fail
        z_done = zoom & ~sufficient_fail & curv_ok
        z_flip = zoom & ~sufficient_fail & ~curv_ok & slope_up
        z_lo = zoom & ~sufficient_fail & ~curv_ok
        sel = z_hi | z_done
        a_hi[sel] = a[sel]
        f_hi[sel] = f_a[sel]
        a_hi[z_flip] = a_lo[z_flip]
        f_hi[z_flip] = f_lo[z_flip]
        sel = z_lo | z_done
        a_lo[sel] = a[sel]
        f_lo[sel] = f_a[sel]
        zoom &= ~z_done

        # widening phase (N&W 3.5)
        w_bracket = widen & sufficient_fail
        w_done = widen & ~sufficient_fail & curv_ok
        w_flip = widen & ~sufficient_fail & ~curv_ok & slope_up
        a_lo[w_bracket] = a_hi[w_bracket]
        f_lo[w_bracket] = f_hi[w_bracket]
        sel = w_bracket | w_done
        a_hi[sel] = a[sel]
        f_hi[sel] = f_a[sel]
        sel = w_done | w_flip
        a_lo[sel] = a[sel]
        f_lo[sel] = f_a[sel]
        zoom |= w_bracket | w_flip
        zoom &= a_lo != a_hi
        widen &= ~(w_bracket | w_done | w_flip)
    return a_hi


def ulp_jitter(t: torch.Tensor, gen: torch.Generator) -> torch.Tensor:
    """t with every finite element moved by -1, 0 or +1 ulp (uniformly at random from `gen`); inf and NaN stay
    (a reordered sum that overflows still overflows: nextafter(inf, -inf) would make it finite)."""
    sign = torch.randint(0, 3, t.shape, generator=gen) - 1
    up = torch.nextafter(t, torch.full_like(t, float("inf")))
    down = torch.nextafter(t, torch.full_like(t, -float("inf")))
    moved = torch.where(sign > 0, up, torch.where(sign < 0, down, t))
    return torch.where(torch.isfinite(t), moved, t)


def _jittered_closure(closure, gen: torch.Generator):
    def fn(x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        out = closure(x, mask)
        d = out.detach()
        # the value moves, its gradient does not; an overflowed value stays as it is (inf - inf would be NaN,
        # and the NaN-blind Wolfe tests branch differently on NaN than on inf)
        delta = torch.where(torch.isfinite(d), ulp_jitter(d, gen) - d, torch.zeros_like(d))
        return out + delta
    return fn


@dataclass
class SolveRecord:
    iterations: torch.Tensor  # int, steps applied per problem
    reason: torch.Tensor  # STOP_* per problem
    closure_calls: int = 0
    line_search_trials: list = field(default_factory=list)


def bfgs_solve(
    x0: torch.Tensor,
    closure: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
    c1: float = 1e-4,
    c2: float = 0.9,
    error_threshold: float = 1e-4,
    iterations: int = 1000,
    minimum_step: float = 1e-8,
    record: Optional[SolveRecord] = None,
    trajectory: Optional[list] = None,
    trial_log: Optional[list] = None,
    training: bool = False,
    drop_path_p: float = 0.0,
    return_second_last: bool = False,
    ulp_noise: Optional[torch.Generator] = None,
) -> torch.Tensor:
    """Eval-mode ``BFGSSolver.forward`` (``bfgs_solver.py:80-215``).
    ``trajectory`` (optional list) receives x after every iteration's step.
    When ``x0.requires_grad`` the solve is differentiable like the reference's
    (``create_graph`` mode, ``:85, :129-135, :213-215``): the closure's gradient keeps its
    graph and x stays attached; the line search is detached as in the reference.
    ``training=True`` adds the training-mode semantics (the caller passes the training
    threshold / iteration count): per-iteration drop-path ``active &= rand_like > p``
    (``:121-125``, drawn with ``torch.rand_like`` so a test can make it deterministic) and
    ``return_second_last`` (``:196-212``), including the reference's scatter of the
    previous active set's rows into the smaller new active set.
    ``ulp_noise`` (a generator; parity diagnostics only, never for the goldens): every objective value the
    solve sees (the iterate's and every line-search trial's) and every gradient at an iterate move by -1, 0
    or +1 ulp at random -- the oracle's own spread under a last-bit change in EVERY evaluation, which is
    what a reordered fp32 sum does, where the 1-ulp nudge of x0 perturbs the start only."""
    create_graph = x0.requires_grad
    if ulp_noise is not None:
        closure = _jittered_closure(closure, ulp_noise)
    x = x0 if create_graph else x0.detach()
    shape = x.shape[:-1]
    p = x.size(-1)
    active = torch.ones(shape, dtype=torch.bool)
    calls = [0]

    def sub_closure(xs: torch.Tensor, sub_mask: torch.Tensor) -> torch.Tensor:
        full = torch.zeros_like(active)
        full[active] = sub_mask
        calls[0] += 1
        return closure(xs, full)

    step = torch.zeros_like(x)
    err = torch.empty(shape, dtype=x.dtype)
    grad = torch.empty_like(x)
    h = torch.zeros(shape + (p, p), dtype=x.dtype)
    h[..., range(p), range(p)] = 1.0
    steps_taken = torch.zeros(shape, dtype=torch.int32)
    reason = torch.full(shape, STOP_ITERATIONS, dtype=torch.int32)
    for k in range(iterations):
        grad_prev = grad
        if training and drop_path_p > 0.0:
            active = active & torch.greater(torch.rand_like(active, dtype=torch.float32), drop_path_p)
        xa = x[active]
        if not xa.requires_grad:
            xa.requires_grad_(True)
        with torch.enable_grad():
            fa = closure(xa, active)
            (ga,) = torch.autograd.grad(fa.sum(), xa, create_graph=create_graph)
        if ulp_noise is not None:
            ga = ulp_jitter(ga.detach(), ulp_noise)
        calls[0] += 1
        err = err.masked_scatter(active, fa.detach())
        grad = grad.masked_scatter(active.unsqueeze(-1).expand_as(grad), ga)

        still = active & (err > error_threshold)
        reason[active & ~still] = STOP_ERROR
        active = still
        if not active.any():
            break
        xa = x[active]
        fa = err[active]
        ga = grad[active]
        if k == 0:
            d = -1.0 * grad[active]
        else:
            y = ga - grad_prev[active]
            ha = h[active]
            if k == 1:
                ha = initial_scale(step[active], y).unsqueeze(-1) * ha
            ha = bfgs_update(ha, step[active], y)
            d = (-1.0 * torch.matmul(ha, ga.unsqueeze(-1))).squeeze(-1)
            h = h.masked_scatter(active.unsqueeze(-1).unsqueeze(-1).expand_as(h), ha)
        alpha = wolfe_line_search(
            xa, d, fa, ga, sub_closure, c1, c2, strong=True,
            trials=None if record is None else record.line_search_trials, trial_log=trial_log,
        )
        s = alpha.unsqueeze(-1) * d
        step = step.masked_scatter(active.unsqueeze(-1).expand_as(step), s)
        if not (training and return_second_last):
            x = x.masked_scatter(active.unsqueeze(-1).expand_as(x), xa + s)
        steps_taken[active] += 1
        if trajectory is not None:
            trajectory.append(x.detach().clone())
        still = active & (torch.linalg.vector_norm(step, dim=-1) > minimum_step)
        reason[active & ~still] = STOP_STEP
        active = still
        if not active.any():
            break
        if training and return_second_last:
            x = x.masked_scatter(active.unsqueeze(-1).expand_as(x), xa + s)
    if record is not None:
        record.iterations = steps_taken
        record.reason = reason
        record.closure_calls = calls[0]
    return x if create_graph else x.detach()
