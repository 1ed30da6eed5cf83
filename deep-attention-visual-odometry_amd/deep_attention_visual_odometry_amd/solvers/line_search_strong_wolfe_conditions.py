"""``LineSearchStrongWolfeConditions`` (reference: ``solvers/line_search_strong_wolfe_conditions.py``).

The legacy line search over an :class:`IOptimisableFunction` (N&W algorithms 3.5/3.6 with a
capped widening phase and secant-interpolated zoom).  Every error / gradient it asks for is a
HIP evaluation of the function object (``PinholeCameraModelL1``: one launch for the whole
B x E batch); this module only keeps the per-estimate bracket state.  The semantics follow the
reference step for step, including its fp32 constants (c1, c2, the step cap and the error
scale 1/sqrt(P) are fp32 tensors there).  One deliberate difference: the fallback step of an
unfinished search broadcasts alpha per estimate (the reference's ``alpha[:, None]`` only
broadcasts for one estimate per batch item).
"""
import math
import warnings

import torch
import torch.nn as nn

from ..utils import secant_alpha
from .i_optimisable_function import IOptimisableFunction


class LineSearchStrongWolfeConditions(nn.Module):
    def __init__(self, max_step_size: float, zoom_iterations: int, sufficient_decrease: float = 1e-4,
                 curvature: float = 0.9):
        super().__init__()
        if not 0.0 < sufficient_decrease < curvature < 1.0:
            warnings.warn(f"Line search conditions should satisfy 0 < c1 < c2 < 1. "
                          f"Got c1={sufficient_decrease} and c2={curvature}")
        self.max_step_size = torch.tensor(float(max_step_size))
        self.widen_iterations = int(math.ceil(math.log2(max_step_size)))
        self.zoom_iterations = int(zoom_iterations)
        self.sufficient_decrease = torch.tensor(float(sufficient_decrease))
        self.curvature = torch.tensor(float(curvature))

    def forward(self, function: IOptimisableFunction, search_direction: torch.Tensor):
        d = search_direction
        shape = (function.batch_size, function.num_estimates)
        c1, c2 = self.sufficient_decrease, self.curvature
        scale = torch.tensor(1.0 / function.num_parameters, device=function.device, dtype=torch.float).sqrt()

        def slope(fn, rows):  # scaled directional derivative on the selected estimates
            return (scale * fn.get_gradient()[rows] * d[rows]).sum(dim=-1)

        f0 = scale * function.get_error()
        slope0 = torch.sum(scale * function.get_gradient() * d, dim=-1)
        a_lo = torch.zeros(shape, dtype=d.dtype, device=d.device)
        a_hi = torch.ones(shape, dtype=d.dtype, device=d.device)
        fn_lo = fn_hi = out_fn = function
        out_step = torch.zeros_like(d)
        f_prev = f0
        widen = torch.ones(shape, dtype=torch.bool, device=d.device)
        zoom = torch.zeros(shape, dtype=torch.bool, device=d.device)

        # ---- widening (N&W 3.5) ----
        for it in range(self.widen_iterations):
            trial_step = a_hi.unsqueeze(-1) * d
            fn_hi = fn_hi.masked_update(function.add(trial_step), widen)
            f = scale * fn_hi.get_error()
            rising = torch.zeros_like(widen)
            rising[widen] = torch.greater(f[widen], f0[widen] + c1 * a_hi[widen] * slope0[widen])
            if it > 0:
                rising[widen] = torch.logical_or(rising[widen], torch.greater_equal(f[widen], f_prev[widen]))
            zoom = zoom | rising
            widen = widen & ~rising
            s = slope(fn_hi, widen)
            done = torch.zeros_like(widen)
            done[widen] = torch.less_equal(s.abs(), -c2 * slope0[widen])
            out_fn = out_fn.masked_update(fn_hi, done)
            out_step = torch.where(done[:, :, None], trial_step, out_step)
            s = s[~done[widen]]
            widen = widen & ~done
            swap = torch.zeros_like(widen)
            swap[widen] = torch.greater_equal(s, 0.0)
            zoom = zoom | swap
            a_lo, a_hi = torch.where(swap, a_hi, a_lo), torch.where(swap, a_lo, a_hi)
            fn_lo, fn_hi = fn_lo.masked_update(fn_hi, swap), fn_hi.masked_update(fn_lo, swap)
            widen = widen & ~swap
            a_lo[widen] = a_hi[widen]
            a_hi[widen] = torch.minimum(2.0 * a_hi[widen], self.max_step_size)
            fn_lo = fn_lo.masked_update(fn_hi, widen)
            f_prev = f

        # ---- zoom (N&W 3.6) with secant interpolation of the slopes ----
        for _ in range(self.zoom_iterations):
            alpha = secant_alpha(a_lo[zoom], a_hi[zoom], slope(fn_lo, zoom), slope(fn_hi, zoom))
            alpha_full = torch.zeros_like(a_hi)
            alpha_full[zoom] = alpha
            trial_step = torch.zeros_like(d)
            trial_step[zoom] = alpha[:, None] * d[zoom]
            trial = function.add(trial_step)
            f_lo = scale * fn_lo.get_error()
            f = scale * trial.get_error()
            rising = torch.zeros_like(zoom)
            rising[zoom] = torch.greater(f[zoom], f0[zoom] + c1 * alpha * slope0[zoom])
            rising = zoom & (torch.greater_equal(f, f_lo) | rising)
            a_hi = torch.where(rising, alpha_full, a_hi)
            fn_hi = fn_hi.masked_update(trial, rising)
            calm = zoom & ~rising
            s = slope(trial, calm)
            done = torch.zeros_like(calm)
            done[calm] = torch.less_equal(s.abs(), -c2 * slope0[calm])
            out_fn = out_fn.masked_update(trial, done)
            out_step = torch.where(done[:, :, None], trial_step, out_step)
            zoom = zoom & ~done
            swap = torch.zeros_like(zoom)
            swap[calm] = torch.logical_and(torch.greater_equal(s * (a_hi[calm] - a_lo[calm]), 0.0), zoom[calm])
            a_hi = torch.where(swap, a_lo, a_hi)
            fn_hi = fn_hi.masked_update(fn_lo, swap)
            calm = calm & zoom
            a_lo = torch.where(calm, alpha_full, a_lo)
            fn_lo = fn_lo.masked_update(trial, calm)

        unfinished = zoom | widen  # take the upper bracket rather than no step
        out_fn = out_fn.masked_update(fn_hi, unfinished)
        out_step = torch.where(unfinished[:, :, None], a_hi.unsqueeze(-1) * d, out_step)
        return out_fn, out_step
